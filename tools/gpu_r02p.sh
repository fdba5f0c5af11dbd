#!/bin/bash
# Pool kernel geometry: 16 waves x 96 slots (default) vs 12 waves x 128 slots (variant pool768).
O=gpurun_out/r02p; mkdir -p $O
export OUT=$O/ab CFGS="cornell
cornellfp32 --precision fp32" ARMS="pool96
pool128 RT_AMD_VARIANT=pool768
chunk RT_AMD_POOL_KERNEL=0"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
