#!/bin/bash
# Pool size sensitivity: 96 (default) vs 80 vs 64 path slots per wave, Cornell ref.
O=gpurun_out/r02ba; mkdir -p $O
export OUT=$O/ab STEPS=10 CFGS="cornell" ARMS="k96
k80 RT_AMD_VARIANT=k80
k64 RT_AMD_VARIANT=k64
k96b
k80b RT_AMD_VARIANT=k80"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
