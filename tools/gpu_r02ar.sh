#!/bin/bash
# Config 5 at its stated workload (spheres-100k 4096^2 spp1024 d100): hand-out A/B.
O=gpurun_out/r02ar; mkdir -p $O
export OUT=$O/ab STEPS=1 TLIM=400 CFGS="c5 --scene spheres100k --width 4096 --spp 1024 --depth 100" ARMS="auto
p4c4 RT_AMD_POOL=4 RT_AMD_CHUNK=4
p4c8 RT_AMD_POOL=4 RT_AMD_CHUNK=8
p4c32 RT_AMD_POOL=4 RT_AMD_CHUNK=32"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
