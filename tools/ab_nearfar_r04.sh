#!/bin/bash
# Round-4 A/B: near / far rows picked by the ray's direction signs (product) vs min / max per plane pair (nf0).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04_n; mkdir -p $O
bash tools/gpu_run.sh r04_n pytest || exit $?
export OUT=$O/ab CFGS="spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16
s100k --scene spheres100k --width 2048 --spp 16 --depth 100" ARMS="nf1 RT_AMD_VARIANT=
nf0 RT_AMD_VARIANT=nf0
nf1b RT_AMD_VARIANT=
nf0b RT_AMD_VARIANT=nf0"
STEPS=5 bash tools/ab_env.sh || exit $?
python tools/ab_table.py $OUT > $OUT/table.txt
