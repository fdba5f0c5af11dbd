#!/bin/bash
# Round-4 A/B: the tree's top in LDS for launches that walk the tree from global memory (RT_AMD_TOP_CACHE).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04_l; mkdir -p $O
bash tools/gpu_run.sh r04_l pytest || exit $?
export OUT=$O/ab CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100
spheres --scene spheres --spp 64 --depth 8" ARMS="top1 RT_AMD_TOP_CACHE=1
top0 RT_AMD_TOP_CACHE=0
top1b RT_AMD_TOP_CACHE=1
top0b RT_AMD_TOP_CACHE=0"
STEPS=5 bash tools/ab_env.sh || exit $?
python tools/ab_table.py $OUT > $OUT/table.txt
