#!/bin/bash
# Walker-pool (HBM slots) A/B: parity tests of the walker pool, then bench arms.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_run.sh ${TAG:-wpab} "pytest:wpool" || exit $?
export OUT=gpurun_out/${TAG:-wpab}/ab
export CFGS="spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16
s100k --scene spheres100k --width 2048 --spp 16 --depth 100"
export ARMS="${ARMS:-base RT_AMD_WPOOL=0
wp RT_AMD_WPOOL=1
wpk128 RT_AMD_WPOOL=1 RT_AMD_WPOOL_K=128
wpk255 RT_AMD_WPOOL=1 RT_AMD_WPOOL_K=255
wp768 RT_AMD_VARIANT=wp768 RT_AMD_WPOOL=1}"
STEPS=3 bash tools/ab_env.sh || exit $?
python tools/ab_table.py $OUT > $OUT/table.txt
