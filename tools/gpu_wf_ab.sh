#!/bin/bash
# Wavefront passes: parity tests, then bench arms (wavefront forced on / off).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_run.sh ${TAG:-wfab} "pytest:wavefront" || exit $?
export OUT=gpurun_out/${TAG:-wfab}/ab
export CFGS="${CFGS:-s100k --scene spheres100k --width 2048 --spp 16 --depth 100
spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16}"
export ARMS="${ARMS:-chunked RT_AMD_WAVEFRONT=0
wf RT_AMD_WAVEFRONT=1}"
STEPS=3 bash tools/ab_env.sh || exit $?
python tools/ab_table.py $OUT > $OUT/table.txt
