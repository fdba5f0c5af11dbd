#!/bin/bash
# Round-4 knob re-check after the cheaper node step: min_ready (RT_AMD_READY) on the BVH scenes.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export OUT=gpurun_out/r04_f/ab CFGS="spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16
s100k --scene spheres100k --width 2048 --spp 16 --depth 100" ARMS="r48 RT_AMD_READY=48
r40 RT_AMD_READY=40
r56 RT_AMD_READY=56
r32 RT_AMD_READY=32
r48b RT_AMD_READY=48"
STEPS=5 bash tools/ab_env.sh || exit $?
python tools/ab_table.py $OUT > $OUT/table.txt
