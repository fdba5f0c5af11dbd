#!/bin/bash
# parity tests + quick benches of the three bench scenes (+ optional section profile)
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -s -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log; ok $rc || exit $rc
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
$B > gpurun_out/b_cornell.log 2>&1 || exit $?
$B --precision fp32 > gpurun_out/b_cornell_fp32.log 2>&1 || exit $?
$B --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres.log 2>&1 || exit $?
$B --scene rain --width 1920 --spp 128 --depth 16 --steps 3 > gpurun_out/b_rain.log 2>&1 || exit $?
if [ -n "$PROFILE" ]; then timeout -k 10 300 python tools/profile_sections.py $PROFILE > gpurun_out/sections.log 2>&1; fi
exit 0
