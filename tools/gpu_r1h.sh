#!/bin/bash
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -s -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log; ok $rc || exit $rc
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
for cp in "4 16" "1 16" "8 16" "4 8" "4 32"; do set -- $cp
  export RT_AMD_REFILL=$1 RT_AMD_CHUNK=$2
  $B > gpurun_out/b_cornell_$1_$2.log 2>&1 || exit $?
  $B --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres_$1_$2.log 2>&1 || exit $?
  RT_AMD_CHUNKED=1 $B --scene rain --width 1920 --spp 128 --depth 16 --steps 3 > gpurun_out/b_rain_$1_$2.log 2>&1 || exit $?
done
unset RT_AMD_REFILL RT_AMD_CHUNK
$B --scene rain --width 1920 --spp 128 --depth 16 --steps 3 > gpurun_out/b_rain_default.log 2>&1 || exit $?
$B --precision fp32 > gpurun_out/b_cornell_fp32.log 2>&1 || exit $?
