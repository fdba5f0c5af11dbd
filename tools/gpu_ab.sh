#!/bin/bash
# A/B: parity on the main lib, then the bench scenes on the main lib and on variant libs ($VARIANTS)
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -s -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log; ok $rc || exit $rc
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
for v in main $VARIANTS; do
  if [ $v = main ]; then unset RT_AMD_VARIANT; else export RT_AMD_VARIANT=$v; fi
  $B > gpurun_out/b_cornell_$v.log 2>&1 || exit $?
  $B --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres_$v.log 2>&1 || exit $?
  $B --scene rain --width 1920 --spp 128 --depth 16 --steps 3 > gpurun_out/b_rain_$v.log 2>&1 || exit $?
  if [ -n "$BIG" ]; then
    timeout -k 10 300 python bench.py --scene spheres100k --width 4096 --spp 16 --depth 100 --steps 2 --warmup 1 --no-cpu > gpurun_out/b_100k_$v.log 2>&1 || exit $?
  fi
done
