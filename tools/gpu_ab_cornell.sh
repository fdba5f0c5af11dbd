#!/bin/bash
# A/B on the headline scene: GPU parity on the main lib, then Cornell (ref + fp32) on main and $VARIANTS.
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log; ok $rc || exit $rc
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
for v in main $VARIANTS; do
  if [ $v = main ]; then unset RT_AMD_VARIANT; else export RT_AMD_VARIANT=$v; fi
  $B > gpurun_out/b_cornell_$v.log 2>&1 || exit $?
  $B --precision fp32 > gpurun_out/b_cornellf_$v.log 2>&1 || exit $?
done
