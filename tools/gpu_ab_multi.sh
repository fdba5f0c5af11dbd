#!/bin/bash
# A/B of library variants (RT_AMD_VARIANT) on the bench scenes; optional parity tests first.
# VARIANTS="sc nostore" [TESTS=1] [PROBE=1] bash tools/gpu_ab_multi.sh
mkdir -p gpurun_out
if [ -n "$PROBE" ]; then timeout -k 10 120 tools/probes/sincos_check > gpurun_out/sincos_check.log 2>&1 || exit $?; fi
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
fi
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
for v in main $VARIANTS; do
  if [ $v = main ]; then unset RT_AMD_VARIANT; else export RT_AMD_VARIANT=$v; fi
  $B > gpurun_out/ab_cornell_$v.log 2>&1 || exit $?
  $B --scene spheres --spp 64 --depth 8 > gpurun_out/ab_spheres_$v.log 2>&1 || exit $?
  if [ -n "$FP32" ]; then $B --precision fp32 > gpurun_out/ab_cornellf32_$v.log 2>&1 || exit $?; fi
  if [ -n "$RAIN" ]; then $B --scene rain --width 1920 --spp 128 --depth 16 --steps 3 > gpurun_out/ab_rain_$v.log 2>&1 || exit $?; fi
done
exit 0
