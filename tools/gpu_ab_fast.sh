#!/bin/bash
# A/B on the fast-traversal configs: GPU parity on the main lib, then spheres-500,
# spheres-100k (spp 16) and rain's 1/8 share on main and $VARIANTS ($SWEEPENV: extra env sets).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
for v in main $VARIANTS; do
  if [ $v = main ]; then unset RT_AMD_VARIANT; else export RT_AMD_VARIANT=$v; fi
  $B --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres_$v.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --scene spheres100k --width 4096 --spp 16 --depth 100 --steps 2 --warmup 1 --no-cpu > gpurun_out/b_100k_$v.log 2>&1 || exit $?
  timeout -k 10 120 python tools/tail_probe.py spheres 1 8 > gpurun_out/tail_$v.log 2>&1 || exit $?
  timeout -k 10 120 python tools/tail_probe.py rain 8 >> gpurun_out/tail_$v.log 2>&1 || exit $?
done
