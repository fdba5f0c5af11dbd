#!/bin/bash
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -s -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log; ok $rc || exit $rc
RT_AMD_VARIANT=imm timeout -k 10 600 python -m pytest tests -m gpu -q -s -x -p no:cacheprovider -k "world_hit or fast_traversal or ref_precision" > gpurun_out/pytest_gpu_imm.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu_imm.log; ok $rc || exit $rc
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
for v in "" imm; do for l in 1 0; do
  export RT_AMD_VARIANT=$v RT_AMD_LDS_SCENE=$l
  $B > gpurun_out/b_cornell_${v}_$l.log 2>&1 || exit $?
  $B --scene rain --width 1920 --spp 128 --depth 16 --steps 3 > gpurun_out/b_rain_${v}_$l.log 2>&1 || exit $?
done; done
unset RT_AMD_VARIANT RT_AMD_LDS_SCENE
$B --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres.log 2>&1 || exit $?
RT_AMD_VARIANT=imm $B --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres_imm.log 2>&1 || exit $?
