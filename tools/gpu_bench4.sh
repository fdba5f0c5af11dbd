#!/bin/bash
# The four bench lines (no CPU leg): Cornell ref, spheres-500, rain 1080p spp512, spheres-100k spp16.
mkdir -p gpurun_out
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
T=${TAG:-main}
$B > gpurun_out/b_cornell_$T.log 2>&1 || exit $?
$B --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres_$T.log 2>&1 || exit $?
$B --scene rain --width 1920 --spp 512 --depth 16 --steps 3 > gpurun_out/b_rain_$T.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --scene spheres100k --width 4096 --spp 16 --depth 100 --steps 2 --warmup 1 --no-cpu > gpurun_out/b_100k_$T.log 2>&1 || exit $?
