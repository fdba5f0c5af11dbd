#!/bin/bash
mkdir -p gpurun_out
B="timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu"
$B --scene spheres100k --width 4096 --spp 16 --depth 100 > gpurun_out/b_100k.log 2>&1 || exit $?
$B --scene rain --width 1920 --spp 512 --depth 16 > gpurun_out/b_rain512.log 2>&1 || exit $?
