#!/bin/bash
bash tools/gpu_quick.sh || exit $?
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
RT_AMD_SAH=0 $B --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres_nosah.log 2>&1 || exit $?
RT_AMD_SAH=0 $B --scene rain --width 1920 --spp 128 --depth 16 --steps 3 > gpurun_out/b_rain_nosah.log 2>&1 || exit $?
