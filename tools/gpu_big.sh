#!/bin/bash
# parity + quick benches + spheres-100k (BASELINE config 5 scene, 4096^2 spp16)
bash tools/gpu_quick.sh || exit $?
timeout -k 10 300 python bench.py --scene spheres100k --width 4096 --spp 16 --depth 100 --steps 2 --warmup 1 --no-cpu > gpurun_out/b_100k.log 2>&1 || exit $?
