#!/bin/bash
# Hand-out sweep for config 5's scene (spheres-100k, BVH from global memory), 2048^2 spp64 d100.
O=gpurun_out/r02aq; mkdir -p $O
SWEEP_POOL="auto 2 4" SWEEP_CHUNK="auto 4 8 16" SWEEP_N="1" timeout -k 10 500 python tools/sched_sweep.py spheres100k > $O/sweep_100k.log 2>&1 || exit $?
