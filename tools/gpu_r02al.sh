#!/bin/bash
# Hand-out sweep for the chunked kernel on spheres-500 (rank shares N = 1, 2, 4, 8).
O=gpurun_out/r02al; mkdir -p $O
SWEEP_POOL="auto 2" SWEEP_CHUNK="auto 1 2 4 8 16" SWEEP_N="1 2 4 8" timeout -k 10 400 python tools/sched_sweep.py spheres > $O/sweep_spheres.log 2>&1 || exit $?
