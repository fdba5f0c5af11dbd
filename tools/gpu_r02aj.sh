#!/bin/bash
# Hand-out sweep (tile-chunks per atomic x first-phase chunk) for the pool kernel, N = 1, 2, 8 shares.
O=gpurun_out/r02aj; mkdir -p $O
timeout -k 10 400 python tools/sched_sweep.py cornell > $O/sweep_cornell.log 2>&1 || exit $?
