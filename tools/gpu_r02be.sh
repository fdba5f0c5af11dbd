#!/bin/bash
# Pool-kernel hand-out sweep with 152 slots per wave (Cornell rank shares N = 1, 2, 8).
O=gpurun_out/r02be; mkdir -p $O
SWEEP_POOL="auto 2 4 8" SWEEP_CHUNK="auto 4 8 16" SWEEP_N="1 2 8" timeout -k 10 500 python tools/sched_sweep.py cornell > $O/sweep_cornell.log 2>&1 || exit $?
