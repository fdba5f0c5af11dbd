#!/bin/bash
# Fixed per-launch cost of the pool kernel at HEAD: T(N) = a + b/N over rank shares, one-tile launches.
O=gpurun_out/r02ai; mkdir -p $O
timeout -k 10 300 python tools/fixed_cost.py cornell > $O/fixed_cornell.log 2>&1 || exit $?
