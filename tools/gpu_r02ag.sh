#!/bin/bash
# Exact-test counts per ray in the brute-force closest hit (candidates after the pre-filter, rays needing 2+ tests).
O=gpurun_out/r02ag; mkdir -p $O
timeout -k 10 300 python tools/count_exact.py cornell > $O/count_exact.log 2>&1 || exit $?
