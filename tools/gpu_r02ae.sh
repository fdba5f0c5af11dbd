#!/bin/bash
# 1-GPU strong-scaling rehearsal at HEAD (rank 0's share for N = 1, 2, 4, 8) + two-rank bench check.
O=gpurun_out/r02ae; mkdir -p $O
timeout -k 10 200 python tools/rank_share.py cornell > $O/rank_share.log 2>&1 || exit $?
timeout -k 10 200 python tools/rank_share.py spheres >> $O/rank_share.log 2>&1 || exit $?
