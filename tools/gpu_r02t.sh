#!/bin/bash
# 1-GPU strong-scaling rehearsal (rank 0's tile share for N = 1, 2, 4, 8) at HEAD.
O=gpurun_out/r02t; mkdir -p $O
for s in cornell spheres; do
  timeout -k 10 300 python tools/rank_share.py $s > $O/rank_share_$s.log 2>&1 || exit $?
done
