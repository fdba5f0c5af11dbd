#!/bin/bash
# Tail hand-out A/B (RT_AMD_TAIL rounds in takes of RT_AMD_TAIL_POOL tile-chunks): rank-0 shares
# for N = 1, 2, 4, 8 (tools/rank_share.py), Cornell and spheres-500.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG:-tail}
mkdir -p $O
ARMS=${ARMS:-"base RT_AMD_TAIL=0
t1p1 RT_AMD_TAIL=4 RT_AMD_TAIL_POOL=1
t2p1 RT_AMD_TAIL=8 RT_AMD_TAIL_POOL=1
t1p2 RT_AMD_TAIL=4 RT_AMD_TAIL_POOL=2"}
echo "$ARMS" | while read -r arm envs; do
  [ -z "$arm" ] && continue
  for sc in cornell spheres; do
    env $envs timeout -k 10 200 python tools/rank_share.py $sc > $O/rs_${sc}_${arm}.log 2>&1 || exit $?
  done
done
