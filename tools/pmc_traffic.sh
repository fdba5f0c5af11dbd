#!/bin/bash
# HBM traffic of the dominant kernel per launch (roofline "traffic"): separate
# rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE (kernel-trace only), then
# tools/pmc_traffic.py folds them into profiles/pmc_traffic.json.
# usage: bash tools/pmc_traffic.sh "<bench args>" ...
R=$GRAFT_REPO_ROOT
T=${TRAFFIC_DIR:-gpurun_out/traffic}
mkdir -p $R/$T
cd /tmp && export TMPDIR=/tmp
n=0
for args in "$@"; do
  n=$((n+1))
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d $R/$T/c${n}_$c -o run --output-format csv -- python3 $R/bench.py $args --steps 2 --warmup 0 --no-cpu --no-count --no-parity > $R/$T/c${n}_$c.log 2>&1
    rc=$?; echo "cfg $n ($args) $c rc=$rc" >> $R/$T/summary.txt
    [ $rc -ge 124 ] && exit $rc
  done
done
cd $R && python3 tools/pmc_traffic.py $T "$@" && cp profiles/pmc_traffic.json $T/
