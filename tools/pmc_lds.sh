#!/bin/bash
# LDS pressure of the dominant kernel: one rocprofv3 --pmc pass (tools/pmc_passes_lds.txt) per
# bench configuration; SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = the share of LDS-array cycles
# lost to bank conflicts (MI355X_MICROARCH.md §LDS). usage: bash tools/pmc_lds.sh <tag> "<bench args>" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1/lds; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
n=0
for args in "$@"; do
  n=$((n+1)); i=0
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -d $O/c${n}_p$i -o run --output-format csv -- python3 $R/bench.py $args --steps 2 --warmup 0 --no-cpu --no-count --no-parity > $O/c${n}_p$i.log 2>&1
    rc=$?; echo "cfg $n ($args) pass $i rc=$rc" >> $O/summary.txt
    [ $rc -ne 0 ] && exit $rc
  done < $R/tools/pmc_passes_lds.txt
done
cd $R && python3 tools/pmc_sum.py $O/c*_p1 >> $O/summary.txt
