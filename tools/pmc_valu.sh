#!/bin/bash
# VALU evidence for the dominant kernel (north_star: "VALU-busy against gfx950 peak"):
# the counter passes of tools/pmc_passes_valu.txt, one rocprofv3 --pmc run each
# (kernel-trace only), per bench configuration; tools/pmc_valu.py folds them
# into profiles/pmc_valu.json.  usage: bash tools/pmc_valu.sh "<bench args>" ...
R=$GRAFT_REPO_ROOT
V=${VALU_DIR:-gpurun_out/valu}
mkdir -p $R/$V
cd /tmp && export TMPDIR=/tmp
n=0
for args in "$@"; do
  n=$((n+1)); i=0
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $line -d $R/$V/c${n}_p$i -o run --output-format csv -- python3 $R/bench.py $args --steps 2 --warmup 0 --no-cpu --no-count --no-parity > $R/$V/c${n}_p$i.log 2>&1
    rc=$?; echo "cfg $n ($args) pass $i rc=$rc" >> $R/$V/summary.txt
    [ $rc -ge 124 ] && exit $rc
  done < $R/tools/pmc_passes_valu.txt
done
cd $R && python3 tools/pmc_valu.py $V "$@" && cp ${PMC_VALU_OUT:-profiles/pmc_valu.json} $V/
