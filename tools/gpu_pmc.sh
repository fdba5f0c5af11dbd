#!/bin/bash
# PMC passes (separate --pmc runs, kernel-trace only) for the headline workload.
# A bad counter name makes rocprofv3 exit non-zero without touching the GPU;
# any fault/abort/timeout status (>=124) ends the script.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1
ARGS="${BENCH_ARGS:---steps 1 --warmup 0 --no-cpu}"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $line -d $R/gpurun_out/pmc/p$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($line) rc=$rc" >> $R/gpurun_out/pmc/summary.txt
  [ $rc -ge 124 ] && exit $rc
done < $R/${PMC_FILE:-tools/pmc_passes.txt}
exit 0
