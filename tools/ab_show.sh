#!/bin/bash
# value / kernel ms of every bench log under gpurun_out (A/B summaries)
for f in ${@:-gpurun_out/b_*.log}; do
  printf "%-40s %s\n" "$(basename $f .log)" "$(tail -1 $f | python3 -c 'import sys,json
try:
    d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["config"]["workload"])
except Exception as e: print("n/a")')"
done
