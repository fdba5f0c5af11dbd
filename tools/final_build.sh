# A build's final measurements, in three gpurun calls that each fit one call's time limit
# (run from the repo root on the GPU box: bash tools/final_build.sh <part> [out-dir]):
#   1  bench lines of the four configs, then VALU / HBM-traffic counters (separate --pmc passes;
#      they become profiles/pmc_valu.json / pmc_traffic.json, keyed by build id)
#   2  config 5 counters, the fp32 / adaptive / config 5 bench lines, rocprof kernel stats, the
#      rank-share rehearsal
#   3  after the counters are committed: the whole -m gpu suite, every bench line (non-stale
#      rooflines) and the smoke
# Exploratory sessions of a round stay with their results (profiles/rNN/sessions/).
OUT=${2:-final}
case "$1" in
  1) bash tools/gpu_run.sh $OUT bench4 valu traffic || exit $? ;;
  2) bash tools/gpu_run.sh $OUT valu5 traffic5 fp32 adaptive config5 prof rankshare || exit $? ;;
  3) bash tools/gpu_run.sh ${OUT}2 pytest bench bench4 fp32 adaptive || exit $?
     timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${OUT}2/smoke.log 2>&1 || exit $? ;;
  *) echo "usage: bash tools/final_build.sh 1|2|3 [out-dir]" >&2; exit 2 ;;
esac
