# round-5 final build: VALU and HBM-traffic counters of BASELINE config 5
bash tools/gpu_run.sh r05_final valu5 traffic5 || exit $?
