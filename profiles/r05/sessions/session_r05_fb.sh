# round-5 final build: config 5 counters, fp32 / adaptive / config 5 bench lines, rocprof stats, rank shares
bash tools/gpu_run.sh r05_fin valu5 traffic5 fp32 adaptive config5 prof rankshare || exit $?
