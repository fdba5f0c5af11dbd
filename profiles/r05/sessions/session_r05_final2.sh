# round-5 final build: bench lines of every config, rocprof kernel stats, the rank-share rehearsal
bash tools/gpu_run.sh r05_final bench4 fp32 adaptive config5 prof rankshare || exit $?
