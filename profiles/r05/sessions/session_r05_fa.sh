# round-5 final build: bench lines of the four configs, then VALU / HBM-traffic counters (separate --pmc passes)
bash tools/gpu_run.sh r05_fin bench4 valu traffic || exit $?
