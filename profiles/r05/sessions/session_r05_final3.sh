# round-5 final build: VALU and HBM-traffic counters (separate --pmc passes) of the bench configs
bash tools/gpu_run.sh r05_final valu traffic || exit $?
