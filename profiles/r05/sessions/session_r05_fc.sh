# round-5 final build, counters committed: the whole -m gpu suite, smoke, every bench line (non-stale rooflines)
bash tools/gpu_run.sh r05_fin2 pytest bench bench4 fp32 adaptive || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_fin2/smoke.log 2>&1 || exit $?
