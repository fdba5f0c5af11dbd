# round-5 final build: the whole -m gpu suite, the default bench line (CPU leg + parity), smoke
bash tools/gpu_run.sh r05_final pytest bench || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_final/smoke.log 2>&1 || exit $?
