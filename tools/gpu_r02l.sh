#!/bin/bash
# Round-2 evidence at HEAD: GPU parity suite, headline bench, config-5 bench, rocprof kernel stats.
O=gpurun_out/r02l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo rc=$rc >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --scene spheres100k --width 4096 --spp 1024 --depth 100 --steps 2 --warmup 1 --no-cpu > $O/bench_100k.json 2> $O/bench_100k.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-cpu --steps 10 > $O/prof.log 2>&1 || exit $?
