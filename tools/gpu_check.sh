#!/bin/bash
# GPU session script: each GPU step has its own time limit; stop on a fault/timeout.
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_quick.log
exit $rc
