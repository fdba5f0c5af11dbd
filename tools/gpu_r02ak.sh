#!/bin/bash
# Pool-kernel hand-out rules: GPU parity, then rank-share times at the new defaults (N = 1, 2, 4, 8)
# and the spheres-500 rank shares (chunked kernel, unchanged rules).
O=gpurun_out/r02ak; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
SWEEP_POOL=auto SWEEP_CHUNK=auto SWEEP_N="1 2 4 8" timeout -k 10 300 python tools/sched_sweep.py cornell > $O/auto_cornell.log 2>&1 || exit $?
SWEEP_POOL="auto 2 4" SWEEP_CHUNK="auto 4 8" SWEEP_N="4" timeout -k 10 300 python tools/sched_sweep.py cornell > $O/sweep4_cornell.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu > $O/bench.log 2>&1 || exit $?
