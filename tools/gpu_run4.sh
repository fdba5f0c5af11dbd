#!/bin/bash
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_gpu4.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu4.log; ok $rc || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters_list.txt 2>&1
echo "list rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/counters_list.txt
