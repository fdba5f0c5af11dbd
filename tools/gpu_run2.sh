#!/bin/bash
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 120 python tools/probe_fp32.py > gpurun_out/probe.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/probe.log; ok $rc || exit $rc
timeout -k 10 300 python -m pytest tests -m gpu -q -s -p no:cacheprovider -k "tile_groups or work_counters or fp32" > gpurun_out/pytest_gpu2.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu2.log; ok $rc || exit $rc
for p in ref fp32; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --precision $p > gpurun_out/bench_$p.log 2>&1 || exit $?
done
for s in spheres rain; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --scene $s --spp 64 --depth 8 > gpurun_out/bench_$s.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_r1.log 2>&1
echo "prof rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/prof_r1.log
