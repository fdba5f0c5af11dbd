#!/bin/bash
# Round-1 GPU session: parity tests, headline bench (+CPU baseline), other scenes, rocprof stats.
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
for p in fp32; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --precision $p > gpurun_out/bench_cornell_$p.log 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --scene spheres --spp 64 --depth 8 > gpurun_out/bench_spheres_ref.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --scene rain --width 1920 --spp 512 --depth 16 > gpurun_out/bench_rain_ref.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
echo "prof rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/prof.log
