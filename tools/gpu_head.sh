#!/bin/bash
# Full round check of HEAD: parity tests, headline bench (with CPU leg), the
# other bench scenes, spheres-100k, and a rocprofv3 kernel-trace profile.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
$B --precision fp32 > gpurun_out/b_cornell_fp32.log 2>&1 || exit $?
$B --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres.log 2>&1 || exit $?
$B --scene rain --width 1920 --spp 512 --depth 16 --steps 3 > gpurun_out/b_rain.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --scene spheres100k --width 4096 --spp 16 --depth 100 --steps 2 --warmup 1 --no-cpu > gpurun_out/b_100k.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/prof.log 2>&1 || exit $?
exit 0
