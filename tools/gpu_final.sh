#!/bin/bash
# Round evidence for HEAD: GPU parity, the default bench line (with CPU leg), the
# same command under rocprofv3 --kernel-trace --stats, the other bench configs,
# HBM traffic passes and VALU passes (separate --pmc runs), the 1-GPU rank-share
# scaling rehearsal. Every GPU step has its own time limit; any failure ends it.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
TAG=final bash tools/gpu_bench4.sh || exit $?
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --precision fp32 > gpurun_out/b_cornellf_final.log 2>&1 || exit $?
timeout -k 10 200 python tools/rank_share.py cornell > gpurun_out/rank_share.log 2>&1 || exit $?
timeout -k 10 200 python tools/rank_share.py spheres >> gpurun_out/rank_share.log 2>&1 || exit $?
bash tools/pmc_traffic.sh "" "--scene spheres --spp 64 --depth 8" "--scene rain --width 1920 --spp 512 --depth 16" || exit $?
bash tools/pmc_valu.sh "" "--precision fp32" "--scene spheres --spp 64 --depth 8" "--scene rain --width 1920 --spp 512 --depth 16" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py > $R/gpurun_out/prof.log 2>&1 || exit $?
exit 0
