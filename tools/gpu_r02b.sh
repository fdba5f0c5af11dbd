#!/bin/bash
# round-2 check: GPU parity suite, headline bench (+CPU baseline), config-5 bench at its stated workload
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/b_cornell.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --scene spheres100k --width 4096 --spp 1024 --depth 100 --steps 1 --warmup 0 --no-cpu > $O/b_100k_spp1024.log 2>&1 || exit $?
timeout -k 10 300 python tools/profile_sections.py cornell spheres spheres100k > $O/sections.log 2>&1 || exit $?
exit 0
