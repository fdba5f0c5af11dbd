#!/bin/bash
# Chunked-kernel hand-out rules for LDS-resident BVH scenes: GPU parity, rank shares at the new
# defaults (spheres-500, rain; rain's N=1 launch is the sequential kernel), bench lines.
O=gpurun_out/r02am; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
SWEEP_POOL=auto SWEEP_CHUNK=auto SWEEP_N="1 2 4 8" timeout -k 10 300 python tools/sched_sweep.py spheres > $O/auto_spheres.log 2>&1 || exit $?
SWEEP_POOL="auto 1" SWEEP_CHUNK="auto" SWEEP_N="1 2 4 8" timeout -k 10 300 python tools/sched_sweep.py rain > $O/auto_rain.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --scene spheres --spp 64 --depth 8 > $O/b_spheres.log 2>&1 || exit $?
