#!/bin/bash
# BVH hand-out rule (pool 4/2, first chunk pow2floor(sqrt(spl)/3)): rank shares of spheres-500
# and rain at the defaults, rain N=1 chunked (forced) vs sequential.
O=gpurun_out/r02ao; mkdir -p $O
SWEEP_POOL=auto SWEEP_CHUNK=auto SWEEP_N="1 2 4 8" timeout -k 10 300 python tools/sched_sweep.py spheres > $O/auto_spheres.log 2>&1 || exit $?
SWEEP_POOL=auto SWEEP_CHUNK=auto SWEEP_N="1 2 4 8" timeout -k 10 300 python tools/sched_sweep.py rain > $O/auto_rain.log 2>&1 || exit $?
RT_AMD_CHUNKED=1 SWEEP_POOL="auto" SWEEP_CHUNK="auto 8 32" SWEEP_N="1" timeout -k 10 300 python tools/sched_sweep.py rain > $O/chunked1_rain.log 2>&1 || exit $?
