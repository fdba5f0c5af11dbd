#!/bin/bash
# Per-launch fixed cost probe (pool and chunked kernels).
O=gpurun_out/r02u; mkdir -p $O
timeout -k 10 300 python tools/fixed_cost.py cornell > $O/fixed_cornell_pool.log 2>&1 || exit $?
RT_AMD_POOL_KERNEL=0 timeout -k 10 300 python tools/fixed_cost.py cornell > $O/fixed_cornell_chunk.log 2>&1 || exit $?
timeout -k 10 300 python tools/fixed_cost.py spheres > $O/fixed_spheres.log 2>&1 || exit $?
