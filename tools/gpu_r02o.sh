#!/bin/bash
# Phase table in LDS: pool vs chunked on Cornell ref / fp32 / a rank share, spheres-500 (chunked), quick parity.
O=gpurun_out/r02o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "pool_kernel or chunked or multipass or ref_precision" > $O/pytest.log 2>&1 || exit $?
export OUT=$O/ab CFGS="cornell
cornellfp32 --precision fp32
cornell8 --width 283
spheres --scene spheres --spp 64 --depth 8" ARMS="pool
chunk RT_AMD_POOL_KERNEL=0"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
