#!/bin/bash
# fma-based exact dot/cross: GPU parity, then A/B against the previous build (variant "old").
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
export OUT=$O/ab CFGS="cornell
spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16" ARMS="old RT_AMD_VARIANT=old
new
old2 RT_AMD_VARIANT=old
new2"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
