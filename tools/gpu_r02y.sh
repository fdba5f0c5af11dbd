#!/bin/bash
# Split diffuse queues in the pool kernel: GPU parity, A/B against RT_POOL_DSPLIT=0 (variant nosplit).
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
export OUT=$O/ab STEPS=10 CFGS="cornell
cornellfp32 --precision fp32" ARMS="nosplit RT_AMD_VARIANT=nosplit
split
nosplit2 RT_AMD_VARIANT=nosplit
split2
splitfp32pool RT_AMD_POOL_KERNEL=1
nosplitfp32pool RT_AMD_VARIANT=nosplit RT_AMD_POOL_KERNEL=1"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
