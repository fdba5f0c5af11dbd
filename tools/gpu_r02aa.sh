#!/bin/bash
# Compact pre-filter records (main) and the fused exact test (variant fused): GPU parity of both,
# A/B against the previous build (variant old).
O=gpurun_out/r02aa; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
RT_AMD_VARIANT=fused timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_fused.log 2>&1 || exit $?
export OUT=$O/ab STEPS=10 CFGS="cornell
cornellfp32 --precision fp32" ARMS="old RT_AMD_VARIANT=old
main
fused RT_AMD_VARIANT=fused
old2 RT_AMD_VARIANT=old
main2
fused2 RT_AMD_VARIANT=fused"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
