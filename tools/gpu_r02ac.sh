#!/bin/bash
# Paired pre-filter record loads (main) vs single loads (variant nopair): GPU parity of both,
# A/B against the previous build (variant old).
O=gpurun_out/r02ac; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
RT_AMD_VARIANT=nopair timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_nopair.log 2>&1 || exit $?
export OUT=$O/ab STEPS=10 CFGS="cornell
cornellfp32 --precision fp32" ARMS="old RT_AMD_VARIANT=old
main
nopair RT_AMD_VARIANT=nopair
old2 RT_AMD_VARIANT=old
main2
nopair2 RT_AMD_VARIANT=nopair"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
