#!/bin/bash
# Light-order primitive copies (main) and paired pre-filter record loads (variant pair): GPU parity of both,
# A/B against the previous build (variant old).
O=gpurun_out/r02ab; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
RT_AMD_VARIANT=pair timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_pair.log 2>&1 || exit $?
export OUT=$O/ab STEPS=10 CFGS="cornell
cornellfp32 --precision fp32" ARMS="old RT_AMD_VARIANT=old
main
pair RT_AMD_VARIANT=pair
old2 RT_AMD_VARIANT=old
main2
pair2 RT_AMD_VARIANT=pair"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
