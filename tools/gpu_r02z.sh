#!/bin/bash
# Pool-kernel stage configurations: GPU parity (main build; the pool tests for each variant),
# A/B against the previous build (variant old).
O=gpurun_out/r02z; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
for v in ${VARS:-n0s0 n1s0}; do
  RT_AMD_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k pool --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1 || exit $?
done
export OUT=$O/ab STEPS=10 CFGS="cornell" ARMS="${ARMS:-old RT_AMD_VARIANT=old
main
n0s0 RT_AMD_VARIANT=n0s0
n1s0 RT_AMD_VARIANT=n1s0
old2 RT_AMD_VARIANT=old
main2
n0s02 RT_AMD_VARIANT=n0s0
n1s02 RT_AMD_VARIANT=n1s0}"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
