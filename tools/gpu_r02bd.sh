#!/bin/bash
# 56-byte pool slots (152 per wave): GPU parity, A/B vs HEAD on Cornell (ref, fp32).
O=gpurun_out/r02bd; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
export OUT=$O/ab STEPS=10 CFGS="cornell
cornellfp32 --precision fp32" ARMS="old RT_AMD_VARIANT=old
main
old2 RT_AMD_VARIANT=old
main2"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
