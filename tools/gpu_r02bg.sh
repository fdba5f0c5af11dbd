#!/bin/bash
# Packed pre-filter pairs of same-code axis quads: GPU parity, A/B (RT_AMD_PRE_PAIRS=0 control, same build).
O=gpurun_out/r02bg; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
export OUT=$O/ab STEPS=10 CFGS="cornell
cornellfp32 --precision fp32" ARMS="nopair RT_AMD_PRE_PAIRS=0
pair
nopair2 RT_AMD_PRE_PAIRS=0
pair2"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
