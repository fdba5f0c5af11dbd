#!/bin/bash
# Overlapped record passes: GPU parity, then A/B (RT_AMD_PASS_OVERLAP) on rain 1080p spp512
# (2 passes) and config 5 (32 passes).
O=gpurun_out/r02as; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
export OUT=$O/ab STEPS=3 CFGS="rain --scene rain --width 1920 --spp 512 --depth 16" ARMS="ovl
serial RT_AMD_PASS_OVERLAP=0
ovl2
serial2 RT_AMD_PASS_OVERLAP=0"
bash tools/ab_env.sh || exit $?
export STEPS=1 TLIM=400 CFGS="c5 --scene spheres100k --width 4096 --spp 1024 --depth 100" ARMS="ovl
serial RT_AMD_PASS_OVERLAP=0"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
