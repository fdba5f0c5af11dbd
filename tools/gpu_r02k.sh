#!/bin/bash
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo rc=$rc >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
export OUT=$O/ab CFGS="spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128
c100k --scene spheres100k --width 2048 --spp 64 --depth 100
cornell" ARMS="auto"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
