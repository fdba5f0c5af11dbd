#!/bin/bash
O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "fast or random or sah or large or world_hit or tiny or full_size or ref_precision" > $O/pytest.log 2>&1; rc=$?; echo rc=$rc >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
export OUT=$O/ab CFGS="spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128
c100k --scene spheres100k --width 2048 --spp 64 --depth 100" ARMS="defer
nodefer RT_AMD_VARIANT=nodefer"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
timeout -k 10 300 python tools/count_exact.py spheres rain spheres100k > $O/count_exact.log 2>&1 || exit $?
