#!/bin/bash
# Stats words on separate lines + persistent accumulate with block-level merge: parity + timing.
O=${O:-gpurun_out/r02q}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
export OUT=$O/ab CFGS="cornell
cornellfp32 --precision fp32
spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128" ARMS="base"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
