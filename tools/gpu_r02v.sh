#!/bin/bash
# Static first pools: parity, bench set, fixed-cost probe.
O=gpurun_out/r02v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
export OUT=$O/ab CFGS="cornell
spheres --scene spheres --spp 64 --depth 8" ARMS="base"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
timeout -k 10 300 python tools/fixed_cost.py cornell > $O/fixed_cornell.log 2>&1 || exit $?
timeout -k 10 300 python tools/fixed_cost.py spheres > $O/fixed_spheres.log 2>&1 || exit $?
