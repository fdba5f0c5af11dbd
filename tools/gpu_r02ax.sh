#!/bin/bash
# Host-precomputed glass constants (1/ior, Schlick r0^2): GPU parity, A/B vs HEAD on Cornell and spheres-500.
O=gpurun_out/r02ax; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
export OUT=$O/ab STEPS=10 CFGS="cornell
spheres --scene spheres --spp 64 --depth 8" ARMS="old RT_AMD_VARIANT=old
main
old2 RT_AMD_VARIANT=old
main2"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
