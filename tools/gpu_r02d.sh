#!/bin/bash
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "chunked or multipass or full_size or ref_precision or golden or config1 or packed" > $O/pytest.log 2>&1; rc=$?; echo "rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
export OUT=$O/ab CFGS="cornell
spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128
cornell8 --scene cornell --width 283" ARMS="base
nofold RT_AMD_FOLD=0
f64 RT_AMD_FOLD=64
f192 RT_AMD_FOLD=192"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
