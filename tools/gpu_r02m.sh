#!/bin/bash
# Pool kernel: parity (pool vs chunked, then the whole GPU suite), Cornell A/B.
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "pool_kernel" > $O/pytest_pool.log 2>&1 || exit $?
export OUT=$O/ab CFGS="cornell
cornellfp32 --precision fp32
cornell8 --width 283" ARMS="pool
chunk RT_AMD_POOL_KERNEL=0"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo rc=$? >> $O/pytest.log
