#!/bin/bash
# Pool-kernel host gates (depth 250/251, spp 65535/65536) against the oracle.
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02bj; mkdir -p $R/$O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "gate or pool_kernel" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
exit 0
