#!/bin/bash
# Pool A queue split into start | in-flight stacks (main): GPU parity, A/B against the previous
# build (variant old); 1-GPU rank-share rehearsal of the previous build.
O=gpurun_out/r02af; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
export OUT=$O/ab STEPS=10 CFGS="cornell
cornellfp32 --precision fp32" ARMS="old RT_AMD_VARIANT=old
main
mainpool RT_AMD_POOL_KERNEL=1
old2 RT_AMD_VARIANT=old
main2"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
RT_AMD_VARIANT=old timeout -k 10 200 python tools/rank_share.py cornell > $O/rank_share.log 2>&1 || exit $?
RT_AMD_VARIANT=old timeout -k 10 200 python tools/rank_share.py spheres >> $O/rank_share.log 2>&1 || exit $?
