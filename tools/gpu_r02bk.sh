#!/bin/bash
# spheres-100k 4096^2 spp64 d100: READY x REFILL sweep of the resumable-walk chunked kernel, then DEFER.
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02bk; mkdir -p $R/$O
cd $R
SWEEP_VARS="RT_AMD_READY=32,48,56,62 RT_AMD_REFILL=1,4,16" timeout -k 10 400 python -u tools/env_sweep.py spheres100k > $O/ready_refill.jsonl 2> $O/err1.log || exit $?
SWEEP_VARS="RT_AMD_DEFER=0,1 RT_AMD_LDS_SCENE=auto" timeout -k 10 200 python -u tools/env_sweep.py spheres100k > $O/defer.jsonl 2> $O/err2.log || exit $?
exit 0
