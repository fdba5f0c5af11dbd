#!/bin/bash
# Resumable-walk READY x REFILL on small launches: rank 0's 1/8 share of spheres-500 and rain, and spheres-500 at N=1.
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02bp; mkdir -p $R/$O
cd $R
V="RT_AMD_READY=16,32,40,48,56 RT_AMD_REFILL=1,4"
SWEEP_TG=8 SWEEP_VARS="$V" timeout -k 10 200 python -u tools/env_sweep.py spheres > $O/spheres_n8.jsonl 2> $O/e1.log || exit $?
SWEEP_TG=8 SWEEP_VARS="$V" timeout -k 10 300 python -u tools/env_sweep.py rain > $O/rain_n8.jsonl 2> $O/e2.log || exit $?
SWEEP_TG=1 SWEEP_VARS="$V" timeout -k 10 200 python -u tools/env_sweep.py spheres > $O/spheres_n1.jsonl 2> $O/e3.log || exit $?
exit 0
