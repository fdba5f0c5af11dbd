#!/bin/bash
# Round-4 probes of the spheres-500 N=8 share floor: fixed-cost fit and hand-out / walk knobs.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04_m; mkdir -p $O
timeout -k 10 200 python tools/fixed_cost.py spheres > $O/fixed_spheres.log 2>&1 || exit $?
ARMS="base
ready16 RT_AMD_READY=16
ready32 RT_AMD_READY=32
ready56 RT_AMD_READY=56
pool1 RT_AMD_POOL=1
pool4 RT_AMD_POOL=4
refill1 RT_AMD_REFILL=1
refill16 RT_AMD_REFILL=16
chunk2 RT_AMD_CHUNK=2
base2" SWEEP_N="8 1" timeout -k 10 300 python tools/knob_sweep.py spheres > $O/knobs_spheres.log 2>&1 || exit $?
