#!/bin/bash
# Rain rank shares: sequential kernel forced (RT_AMD_CHUNKED=0) vs the chunked defaults.
O=gpurun_out/r02an; mkdir -p $O
RT_AMD_CHUNKED=0 SWEEP_POOL=auto SWEEP_CHUNK=auto SWEEP_N="1 2 4 8" timeout -k 10 300 python tools/sched_sweep.py rain > $O/seq_rain.log 2>&1 || exit $?
SWEEP_POOL="auto 4" SWEEP_CHUNK="auto 8 16" SWEEP_N="2 8" timeout -k 10 300 python tools/sched_sweep.py rain > $O/chunk_rain.log 2>&1 || exit $?
