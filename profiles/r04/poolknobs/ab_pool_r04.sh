#!/bin/bash
# Pool-kernel hand-out knobs at the round-4 build: Cornell N=1 and a 1/8 share.
set -o pipefail
O=gpurun_out/r04_pool; mkdir -p $O
export ARMS=$'base\npool4 RT_AMD_POOL=4\npool16 RT_AMD_POOL=16\nchunk2 RT_AMD_CHUNK=2\nchunk8 RT_AMD_CHUNK=8\nchunk16 RT_AMD_CHUNK=16\nunguided RT_AMD_GUIDED=0 RT_AMD_CHUNK=4\nbase2'
SWEEP_N="1 8" timeout -k 10 400 python -u tools/knob_sweep.py cornell > $O/cornell.log 2>&1
