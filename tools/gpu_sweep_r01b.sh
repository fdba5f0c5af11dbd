#!/bin/bash
SWEEP="c_base RT_AMD_REFILL=4
c_ref2 RT_AMD_REFILL=2
c_ref8 RT_AMD_REFILL=8
c_ref16 RT_AMD_REFILL=16
c_pool2 RT_AMD_POOL=2
c_ch16 RT_AMD_CHUNK=16
c_ch64 RT_AMD_CHUNK=64" bash tools/gpu_env_sweep.sh || exit $?
SWEEP="s_base RT_AMD_REFILL=4
s_ref8 RT_AMD_REFILL=8
s_ref16 RT_AMD_REFILL=16
s_rdy40 RT_AMD_READY=40
s_rdy56 RT_AMD_READY=56" BENCH_ARGS="--scene spheres --spp 64 --depth 8" bash tools/gpu_env_sweep.sh || exit $?
