#!/bin/bash
# parity + benches with and without an env switch ($ABENV, e.g. RT_AMD_BORDER=0)
bash tools/gpu_quick.sh || exit $?
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
env $ABENV $B > gpurun_out/b_cornell_env.log 2>&1 || exit $?
env $ABENV $B --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres_env.log 2>&1 || exit $?
