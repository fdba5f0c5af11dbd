#!/bin/bash
# Round-3 schedule re-check at the final build: rank shares (SWEEP_TG) under the item-chunk
# (Cornell pool kernel) and min_ready (spheres-500 chunked kernel) knobs, three repeats each.
mkdir -p gpurun_out/sweep2
for rep in 1 2 3; do
  for tg in 1 2 4 8; do
    SWEEP_TG=$tg SWEEP_VARS="RT_AMD_CHUNK=auto,2,1" timeout -k 10 120 python tools/env_sweep.py cornell >> gpurun_out/sweep2/cornell.log 2>&1 || exit $?
    SWEEP_TG=$tg SWEEP_VARS="RT_AMD_READY=auto,40" timeout -k 10 120 python tools/env_sweep.py spheres >> gpurun_out/sweep2/spheres.log 2>&1 || exit $?
  done
done
