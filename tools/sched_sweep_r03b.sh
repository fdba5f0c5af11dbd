#!/bin/bash
# smoke at the last build, then rank-share sweeps of the remaining hand-out knobs
# (spheres-500 chunked kernel: tile-chunks per atomic; Cornell fp32 under the spl/64 rule).
mkdir -p gpurun_out/sweep3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/sweep3/smoke.log 2>&1 || exit $?
for rep in 1 2; do
  for tg in 4 8; do
    SWEEP_TG=$tg SWEEP_VARS="RT_AMD_POOL=auto,1,4" timeout -k 10 120 python tools/env_sweep.py spheres >> gpurun_out/sweep3/spheres_pool.log 2>&1 || exit $?
  done
done
