#!/bin/bash
# Runtime-knob sweep (each line of $SWEEP: "name ENV=V ...") on the fast-traversal configs.
mkdir -p gpurun_out
echo "$SWEEP" | while read -r name envs; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 300 python bench.py --scene spheres100k --width 4096 --spp 16 --depth 100 --steps 2 --warmup 1 --no-cpu > gpurun_out/b_100k_$name.log 2>&1 || exit $?
  env $envs timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --scene spheres --spp 64 --depth 8 > gpurun_out/b_spheres_$name.log 2>&1 || exit $?
  env $envs timeout -k 10 120 python tools/tail_probe.py rain 8 > gpurun_out/tail_$name.log 2>&1 || exit $?
done
