#!/bin/bash
# Runtime-knob sweep on the headline bench: each line of $SWEEP is "name ENV=V ..." (no rebuild).
mkdir -p gpurun_out
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu $BENCH_ARGS"
echo "$SWEEP" | while read -r name envs; do
  [ -z "$name" ] && continue
  env $envs $B > gpurun_out/b_${name}.log 2>&1 || exit $?
done
