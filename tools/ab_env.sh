#!/bin/bash
# Runtime-knob A/B on several bench configs. $CFGS: lines "tag bench-args"; $ARMS: lines "arm ENV=V ..."
# (arm "base" with no env = defaults). Logs: $OUT/<tag>_<arm>.log; summary via tools/ab_table.py $OUT.
OUT=${OUT:-gpurun_out/ab}; mkdir -p $OUT
echo "$CFGS" | while read -r tag args; do
  [ -z "$tag" ] && continue
  echo "$ARMS" | while read -r arm envs; do
    [ -z "$arm" ] && continue
    env $envs timeout -k 10 ${TLIM:-200} python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu --no-count --no-parity $args > $OUT/${tag}_${arm}.log 2>&1 || exit $?
  done || exit $?
done
