#!/bin/bash
# parity, then bench scenes for the default and each env setting in $ABENVS
# (space-separated; commas inside one setting separate variables, e.g. "A=0,B=1 C=2")
mkdir -p gpurun_out
ok() { [ $1 -eq 0 ]; }
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log; ok $rc || exit $rc
fi
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
n=0
for e in base $ABENVS; do
  n=$((n+1)); tag=$n
  if [ $e = base ]; then EV=""; else EV="${e//,/ }"; fi
  env $EV $B > gpurun_out/b_${tag}_cornell.log 2>&1 || exit $?
  env $EV $B --scene spheres --spp 64 --depth 8 > gpurun_out/b_${tag}_spheres.log 2>&1 || exit $?
  if [ -n "$RAIN" ]; then env $EV $B --scene rain --width 1920 --spp 128 --depth 16 --steps 3 > gpurun_out/b_${tag}_rain.log 2>&1 || exit $?; fi
  if [ -n "$BIG" ]; then env $EV timeout -k 10 300 python bench.py --scene spheres100k --width 4096 --spp 16 --depth 100 --steps 2 --warmup 1 --no-cpu > gpurun_out/b_${tag}_100k.log 2>&1 || exit $?; fi
  echo "$tag: $e" >> gpurun_out/b_tags.txt
done
exit 0
