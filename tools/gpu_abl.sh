#!/bin/bash
mkdir -p gpurun_out
B="timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu"
for v in main $VARIANTS; do
  if [ $v = main ]; then unset RT_AMD_VARIANT; else export RT_AMD_VARIANT=$v; fi
  $B > gpurun_out/b_cornell_$v.log 2>&1 || exit $?
done
