#!/bin/bash
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_gpu3.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu3.log; ok $rc || exit $rc
for s in cornell spheres rain; do
  for p in ref fp32; do
    a="--spp 256 --depth 16"; [ $s = spheres ] && a="--spp 64 --depth 8"
    [ $s = rain ] && a="--width 1920 --spp 64 --depth 16"
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --scene $s --precision $p $a > gpurun_out/b3_${s}_$p.log 2>&1 || exit $?
  done
done
