#!/bin/bash
# Chunked kernel for every fixed-spp launch + BVH hand-out rule: GPU parity, bench lines,
# rank-share rehearsal (Cornell, spheres-500, rain).
O=gpurun_out/r02ap; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
B="timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu"
$B > $O/b_cornell.log 2>&1 || exit $?
$B --scene spheres --spp 64 --depth 8 > $O/b_spheres.log 2>&1 || exit $?
$B --scene rain --width 1920 --spp 512 --depth 16 --steps 3 > $O/b_rain.log 2>&1 || exit $?
for s in cornell spheres rain; do
  timeout -k 10 300 python tools/rank_share.py $s >> $O/rank_share.log 2>&1 || exit $?
done
