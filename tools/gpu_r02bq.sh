#!/bin/bash
# Quantised 64-byte 4-wide nodes (variant q) vs main: BVH parity tests on q, then spheres-100k / spheres-500 / rain.
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02bq; mkdir -p $R/$O
cd $R
RT_AMD_VARIANT=q timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ref_precision or tiny or random or world_hit or config1 or strateg" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_q.log 2>&1 || exit $?
for v in main q; do
  if [ $v = main ]; then unset RT_AMD_VARIANT; else export RT_AMD_VARIANT=$v; fi
  B="timeout -k 10 200 python bench.py --no-cpu --no-count --steps 3 --warmup 1"
  $B --scene spheres100k --width 4096 --spp 16 --depth 100 > $O/b100k_$v.log 2>&1 || exit $?
  $B --scene spheres --spp 64 --depth 8 > $O/bsph_$v.log 2>&1 || exit $?
  $B --scene rain --width 1920 --spp 512 --depth 16 > $O/brain_$v.log 2>&1 || exit $?
done
exit 0
