#!/bin/bash
# Non-temporal record stores (variant nt) vs main: Cornell bench, WRITE_SIZE of the path kernel, pool parity.
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02bm; mkdir -p $R/$O
cd $R
RT_AMD_VARIANT=nt timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pool_kernel or config1 or gate" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_nt.log 2>&1 || exit $?
for v in main nt; do
  if [ $v = main ]; then unset RT_AMD_VARIANT; else export RT_AMD_VARIANT=$v; fi
  timeout -k 10 200 python bench.py --no-cpu > $O/bench_$v.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --no-cpu --scene spheres --spp 64 --depth 8 > $O/bench_sph_$v.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
for v in main nt; do
  if [ $v = main ]; then unset RT_AMD_VARIANT; else export RT_AMD_VARIANT=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/$O/w_$v -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-count > $R/$O/w_$v.log 2>&1 || exit $?
done
exit 0
