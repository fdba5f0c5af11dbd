#!/bin/bash
# Round-2 final evidence at HEAD (non-temporal record stores in the pool kernel): GPU parity (verbose), default bench line (CPU leg), the other
# bench configs (config 5 at spp 1024), rocprofv3 kernel stats of the default bench, HBM traffic
# and VALU passes (separate --pmc runs), rank-share rehearsal. Any failure ends the script.
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02bo; mkdir -p $R/$O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit $?
B="timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu"
$B --precision fp32 > $O/b_cornell_fp32.log 2>&1 || exit $?
$B --scene spheres --spp 64 --depth 8 > $O/b_spheres.log 2>&1 || exit $?
$B --scene rain --width 1920 --spp 512 --depth 16 --steps 3 > $O/b_rain.log 2>&1 || exit $?
$B --scene spheres10 --width 200 --spp 4 --depth 4 > $O/b_config1.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --scene spheres100k --width 4096 --spp 1024 --depth 100 --steps 2 --warmup 1 --no-cpu > $O/b_100k.log 2>&1 || exit $?
for s in cornell spheres rain; do
  timeout -k 10 300 python tools/rank_share.py $s >> $O/rank_share.log 2>&1 || exit $?
done
bash tools/pmc_traffic.sh "" "--scene spheres --spp 64 --depth 8" || exit $?
VALU_DIR=$O/valu PMC_VALU_OUT=$O/pmc_valu.json bash tools/pmc_valu.sh "" "--precision fp32" "--scene spheres --spp 64 --depth 8" "--scene rain --width 1920 --spp 512 --depth 16" "--scene spheres100k --width 4096 --spp 16 --depth 100" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu > $R/$O/prof.log 2>&1 || exit $?
exit 0
