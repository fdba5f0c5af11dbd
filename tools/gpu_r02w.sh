#!/bin/bash
# Round-2 evidence at HEAD (re-entry): GPU parity, the default bench line (with CPU
# leg), config 5 at its stated workload, rocprofv3 kernel stats of the default
# bench, VALU passes for Cornell ref. Any failure ends the script.
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02w; mkdir -p $R/$O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --scene spheres100k --width 4096 --spp 1024 --depth 100 --steps 2 --warmup 1 --no-cpu > $O/bench_100k.log 2>&1 || exit $?
VALU_DIR=$O/valu PMC_VALU_OUT=$O/pmc_valu_cornell.json bash tools/pmc_valu.sh "" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu > $R/$O/prof.log 2>&1 || exit $?
exit 0
