#!/bin/bash
# VALU counter passes for Cornell ref at HEAD (pool kernel), folded into profiles/pmc_valu.json.
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02ad; mkdir -p $R/$O
cd $R
VALU_DIR=$O/valu PMC_VALU_OUT=$O/pmc_valu_cornell.json bash tools/pmc_valu.sh "" || exit $?
timeout -k 10 300 python bench.py --no-cpu > $O/bench.log 2>&1 || exit $?
