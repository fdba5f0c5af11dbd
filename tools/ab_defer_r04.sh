#!/bin/bash
# Round-4 A/B: deferred exact sphere tests (RT_AMD_DEFER) after the cheaper node step.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04_j; mkdir -p $O
RT_AMD_DEFER=1 timeout -k 10 200 python tools/count_exact.py spheres100k > $O/count_exact_defer1.log 2>&1 || exit $?
RT_AMD_DEFER=0 timeout -k 10 200 python tools/count_exact.py spheres100k spheres rain > $O/count_exact_defer0.log 2>&1 || exit $?
export OUT=$O/ab CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100
spheres --scene spheres --spp 64 --depth 8" ARMS="auto
d1 RT_AMD_DEFER=1
d0 RT_AMD_DEFER=0
autob
d1b RT_AMD_DEFER=1"
STEPS=5 bash tools/ab_env.sh || exit $?
python tools/ab_table.py $OUT > $OUT/table.txt
