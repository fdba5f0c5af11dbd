#!/bin/bash
# Round-4 A/B: the axis-quad pre-filter's t margin (kEt 1e-6, product) vs the round-3 margin (1e-5, variant ket5).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04_i; mkdir -p $O
bash tools/gpu_run.sh r04_i pytest || exit $?
timeout -k 10 200 python tools/count_exact.py cornell > $O/count_exact.log 2>&1 || exit $?
RT_AMD_VARIANT=ket5 timeout -k 10 200 python tools/count_exact.py cornell > $O/count_exact_ket5.log 2>&1 || exit $?
export OUT=$O/ab CFGS="cornell --steps 10
cornellfp32 --precision fp32 --steps 10" ARMS="ket6 RT_AMD_VARIANT=
ket5 RT_AMD_VARIANT=ket5
ket6b RT_AMD_VARIANT=
ket5b RT_AMD_VARIANT=ket5"
STEPS=10 bash tools/ab_env.sh || exit $?
python tools/ab_table.py $OUT > $OUT/table.txt
