# round-6 session 11: the pre-filter record loop unrolled by 2 (variant unroll2) vs the final build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r06_unroll2; mkdir -p $O
export STEPS=20
export CFGS="cornell
fp32 --precision fp32"
export ARMS="d RT_AMD_NONE=0
u2 RT_AMD_VARIANT=unroll2
d2 RT_AMD_NONE=0
u22 RT_AMD_VARIANT=unroll2"
OUT=$O/ab bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab/table.txt
