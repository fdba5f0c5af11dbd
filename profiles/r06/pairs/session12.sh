# round-6 session 12: pass 2 without the per-test ray barrier (variant rayhoist) vs the final build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r06_rayhoist; mkdir -p $O
export STEPS=20
export CFGS="cornell
fp32 --precision fp32"
export ARMS="d RT_AMD_NONE=0
h RT_AMD_VARIANT=rayhoist
d2 RT_AMD_NONE=0
h2 RT_AMD_VARIANT=rayhoist"
OUT=$O/ab bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab/table.txt
