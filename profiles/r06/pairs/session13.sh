# round-6 session 13: accumulate with 16 record loads in flight per lane (variant acc16) vs 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r06_acc16; mkdir -p $O
export STEPS=20
export CFGS="cornell
rain --scene rain --width 1920 --spp 512 --depth 16"
export ARMS="d RT_AMD_NONE=0
a RT_AMD_VARIANT=acc16
d2 RT_AMD_NONE=0
a2 RT_AMD_VARIANT=acc16"
OUT=$O/ab bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab/table.txt
