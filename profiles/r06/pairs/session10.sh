# round-6 session 10: pool hand-out knobs re-checked at the final kernel (Cornell N=1, fp32, adaptive)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r06_knobs; mkdir -p $O
export STEPS=20
export CFGS="cornell
fp32 --precision fp32"
export ARMS="d RT_AMD_NONE=0
p4 RT_AMD_POOL=4
p16 RT_AMD_POOL=16
c2 RT_AMD_CHUNK=2
c8 RT_AMD_CHUNK=8
p16c8 RT_AMD_POOL=16 RT_AMD_CHUNK=8
d2 RT_AMD_NONE=0"
OUT=$O/ab bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab/table.txt
