# round-6 session 7: first four candidate bounds in registers - A/B vs HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r06_lotreg; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "(pair_records or pool or axis_quad or random_scenes or tiny or ref_precision or edge_cases or mixed or near_parallel or world_hit or lds_budget)" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_k.log 2>&1 || exit $?
export STEPS=20
export CFGS="cornell
fp32 --precision fp32"
export ARMS="new RT_AMD_NONE=0
base RT_AMD_VARIANT=base
new2 RT_AMD_NONE=0
base2 RT_AMD_VARIANT=base"
OUT=$O/ab bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab/table.txt
