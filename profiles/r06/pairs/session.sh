# round-6 session: packed-fp32 pair records in the brute-force pre-filter - parity subset, A/B vs HEAD (variant base)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r06_pairs; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -k "pair_records or pool or ref_precision or random_scenes or tiny or axis_quad or near_parallel or mixed or edge_cases or full_size_config_rows or adaptive_sampling or fp32 or multi_split" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_k.log 2>&1 || exit $?
export STEPS=20
export CFGS="cornell
fp32 --precision fp32
adaptive --adaptive"
export ARMS="new RT_AMD_NONE=0
base RT_AMD_VARIANT=base
new2 RT_AMD_NONE=0
base2 RT_AMD_VARIANT=base"
OUT=$O/ab bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab/table.txt
