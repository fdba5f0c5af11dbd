# round-6 session 8: explicit wait after the active-list load (no vmcnt(0) on later writes of its register) - parity subset, A/B vs base
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r06_vmcnt; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "(pair_records or pool or axis_quad or random_scenes or tiny or ref_precision or edge_cases or mixed or near_parallel or lds_budget or adaptive or multi_split or large_scene or chunked_kernel_equals)" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_k.log 2>&1 || exit $?
export STEPS=10
export CFGS="cornell
fp32 --precision fp32
adaptive --adaptive
spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 512 --depth 16
s100k --scene spheres100k --width 4096 --spp 16 --depth 100"
export ARMS="new RT_AMD_NONE=0
base RT_AMD_VARIANT=base"
OUT=$O/ab bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab/table.txt
