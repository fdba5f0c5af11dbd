# round-6 session: cost-ordered final phase - parity, A/B on the BVH configs and Cornell, rank shares
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r06_cost; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "cost_order or large_scene or spheres or rain or partition or tile_groups or pool" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_k.log 2>&1 || exit $?
export CFGS="cornell
spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 512 --depth 16
s100k --scene spheres100k --width 4096 --spp 16 --depth 100"
export ARMS="on RT_AMD_COST_ORDER=1
off RT_AMD_COST_ORDER=0"
OUT=$O/ab bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab/table.txt
RT_AMD_COST_ORDER=1 timeout -k 10 500 python tools/rank_share.py spheres cornell rain > $O/rank_share_on.log 2>&1 || exit $?
RT_AMD_COST_ORDER=0 timeout -k 10 400 python tools/rank_share.py spheres cornell > $O/rank_share_off.log 2>&1 || exit $?
