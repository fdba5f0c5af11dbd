# round-6 session 9: the leaf slot loaded with the leaf-order sphere record - parity subset, A/B vs HEAD (variant head)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r06_kpre; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "(large_scene or random_scenes or tiny or sah_tree or near_parallel or full_size_config_rows or chunked_kernel_equals or fast_traversal_equals or ref_precision)" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_k.log 2>&1 || exit $?
export STEPS=10
export CFGS="spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 512 --depth 16
s100k --scene spheres100k --width 4096 --spp 16 --depth 100"
export ARMS="new RT_AMD_NONE=0
head RT_AMD_VARIANT=head
new2 RT_AMD_NONE=0
head2 RT_AMD_VARIANT=head"
OUT=$O/ab bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab/table.txt
