# binary children-in-parent tree (variant bvh2) vs 4-wide on one-primitive-leaf trees; top cache off
export CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100
rain --scene rain --width 1920 --spp 128 --depth 16"
export ARMS="base -
bvh2 bvh2"
bash tools/gpu_run.sh r05_m abvar || exit $?
export CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100"
export ARMS="top1 RT_AMD_TOP_CACHE=1
top0 RT_AMD_TOP_CACHE=0"
bash tools/gpu_run.sh r05_mt ab || exit $?
