# no machine-code loop-invariant motion (-mllvm -disable-machine-licm, variant nolicm): the fp64
# constants of ocml's sincos are no longer hoisted into VGPRs and spilled (0 B scratch, 97-126 VGPRs)
export CFGS="cor --scene cornell
sph --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16
s100k --scene spheres100k --width 2048 --spp 16 --depth 100"
export ARMS="base -
nolicm nolicm
base2 -
nolicm2 nolicm"
bash tools/gpu_run.sh r05_o abvar || exit $?
RT_AMD_VARIANT=nolicm bash tools/gpu_run.sh r05_o "pytest:ref_precision_matches_oracle or fast_traversal_equals or sah_tree or chunked_kernel_equals or large_scene_global or random_scenes or edge_cases or config1 or tiny_scenes or pool" || exit $?
