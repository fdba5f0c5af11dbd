# leaf 1 default for global trees: parity; parked-leaf record preload (variant pre); SAH for LDS trees; config 5
bash tools/gpu_run.sh r05_h "pytest:large_scene_global or full_size_config_rows or config5 or sah_tree or world_hit or random_scenes" || exit $?
export CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100"
export ARMS="base -
pre pre
base2 -
pre2 pre"
bash tools/gpu_run.sh r05_h abvar || exit $?
export CFGS="sph --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16"
export ARMS="base RT_AMD_SAH_CT=1
leaf3 RT_AMD_SAH_MAXLEAF=3
leaf3f1 RT_AMD_SAH_MAXLEAF=3 RT_AMD_SAH_FORCELEAF=1
ct15 RT_AMD_SAH_CT=1.5
leaf5 RT_AMD_SAH_MAXLEAF=5"
bash tools/gpu_run.sh r05_hs ab || exit $?
bash tools/gpu_run.sh r05_h config5 || exit $?
