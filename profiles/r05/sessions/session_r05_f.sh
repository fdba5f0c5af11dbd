# compile-time fp64 leaf records for LDSS-0 kernels (variant nol2 = without) x SAH leaf size (env), parity
bash tools/gpu_run.sh r05_f "pytest:large_scene_global or full_size_config_rows or config5 or sah_tree or world_hit" || exit $?
export CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100"
export ARMS="l2 -
nol2 nol2
l2b -
nol2b nol2"
bash tools/gpu_run.sh r05_f abvar || exit $?
export ARMS="leaf2 RT_AMD_SAH_MAXLEAF=2
leaf3 RT_AMD_SAH_MAXLEAF=3
leaf1 RT_AMD_SAH_MAXLEAF=1
leaf4 RT_AMD_SAH_MAXLEAF=4 RT_AMD_SAH_FORCELEAF=2
leaf2f2 RT_AMD_SAH_MAXLEAF=2 RT_AMD_SAH_FORCELEAF=2"
bash tools/gpu_run.sh r05_fs ab || exit $?
bash tools/gpu_run.sh r05_f config5 || exit $?
