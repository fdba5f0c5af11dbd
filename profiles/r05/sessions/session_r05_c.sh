# deferred diffuse shading (RT_DEFER_DIFFUSE 32 / 48) and compressed nodes (RT_AMD_QNODES):
# parity, A/B; the all-group rank-share rehearsal
K="ref_precision_matches_oracle or fast_traversal_equals or reference_bvh_and_list or sah_tree or chunked_kernel_equals or large_scene_global or full_size_config_rows or random_scenes or edge_cases or config1 or tiny_scenes or adaptive_rounds_match"
RT_AMD_VARIANT=dd32 bash tools/gpu_run.sh r05_c_dd32 "pytest:$K" || exit $?
RT_AMD_QNODES=1 bash tools/gpu_run.sh r05_c_q "pytest:large_scene_global or full_size_config_rows or config5" || exit $?
export CFGS="sph --scene spheres --spp 64 --depth 8
s100k --scene spheres100k --width 2048 --spp 16 --depth 100
rain --scene rain --width 1920 --spp 128 --depth 16"
export ARMS="base -
dd32 dd32
dd48 dd48"
bash tools/gpu_run.sh r05_c abvar || exit $?
export CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100"
export ARMS="q0 RT_AMD_QNODES=0
q1 RT_AMD_QNODES=1
q0b RT_AMD_QNODES=0
q1b RT_AMD_QNODES=1"
bash tools/gpu_run.sh r05_cq ab || exit $?
bash tools/gpu_run.sh r05_c rankshare || exit $?
