# coop v2 / leaf prefetch: parity of each variant, then the A/B
K="ref_precision_matches_oracle or fast_traversal_equals or reference_bvh_and_list or sah_tree or chunked_kernel_equals or large_scene_global or full_size_config_rows or random_scenes or edge_cases or config1 or tiny_scenes"
RT_AMD_VARIANT=coop2 bash tools/gpu_run.sh r05_b_coop2 "pytest:$K" || exit $?
RT_AMD_VARIANT=pf2 bash tools/gpu_run.sh r05_b_pf2 "pytest:$K" || exit $?
export CFGS="sph --scene spheres --spp 64 --depth 8
s100k --scene spheres100k --width 2048 --spp 16 --depth 100
rain --scene rain --width 1920 --spp 128 --depth 16"
export ARMS="base -
coop2 coop2
pf1 pf1
pf2 pf2"
bash tools/gpu_run.sh r05_b abvar || exit $?
RT_AMD_VARIANT=coop2 bash tools/gpu_run.sh r05_b_coop2 sections:spheres sections:spheres100k || exit $?
