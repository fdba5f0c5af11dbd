# 16-bit LDS walk stacks (LDS-resident trees: materials fit the LDS copy) vs 32-bit (variant stk32):
# parity on every LDS-tree scene, A/B
K="ref_precision_matches_oracle or fast_traversal_equals or reference_bvh_and_list or sah_tree or chunked_kernel_equals or random_scenes or edge_cases or config1 or tiny_scenes or full_size_config_rows or adaptive_rounds_match or camera_configurations or world_hit"
bash tools/gpu_run.sh r05_j "pytest:$K" || exit $?
export CFGS="sph --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16"
export ARMS="base -
stk32 stk32
base2 -
stk32b stk32"
bash tools/gpu_run.sh r05_j abvar || exit $?
RT_AMD_LAUNCH_LOG=1 timeout 120 python bench.py --scene spheres --spp 64 --depth 8 --steps 1 --warmup 0 --repeats 1 --no-cpu --no-count --no-parity > gpurun_out/r05_j/launch_log.txt 2>&1 || exit $?
