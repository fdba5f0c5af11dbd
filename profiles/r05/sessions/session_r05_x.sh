# tile hand-out order: ascending (default) vs descending (RT_AMD_TILE_ORDER=1) - parity subset with the
# reversed order, then every tile group of N = 2, 4, 8 (tools/rank_share.py) under both
mkdir -p gpurun_out/r05_x
RT_AMD_TILE_ORDER=1 bash tools/gpu_run.sh r05_x "pytest:ref_precision_matches_oracle or chunked_kernel_equals or pool or adaptive_rounds or tile_group or config1 or random_scenes" || exit $?
timeout -k 10 400 python tools/rank_share.py spheres cornell rain > gpurun_out/r05_x/rank_share_base.log 2>&1 || exit $?
RT_AMD_TILE_ORDER=1 timeout -k 10 400 python tools/rank_share.py spheres cornell rain > gpurun_out/r05_x/rank_share_rev.log 2>&1 || exit $?
