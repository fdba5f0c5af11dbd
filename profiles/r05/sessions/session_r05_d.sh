# fp64 leaf records (RT_AMD_TSPH2) + 24-bit node addressing: parity, A/B, the four bench configs
RT_AMD_TSPH2=1 bash tools/gpu_run.sh r05_d_l2 "pytest:large_scene_global or full_size_config_rows or config5 or sah_tree or tiny_scenes" || exit $?
export CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100"
export ARMS="l0 RT_AMD_TSPH2=0
l1 RT_AMD_TSPH2=1
l0b RT_AMD_TSPH2=0
l1b RT_AMD_TSPH2=1"
bash tools/gpu_run.sh r05_d ab || exit $?
bash tools/gpu_run.sh r05_d bench4 || exit $?
