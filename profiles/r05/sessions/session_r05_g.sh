# SAH leaf size for trees walked from global memory (1 vs 2) and for LDS-resident trees; config 5
export CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100"
export ARMS="leaf2 RT_AMD_SAH_MAXLEAF=2
leaf1 RT_AMD_SAH_MAXLEAF=1
leaf2b RT_AMD_SAH_MAXLEAF=2
leaf1b RT_AMD_SAH_MAXLEAF=1
leaf1ct05 RT_AMD_SAH_MAXLEAF=1 RT_AMD_SAH_CT=0.5
leaf1q RT_AMD_SAH_MAXLEAF=1 RT_AMD_QNODES=1"
bash tools/gpu_run.sh r05_g ab || exit $?
export CFGS="sph --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16"
export ARMS="base -
leaf3 RT_AMD_SAH_MAXLEAF=3
leaf3f1 RT_AMD_SAH_MAXLEAF=3 RT_AMD_SAH_FORCELEAF=1
ct15 RT_AMD_SAH_CT=1.5
leaf5 RT_AMD_SAH_MAXLEAF=5"
bash tools/gpu_run.sh r05_gs ab || exit $?
RT_AMD_SAH_MAXLEAF=1 bash tools/gpu_run.sh r05_g config5 || exit $?
