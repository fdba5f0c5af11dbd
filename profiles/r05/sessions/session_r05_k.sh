# LDS-resident trees: leaf size x deferred exact tests (env)
export CFGS="sph --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16"
export ARMS="base RT_AMD_SAH_CT=1
d0 RT_AMD_DEFER=0
d0l1 RT_AMD_DEFER=0 RT_AMD_SAH_MAXLEAF=1 RT_AMD_SAH_FORCELEAF=1
d0l2 RT_AMD_DEFER=0 RT_AMD_SAH_MAXLEAF=2 RT_AMD_SAH_FORCELEAF=1
d1l1 RT_AMD_DEFER=1 RT_AMD_SAH_MAXLEAF=1 RT_AMD_SAH_FORCELEAF=1
l1 RT_AMD_SAH_MAXLEAF=1 RT_AMD_SAH_FORCELEAF=1"
bash tools/gpu_run.sh r05_k ab || exit $?
