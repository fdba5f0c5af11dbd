# 24-bit node multiply (variant nomul = without), fp64 leaf records, SAH constants (env, host-side tree)
export CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100
sph --scene spheres --spp 64 --depth 8"
export ARMS="base -
nomul nomul
base2 -
nomul2 nomul"
bash tools/gpu_run.sh r05_e abvar || exit $?
export ARMS="l1 RT_AMD_TSPH2=1
ct05 RT_AMD_TSPH2=1 RT_AMD_SAH_CT=0.5
ct2 RT_AMD_TSPH2=1 RT_AMD_SAH_CT=2
leaf2 RT_AMD_TSPH2=1 RT_AMD_SAH_MAXLEAF=2 RT_AMD_SAH_FORCELEAF=1
leaf6 RT_AMD_TSPH2=1 RT_AMD_SAH_MAXLEAF=6"
bash tools/gpu_run.sh r05_es ab || exit $?
