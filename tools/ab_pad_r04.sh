cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh r04_e pytest || exit $?
export OUT=gpurun_out/r04_e/ab CFGS="spheres --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16" ARMS="pad1 RT_AMD_NODE_PAD=1
pad0 RT_AMD_NODE_PAD=0
pad1b RT_AMD_NODE_PAD=1
pad0b RT_AMD_NODE_PAD=0"
STEPS=10 bash tools/ab_env.sh || exit $?
python tools/ab_table.py $OUT > $OUT/table.txt
RT_AMD_VARIANT=poolprof timeout -k 10 300 python tools/profile_sections.py cornell > gpurun_out/r04_e/sections_pool.log 2>&1
