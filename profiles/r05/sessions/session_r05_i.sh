# global trees with one-primitive leaves: two parked leaves (variant wl2), min_ready, hand-out knobs
export CFGS="s100k --scene spheres100k --width 2048 --spp 16 --depth 100
s4k --scene spheres100k --width 4096 --spp 16 --depth 100"
export ARMS="base -
wl2 wl2"
bash tools/gpu_run.sh r05_i abvar || exit $?
export CFGS="s4k --scene spheres100k --width 4096 --spp 16 --depth 100"
export ARMS="r40 RT_AMD_READY=40
r32 RT_AMD_READY=32
r48 RT_AMD_READY=48
r24 RT_AMD_READY=24
p4 RT_AMD_POOL=4
c1 RT_AMD_CHUNK=1
c4 RT_AMD_CHUNK=4"
bash tools/gpu_run.sh r05_ik ab || exit $?
