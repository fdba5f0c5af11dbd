# codegen options on top of the no-LICM kernel units: scheduler metric bias 0, AMDGPU register
# pressure trackers, no loop strength reduction, sinking into loops to avoid spills
export CFGS="cor --scene cornell
sph --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16
s100k --scene spheres100k --width 2048 --spp 16 --depth 100"
export ARMS="base -
bias0 bias0
trk trk
nolsr nolsr
sinksp sinksp
base2 -"
bash tools/gpu_run.sh r05_t abvar || exit $?
