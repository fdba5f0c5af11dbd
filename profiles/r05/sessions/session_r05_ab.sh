# adapt kernel: integer countdown to the convergence checks (new default) vs the fp64 fmod per sample
# (variant prev = the previous build's library) - adaptive parity tests, then adaptive lines
bash tools/gpu_run.sh r05_ab "pytest:adaptive" || exit $?
export CFGS="cor --scene cornell --adaptive
sph --scene spheres --spp 64 --depth 8 --adaptive
rain --scene rain --width 1920 --spp 512 --depth 16 --adaptive
def --scene default --adaptive"
export ARMS="base -
prev prev
base2 -
prev2 prev"
bash tools/gpu_run.sh r05_ab abvar || exit $?
