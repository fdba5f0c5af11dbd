# machine scheduler strategy on top of the no-LICM kernel units (variants ilp / memclause)
export CFGS="cor --scene cornell
sph --scene spheres --spp 64 --depth 8
rain --scene rain --width 1920 --spp 128 --depth 16
s100k --scene spheres100k --width 2048 --spp 16 --depth 100"
export ARMS="base -
ilp ilp
mc memclause
base2 -
ilp2 ilp"
bash tools/gpu_run.sh r05_p abvar || exit $?
