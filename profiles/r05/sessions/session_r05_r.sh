# pool-kernel record stores: non-temporal (default) vs plain (variant recnt0) on the no-LICM build,
# with the path kernel's HBM WRITE_SIZE of each (Cornell records: 1.97 GB per frame)
export CFGS="cor --scene cornell"
export ARMS="base -
nt0 recnt0
base2 -
nt02 recnt0"
bash tools/gpu_run.sh r05_r abvar || exit $?
TRAFFIC_DIR=gpurun_out/r05_r/traffic_base bash tools/pmc_traffic.sh "" || exit $?
RT_AMD_VARIANT=recnt0 TRAFFIC_DIR=gpurun_out/r05_r/traffic_nt0 bash tools/pmc_traffic.sh "" || exit $?
