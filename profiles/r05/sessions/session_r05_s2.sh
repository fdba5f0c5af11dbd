# 5-wave pool kernel: smaller pools (104 / 96 slots) in case two 640-thread workgroups did not fit
# one CU's LDS at 116 slots; the launch log prints the LDS layout
RT_AMD_LAUNCH_LOG=1 RT_AMD_VARIANT=p5k116 timeout -k 10 120 python bench.py --no-cpu --no-count --no-parity --steps 2 --warmup 1 > gpurun_out/r05_s2_log.txt 2>&1 || exit $?
export CFGS="cor --scene cornell"
export ARMS="base -
k104 p5k104
k96 p5k96"
bash tools/gpu_run.sh r05_s2 abvar || exit $?
