# pool kernel at 5 waves per SIMD: two 640-thread workgroups per CU (<= 96 VGPRs, 112 / 116 path
# slots per wave) vs one 1024-thread workgroup (4 waves per SIMD, 152 slots)
export CFGS="cor --scene cornell
fp32 --scene cornell --precision fp32"
export ARMS="base -
k112 p5k112
k116 p5k116
base2 -
k1162 p5k116"
bash tools/gpu_run.sh r05_s abvar || exit $?
RT_AMD_VARIANT=p5k116 bash tools/gpu_run.sh r05_s "pytest:pool or cornell or adaptive_rounds or chunked_kernel_equals" || exit $?
