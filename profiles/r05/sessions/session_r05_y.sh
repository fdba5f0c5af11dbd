mkdir -p gpurun_out/r05_y
RT_AMD_LAUNCH_LOG=1 timeout -k 10 120 python bench.py --scene spheres100k --width 2048 --spp 16 --depth 100 --steps 1 --warmup 0 --no-cpu --no-count --no-parity --repeats 1 > gpurun_out/r05_y/launch_log.txt 2>&1 || exit $?
