mkdir -p gpurun_out/r02a
timeout -k 10 500 python bench.py --scene spheres100k --width 4096 --spp 1024 --depth 100 --steps 1 --warmup 0 --no-cpu > gpurun_out/r02a/b_100k_spp1024.log 2>&1; echo rc=$? >> gpurun_out/r02a/b_100k_spp1024.log
