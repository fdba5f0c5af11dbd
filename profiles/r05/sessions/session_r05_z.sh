# adaptive rounds: pixels per round (RT_AMD_ADAPT_LOG) for Cornell, spheres-500, rain and the default scene
mkdir -p gpurun_out/r05_z
for sc in "--scene cornell" "--scene spheres --spp 64 --depth 8" "--scene rain --width 1920 --spp 512 --depth 16" "--scene default"; do
  RT_AMD_ADAPT_LOG=1 timeout -k 10 120 python bench.py $sc --adaptive --steps 1 --warmup 0 --repeats 1 --no-cpu --no-count --no-parity >> gpurun_out/r05_z/adapt_log.txt 2>&1 || exit $?
  RT_AMD_ADAPT_LOG=1 RT_AMD_ADAPT_JUMP=300 timeout -k 10 120 python bench.py $sc --adaptive --steps 3 --warmup 1 --repeats 1 --no-cpu --no-count --no-parity >> gpurun_out/r05_z/adapt_log_j300.txt 2>&1 || exit $?
  timeout -k 10 120 python bench.py $sc --adaptive --steps 3 --warmup 1 --repeats 1 --no-cpu --no-count --no-parity >> gpurun_out/r05_z/adapt_base.txt 2>&1 || exit $?
done
