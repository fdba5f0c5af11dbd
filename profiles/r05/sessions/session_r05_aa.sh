# adaptive round-length rule: jump to the remaining samples when few carried pixels are expected to
# converge within the next round (RT_AMD_ADAPT_LIKELY per mille) - logs, timing, parity
mkdir -p gpurun_out/r05_aa
for sc in "--scene cornell" "--scene spheres --spp 64 --depth 8" "--scene rain --width 1920 --spp 512 --depth 16" "--scene default"; do
  RT_AMD_ADAPT_LOG=1 timeout -k 10 120 python bench.py $sc --adaptive --steps 1 --warmup 0 --repeats 1 --no-cpu --no-count --no-parity >> gpurun_out/r05_aa/log_base.txt 2>&1 || exit $?
  RT_AMD_ADAPT_LOG=1 RT_AMD_ADAPT_LIKELY=100 timeout -k 10 120 python bench.py $sc --adaptive --steps 1 --warmup 0 --repeats 1 --no-cpu --no-count --no-parity >> gpurun_out/r05_aa/log_l100.txt 2>&1 || exit $?
done
export CFGS="cor --scene cornell --adaptive
sph --scene spheres --spp 64 --depth 8 --adaptive
rain --scene rain --width 1920 --spp 512 --depth 16 --adaptive
def --scene default --adaptive"
export ARMS="base RT_AMD_ADAPT_LIKELY=0
l100 RT_AMD_ADAPT_LIKELY=100
l200 RT_AMD_ADAPT_LIKELY=200
l50 RT_AMD_ADAPT_LIKELY=50
base2 RT_AMD_ADAPT_LIKELY=0"
bash tools/gpu_run.sh r05_aa ab || exit $?
RT_AMD_ADAPT_LIKELY=100 bash tools/gpu_run.sh r05_aa "pytest:adaptive" || exit $?
