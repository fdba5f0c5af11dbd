# pool-kernel hand-out knobs re-checked on the no-LICM build (Cornell headline, fp32):
# tile-chunks per atomic (auto 8), first item length (auto 4), refill threshold (auto 4)
export CFGS="cor --scene cornell"
export ARMS="base RT_AMD_POOL=8
pool4 RT_AMD_POOL=4
pool16 RT_AMD_POOL=16
chunk2 RT_AMD_CHUNK=2
chunk8 RT_AMD_CHUNK=8
refill2 RT_AMD_REFILL=2
refill8 RT_AMD_REFILL=8
base2 RT_AMD_POOL=8"
bash tools/gpu_run.sh r05_u ab || exit $?
