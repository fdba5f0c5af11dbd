# record-buffer budget: Cornell in passes small enough for each pass's records to stay in the
# 256 MB MALL (rain in one pass vs two: profiles/r04/sbuf/, within noise)
export CFGS="cor --scene cornell"
export ARMS="base RT_AMD_SBUF_MB=8192
m1024 RT_AMD_SBUF_MB=1024
m512 RT_AMD_SBUF_MB=512
m256 RT_AMD_SBUF_MB=256"
bash tools/gpu_run.sh r05_n ab || exit $?
