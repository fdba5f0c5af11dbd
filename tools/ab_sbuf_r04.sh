#!/bin/bash
# Record-buffer budget A/B (RT_AMD_SBUF_MB): fewer, larger passes for rain 1080p spp512 and config 5.
export OUT=${OUT:-gpurun_out/r04_sbuf} CFGS=$'rain --scene rain --width 1920 --spp 512 --depth 16'
export ARMS=$'mb8192\nmb16384 RT_AMD_SBUF_MB=16384\nmb32768 RT_AMD_SBUF_MB=32768\nmb8192b'
bash tools/ab_env.sh || exit $?
export CFGS=$'cfg5 --scene spheres100k --width 4096 --spp 1024 --depth 100' ARMS=$'mb8192\nmb32768 RT_AMD_SBUF_MB=32768' STEPS=1 TLIM=300
bash tools/ab_env.sh && python tools/ab_table.py $OUT > $OUT/table.txt
