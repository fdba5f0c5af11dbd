#!/bin/bash
# Stage policy A/B (variant pol1: trace first when its queue fills a wave) and the section profile
# of the current pool kernel (variant poolprof: 146 slots + LDS timers).
O=gpurun_out/r02bh; mkdir -p $O
export OUT=$O/ab STEPS=10 CFGS="cornell" ARMS="main
pol1 RT_AMD_VARIANT=pol1
main2
pol12 RT_AMD_VARIANT=pol1"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
RT_AMD_VARIANT=poolprof timeout -k 10 300 python tools/profile_sections.py cornell > $O/sections_pool.log 2>&1 || exit $?
