#!/bin/bash
# 12-byte records A/B (RT_AMD_REC12=0: 16-byte records with the bounce word).
export OUT=${OUT:-gpurun_out/r04_rec12} CFGS=$'cornell \nspheres --scene spheres --spp 64 --depth 8\nrain --scene rain --width 1920 --spp 512 --depth 16\n100k --scene spheres100k --width 4096 --spp 16 --depth 100'
export ARMS=$'rec12\nrec16 RT_AMD_REC12=0\nrec12b\nrec16b RT_AMD_REC12=0'
bash tools/ab_env.sh && python tools/ab_table.py $OUT > $OUT/table.txt
