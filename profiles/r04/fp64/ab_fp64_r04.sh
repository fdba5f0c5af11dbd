#!/bin/bash
# fp64 sqrt / reciprocal shortcuts A/B: RT_FP64_SHORT 3 (main build), 0, 1 (unit / divide only), 2 (sqrt only).
export OUT=${OUT:-gpurun_out/r04_fp64b} CFGS=$'cornell \nspheres --scene spheres --spp 64 --depth 8\nrain --scene rain --width 1920 --spp 512 --depth 16'
export ARMS=$'s3\ns0 RT_AMD_VARIANT=nofp64short\ns1 RT_AMD_VARIANT=fp64unit\ns2 RT_AMD_VARIANT=fp64sqrt\ns3b\ns0b RT_AMD_VARIANT=nofp64short\ns1b RT_AMD_VARIANT=fp64unit\ns2b RT_AMD_VARIANT=fp64sqrt'
bash tools/ab_env.sh && python tools/ab_table.py $OUT > $OUT/table.txt
