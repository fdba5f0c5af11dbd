#!/bin/bash
# fp64 sqrt / reciprocal shortcuts A/B (RT_FP64_SHORT=0 variant), interleaved arms.
export OUT=gpurun_out/r04_fp64 CFGS=$'cornell \nspheres --scene spheres --spp 64 --depth 8'
export ARMS=$'base\nnoshort RT_AMD_VARIANT=nofp64short\nbase2\nnoshort2 RT_AMD_VARIANT=nofp64short'
bash tools/ab_env.sh && python tools/ab_table.py $OUT > $OUT/table.txt
