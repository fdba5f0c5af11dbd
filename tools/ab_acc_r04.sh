#!/bin/bash
# Accumulate-pass A/B: unroll (variants acc4 / acc16) and grid cap (RT_AMD_ACC_BLOCKS).
export OUT=${OUT:-gpurun_out/r04_acc} CFGS=$'cornell \nrain --scene rain --width 1920 --spp 512 --depth 16'
export ARMS=$'base\nu4 RT_AMD_VARIANT=acc4\nu16 RT_AMD_VARIANT=acc16\ng4096 RT_AMD_ACC_BLOCKS=4096\ng1024 RT_AMD_ACC_BLOCKS=1024\ng8192 RT_AMD_ACC_BLOCKS=8192\nu16g4096 RT_AMD_VARIANT=acc16 RT_AMD_ACC_BLOCKS=4096\nbase2'
bash tools/ab_env.sh && python tools/ab_table.py $OUT > $OUT/table.txt
