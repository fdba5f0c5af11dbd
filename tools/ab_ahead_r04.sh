#!/bin/bash
# Brute-force pre-filter record prefetch A/B (RT_PRE_AHEAD=0 variant 'noahead').
export OUT=${OUT:-gpurun_out/r04_ahead} CFGS=$'cornell \ncornell32 --precision fp32'
export ARMS=$'ahead\nnoahead RT_AMD_VARIANT=noahead\nahead2\nnoahead2 RT_AMD_VARIANT=noahead'
bash tools/ab_env.sh && python tools/ab_table.py $OUT > $OUT/table.txt
