#!/bin/bash
# VALU counters: pool kernel vs chunked kernel on Cornell (ref).
export PMC_VALU_OUT=gpurun_out/r02n/pmc_ab.json
VALU_DIR=gpurun_out/r02n/pool PMC_TAG=_pool bash tools/pmc_valu.sh "" || exit $?
RT_AMD_POOL_KERNEL=0 VALU_DIR=gpurun_out/r02n/chunk PMC_TAG=_chunk bash tools/pmc_valu.sh "" || exit $?
