#!/bin/bash
# Diagnostics of the headline kernel: section profile + PMC passes (separate runs).
mkdir -p gpurun_out
timeout -k 10 300 python tools/profile_sections.py ${SECTIONS:-cornell spheres} > gpurun_out/sections.log 2>&1 || exit $?
PMC_FILE=${PMC_FILE:-tools/pmc_passes2.txt} bash tools/gpu_pmc.sh || exit $?
cd $GRAFT_REPO_ROOT && python3 tools/pmc_parse.py gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1
exit 0
