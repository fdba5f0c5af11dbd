#!/bin/bash
# section profile (active lanes per section) + VALU / traffic counter passes for the headline configs
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 300 python tools/profile_sections.py cornell spheres spheres100k > $O/sections.log 2>&1 || exit $?
bash tools/pmc_valu.sh "" "--scene spheres --spp 64 --depth 8" > $O/valu.log 2>&1 || exit $?
bash tools/pmc_traffic.sh "" > $O/traffic.log 2>&1 || exit $?
exit 0
