#!/bin/bash
O=gpurun_out/r02h; mkdir -p $O
timeout -k 10 300 python tools/count_exact.py > $O/count_exact.log 2>&1 || exit $?
timeout -k 10 300 python tools/profile_sections.py rain spheres100k > $O/sections.log 2>&1 || exit $?
