#!/bin/bash
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 300 python tools/profile_sections.py cornell spheres > $O/sections.log 2>&1 || exit $?
RT_AMD_FOLD=128 RT_AMD_POOL=1 timeout -k 10 300 python tools/profile_sections.py cornell > $O/sections_fold128.log 2>&1 || exit $?
