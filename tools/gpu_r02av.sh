#!/bin/bash
# Pool-kernel section profile with the pre-filter timed apart ("tile" = make_fray + pre-filter pass).
O=gpurun_out/r02av; mkdir -p $O
RT_AMD_VARIANT=poolprof timeout -k 10 300 python tools/profile_sections.py cornell > $O/sections_pool.log 2>&1 || exit $?
