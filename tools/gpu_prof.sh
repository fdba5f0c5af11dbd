#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python tools/profile_sections.py > gpurun_out/sections.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/sections.log; exit $rc
