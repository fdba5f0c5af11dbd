#!/bin/bash
# Config-5 knob sweep: spheres-100k 4096^2 spp1024, a 1/8 rank share (path kernel over all passes),
# then the combination on the spp16 frame at N=1 and N=8.
set -o pipefail
O=gpurun_out/r04_cfg5
mkdir -p $O
export ARMS=$'base\nr40c2p8 RT_AMD_READY=40 RT_AMD_CHUNK=2 RT_AMD_POOL=8\nc2p8 RT_AMD_CHUNK=2 RT_AMD_POOL=8\nr40p8 RT_AMD_READY=40 RT_AMD_POOL=8\nr40c2 RT_AMD_READY=40 RT_AMD_CHUNK=2'
SWEEP_N="8" SWEEP_SPP=1024 timeout -k 10 600 python -u tools/knob_sweep.py spheres100k > $O/combo.log 2>&1 &&
SWEEP_N="1 8" timeout -k 10 300 python -u tools/knob_sweep.py spheres100k > $O/combo_spp16.log 2>&1
