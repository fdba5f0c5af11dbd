#!/bin/bash
# Tile hand-out order A/B (RT_AMD_TILE_ORDER) on one rank's share at N=8 and N=1.
set -o pipefail
O=gpurun_out/r04_order
mkdir -p $O
export ARMS=$'base\ncenter RT_AMD_TILE_ORDER=1\nedge RT_AMD_TILE_ORDER=2'
for sc in spheres rain cornell; do
  SWEEP_N="8 1" timeout -k 10 300 python -u tools/knob_sweep.py $sc > $O/$sc.log 2>&1 || exit $?
done
