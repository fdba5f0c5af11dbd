#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each) for the wavefront walk kernel vs the chunked kernel.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd); O=$R/gpurun_out/${TAG:-wfpmc}; mkdir -p $O
A="--scene spheres100k --width 2048 --spp 16 --depth 100 --no-cpu --no-count --no-parity --steps 1 --warmup 0"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r line; do
  i=$((i+1))
  for arm in 1 0; do
    RT_AMD_WAVEFRONT=$arm timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -d $O/wf${arm}_p$i -o run --output-format csv -- python3 $R/bench.py $A > $O/wf${arm}_p$i.log 2>&1 || exit $?
  done
done <<'PASSES'
SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE
SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES
TCC_HIT_sum TCC_MISS_sum
PASSES
