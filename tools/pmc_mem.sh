#!/bin/bash
# Memory-stall evidence for one bench config: wave-cycle breakdown (SQ) and L1/L2 traffic (TCP/TCC),
# separate rocprofv3 --pmc passes (kernel-trace only). usage: bash tools/pmc_mem.sh <outdir> "<bench args>"
R=$GRAFT_REPO_ROOT; O=$R/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $O/p$i -o run --output-format csv -- python3 $R/bench.py $2 --steps 2 --warmup 0 --no-cpu --no-count --no-parity > $O/p$i.log 2>&1 || exit $?
done
