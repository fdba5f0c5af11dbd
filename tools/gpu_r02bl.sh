#!/bin/bash
# spheres-100k 4096^2 spp16 d100 (chunked kernel, tree in global memory): L2 and L1 hit
# counts of the path kernel, to size a node-compression change. One --pmc pass per run.
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02bl; mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
A="--scene spheres100k --width 4096 --spp 16 --depth 100 --steps 1 --warmup 0 --no-cpu --no-count"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/$O/p1 -o run --output-format csv -- python3 $R/bench.py $A > $R/$O/p1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $R/$O/p2 -o run --output-format csv -- python3 $R/bench.py $A > $R/$O/p2.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM -d $R/$O/p3 -o run --output-format csv -- python3 $R/bench.py $A > $R/$O/p3.log 2>&1 || exit $?
exit 0
