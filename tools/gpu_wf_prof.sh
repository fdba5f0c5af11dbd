#!/bin/bash
# rocprofv3 kernel stats of the wavefront passes vs the chunked kernel (spheres-100k 2048^2 spp16).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd); O=$R/gpurun_out/${TAG:-wfprof}; mkdir -p $O
A="--scene spheres100k --width 2048 --spp 16 --depth 100 --no-cpu --no-count --no-parity --steps 2 --warmup 1"
cd /tmp && export TMPDIR=/tmp
RT_AMD_WAVEFRONT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/wf -o run --output-format csv -- python3 $R/bench.py $A > $O/wf.log 2>&1 || exit $?
RT_AMD_WAVEFRONT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/chunked -o run --output-format csv -- python3 $R/bench.py $A > $O/chunked.log 2>&1 || exit $?
