#!/bin/bash
# Round-end rehearsal: __graft_entry__.smoke() and the default bench line on the final build.
O=gpurun_out/r02bi; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu > $O/bench.log 2>&1 || exit $?
