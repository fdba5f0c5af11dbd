#!/bin/bash
# Pool-kernel section profile (diagnostic variant poolprof: 88 slots + LDS section timers), GPU parity
# of the main build, bench line.
O=gpurun_out/r02au; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
RT_AMD_VARIANT=poolprof timeout -k 10 300 python tools/profile_sections.py cornell > $O/sections_pool.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu > $O/bench.log 2>&1 || exit $?
