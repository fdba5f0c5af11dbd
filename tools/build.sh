#!/bin/bash
# Local build + CPU tests; non-zero exit on any failure (gate GPU runs on it).
cd /root/repo || exit 1
python -c "
import sys; sys.path.insert(0,'mcp-raytracer_amd')
from raytracer_amd import _build; _build.build_native()" > /tmp/build.log 2>&1 || { grep -E "error" -A3 /tmp/build.log | head -30; exit 1; }
python -m pytest tests -x -q -m "not gpu" > /tmp/cputest.log 2>&1 || { tail -20 /tmp/cputest.log; exit 1; }
tail -1 /tmp/cputest.log
