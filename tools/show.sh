#!/bin/bash
tail -n2 gpurun_out/pytest_gpu.log
for f in gpurun_out/b_*.log; do python3 -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')]
d=json.loads(l[-1]) if l else None
print('$f', d and (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline'].get('accum_kernel_ms')))"; done
[ -f gpurun_out/sections.log ] && grep -v amdgpu gpurun_out/sections.log
