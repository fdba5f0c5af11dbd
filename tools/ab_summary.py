#!/usr/bin/env python3
"""Print value / kernel ms of every gpurun_out/ab_*.log bench line."""
import glob, json
for f in sorted(glob.glob("gpurun_out/ab_*.log")):
    for ln in open(f):
        if ln.startswith("{"):
            d = json.loads(ln)
            print(f"{f.split('/')[-1]:32s} {d['value']:10.1f} Msamples/s  kernel {d['roofline']['kernel_ms']:8.3f} ms")
