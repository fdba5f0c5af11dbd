#!/usr/bin/env python3
"""Table of value / kernel ms / accumulate ms of the bench lines under a directory (tools/ab_env.sh)."""
import glob, json, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
for f in sorted(glob.glob(f"{d}/*.log")):
    for ln in open(f):
        if ln.startswith("{"):
            x = json.loads(ln)
            r = x["roofline"]
            print(f"{f.split('/')[-1][:-4]:28s} {x['value']:10.1f} Msamples/s  path {r['kernel_ms']:9.3f} ms  "
                  f"accum {r.get('accum_kernel_ms', 0):7.3f} ms  passes {r.get('passes')}")
