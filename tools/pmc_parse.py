#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv) per kernel variant."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
res = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if not any(k in r["Kernel_Name"] for k in ("pt_render", "pt_chunk", "pt_accum")):
            continue
        kn = r["Kernel_Name"].split("(")[0].replace("void rt::", "")
        per[(kn, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (kn, _), cs in per.items():
        for c, v in cs.items():
            res[kn][c] = v  # last dispatch of this variant
for kn, cs in res.items():
    print(kn)
    for c in sorted(cs):
        print(f"   {c:28s} {cs[c]:.4g}")
