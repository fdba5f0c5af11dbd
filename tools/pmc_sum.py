#!/usr/bin/env python3
"""Average counters per dispatch of the dominant path kernel from rocprofv3 --pmc output dirs."""
import collections, csv, glob, json, sys
for d in sys.argv[1:]:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "pt_chunk_kernel" in k or "pt_render_kernel" in k or "pt_pool_kernel" in k:
                per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(d, json.dumps({c: sum(v.values()) / len(v) for c, v in sorted(per.items())}, indent=0))
