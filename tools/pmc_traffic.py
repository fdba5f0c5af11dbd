#!/usr/bin/env python3
"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json.

Per configuration: the dominant kernel's (pt_pool_kernel, else pt_chunk_kernel, else
pt_render_kernel; product build INSTR=0) counters averaged over its dispatches,
times the dispatches per render of a multi-pass launch (roofline.passes). FETCH_SIZE and
WRITE_SIZE are in KiB. gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE counts half the bytes of wide coalesced streaming reads, so the
corrected read bytes are 2x FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane
stores (the sample-record writes). The path kernel's other reads (scene, L2-
resident) are narrow and uncalibrated: both raw and corrected values are kept.
"""
import collections
import csv
import glob
import json
import re
import sys
from pathlib import Path

root = Path(sys.argv[1])
cfgs = sys.argv[2:]
out_path = Path(sys.argv[0]).resolve().parents[1] / "profiles" / "pmc_traffic.json"
data = json.loads(out_path.read_text()) if out_path.exists() else {}


def kernel_avg(csv_path, counter):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(csv_path)):
        name = r["Kernel_Name"]
        m = re.search(r"(pt_pool_kernel|pt_chunk_kernel|pt_render_kernel|pt_accum_kernel)<?([^>(]*)", name)
        if not m or r["Counter_Name"] != counter:
            continue
        tmpl = m.group(2)
        if m.group(1) not in ("pt_accum_kernel", "pt_pool_kernel") and ", 0, " not in tmpl:
            continue  # instrumented builds (the pool kernel has product builds only)
        per[m.group(1)][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in per.items() if v}


for n, args in enumerate(cfgs, 1):
    fetch = kernel_avg(next(iter(glob.glob(str(root / f"c{n}_FETCH_SIZE" / "*counter_collection.csv")))), "FETCH_SIZE")
    write = kernel_avg(next(iter(glob.glob(str(root / f"c{n}_WRITE_SIZE" / "*counter_collection.csv")))), "WRITE_SIZE")
    log = (root / f"c{n}_FETCH_SIZE.log").read_text()
    line = json.loads([x for x in log.splitlines() if x.startswith("{")][-1])
    cfg = line["config"]
    key = f"{cfg['scene']}_{cfg['width']}x{cfg['height']}_spp{cfg['spp']}_d{cfg['depth']}_{cfg['precision']}_n{line['n_gpus']}{'_adaptive' if cfg.get('adaptive') else ''}"
    dom = next((k for k in ("pt_pool_kernel", "pt_chunk_kernel") if k in fetch), "pt_render_kernel")
    # per RENDER (the bench line's roofline divides by the whole launch's kernel time):
    # a multi-pass launch makes `passes` dispatches of the path kernel per render
    passes = int(line.get("roofline", {}).get("passes") or 1)
    f_kib, w_kib = fetch.get(dom, 0.0) * passes, write.get(dom, 0.0) * passes
    entry = {
        "kernel": dom, "passes": passes,
        "fetch_size_kib": f_kib, "write_size_kib": w_kib,
        "hbm_bytes_per_launch": (2.0 * f_kib + w_kib) * 1024.0,
        "hbm_bytes_per_launch_raw": (f_kib + w_kib) * 1024.0,
        "accum_kernel": {"fetch_size_kib": fetch.get("pt_accum_kernel"), "write_size_kib": write.get("pt_accum_kernel")},
        "bench_args": args,
        "build_id": line.get("build_id"),
    }
    data[key] = entry
    print(key, json.dumps(entry))
out_path.parent.mkdir(exist_ok=True)
out_path.write_text(json.dumps(data, indent=1, sort_keys=True) + "\n")
