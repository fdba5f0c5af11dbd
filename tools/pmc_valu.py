#!/usr/bin/env python3
"""Fold the VALU counter passes (tools/pmc_valu.sh) into profiles/pmc_valu.json.

Per configuration, for the dominant product kernel (pt_pool_kernel, else
pt_chunk_kernel, else pt_render_kernel; INSTR=0 build), counters averaged over
its dispatches and the dispatch duration from the same runs' kernel traces.
Per-sample figures are per RENDER: a multi-pass launch (record budget) makes
`passes` dispatches per render (the bench line's roofline.passes), so the
per-dispatch average is multiplied by passes before dividing by the samples. Derived figures
(units per MI355X_MICROARCH.md: SQ_ACTIVE_INST_* count quad-cycles,
GRBM_GUI_ACTIVE is summed over the 8 XCDs):
  clock_ghz   = GRBM_GUI_ACTIVE / 8 / duration
  lane_util   = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)  (active lanes per VALU op)
  valu_busy   = estimated VALU issue cycles / (1024 SIMDs * duration cycles), issue cost per
                wave64 instruction on a SIMD-32: 2 cycles (f32/int/move/compare/convert),
                4 (f64 add/mul/fma: half rate), 8 (f32 transcendental), 16 (f64 transcendental)
  f64_tflops  = (ADD_F64 + MUL_F64 + 2 FMA_F64) * 64 * lane_util / duration
  vs the MI355X vector peaks: fp64 78.6 TFLOP/s (datasheet), fp32 157.3 (MI355X_MICROARCH.md).
"""
import collections
import csv
import glob
import json
import os
import re
import sys
from pathlib import Path

root = Path(sys.argv[1])
cfgs = sys.argv[2:]
# PMC_VALU_OUT: another output file (A/B runs); PMC_TAG: suffix of the configuration key
out_path = Path(os.environ.get("PMC_VALU_OUT") or Path(sys.argv[0]).resolve().parents[1] / "profiles" / "pmc_valu.json")
TAG = os.environ.get("PMC_TAG", "")
data = json.loads(out_path.read_text()) if out_path.exists() else {}
F64_PEAK, F32_PEAK, SIMDS = 78.6, 157.3, 1024


def dominant(name):
    if re.search(r"pt_pool_kernel<", name):
        return "pt_pool_kernel"  # product-only kernel
    m = re.search(r"(pt_chunk_kernel|pt_render_kernel)<([^>(]*)>", name)
    if not m or [a.strip() for a in m.group(2).split(",")][2] != "0":
        return None  # other kernels / instrumented builds (template args: Real, EMIT, INSTR, TRAV, LDSS)
    return m.group(1)


def pass_counters(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(str(d / "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = dominant(r["Kernel_Name"])
            if k:
                per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return per


def pass_durations(d):
    out = collections.defaultdict(list)
    for f in glob.glob(str(d / "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            k = dominant(r["Kernel_Name"])
            if k:
                out[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return out


for n, args in enumerate(cfgs, 1):
    acc = collections.defaultdict(list)
    durs = collections.defaultdict(list)
    kern = None
    line = None
    for p in sorted(glob.glob(str(root / f"c{n}_p*")), key=lambda x: x):
        pd = Path(p)
        if not pd.is_dir():
            continue
        for (k, _), cs in pass_counters(pd).items():
            kern = k if kern is None or k in ("pt_chunk_kernel", "pt_pool_kernel") else kern
            for c, v in cs.items():
                acc[(k, c)].append(v)
        for k, v in pass_durations(pd).items():
            durs[k] += v
        log = Path(str(pd) + ".log").read_text()
        js = [x for x in log.splitlines() if x.startswith("{")]
        if js:
            line = json.loads(js[-1])
    if kern is None or line is None:
        print(f"cfg {n}: no data", file=sys.stderr)
        continue
    c = {name: sum(v) / len(v) for (k, name), v in acc.items() if k == kern}
    dur = sum(durs[kern]) / len(durs[kern])
    clock = c["GRBM_GUI_ACTIVE"] / 8 / dur
    lane = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
    f64 = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_FMA_F64"]
    tr64, tr32 = c["SQ_INSTS_VALU_TRANS_F64"], c["SQ_INSTS_VALU_TRANS_F32"]
    other = c["SQ_INSTS_VALU"] - f64 - tr64 - tr32
    issue = 2 * other + 4 * f64 + 8 * tr32 + 16 * tr64
    busy = issue / (SIMDS * dur * clock)
    f64_flops = (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + 2 * c["SQ_INSTS_VALU_FMA_F64"]) * 64 * lane
    f32_flops = (c["SQ_INSTS_VALU_ADD_F32"] + c["SQ_INSTS_VALU_MUL_F32"] + 2 * c["SQ_INSTS_VALU_FMA_F32"]) * 64 * lane
    cfg = line["config"]
    # a render of a multi-pass launch (config 4's rain, config 5) is `passes` dispatches:
    # counters are averaged per dispatch above, so per-sample figures scale by passes
    passes = int(line.get("roofline", {}).get("passes") or 1)
    key = f"{cfg['scene']}_{cfg['width']}x{cfg['height']}_spp{cfg['spp']}_d{cfg['depth']}_{cfg['precision']}_n{line['n_gpus']}{'_adaptive' if cfg.get('adaptive') else ''}{TAG}"
    samples = cfg.get("samples_per_frame") or cfg["width"] * cfg["height"] * cfg["spp"]
    entry = {
        "kernel": kern, "duration_ms": round(dur * 1e3, 4), "clock_ghz": round(clock / 1e9, 3),
        "valu_busy": round(busy, 4), "lane_util": round(lane, 4),
        "passes": passes, "launch_ms": round(dur * passes * 1e3, 4),
        "valu_insts_per_sample": round(c["SQ_INSTS_VALU"] * passes * 64 / samples, 1),
        "salu_insts_per_sample": round(c["SQ_INSTS_SALU"] * passes * 64 / samples, 1),
        "f64_tflops": round(f64_flops / dur / 1e12, 3), "f64_peak_tflops": F64_PEAK,
        "f64_frac": round(f64_flops / dur / 1e12 / F64_PEAK, 4),
        "f32_tflops": round(f32_flops / dur / 1e12, 3), "f32_peak_tflops": F32_PEAK,
        "mix": {k.replace("SQ_INSTS_VALU_", "").lower(): round(v / c["SQ_INSTS_VALU"], 4)
                for k, v in c.items() if k.startswith("SQ_INSTS_VALU_")},
        "counters": {k: v for k, v in sorted(c.items())},
        "bench_args": args,
        "build_id": line.get("build_id"),
    }
    data[key] = entry
    print(key, json.dumps({k: v for k, v in entry.items() if k != "counters"}))
out_path.parent.mkdir(exist_ok=True)
out_path.write_text(json.dumps(data, indent=1, sort_keys=True) + "\n")
