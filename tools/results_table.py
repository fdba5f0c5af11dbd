#!/usr/bin/env python3
"""Markdown result rows from a folder of bench logs (the JSON line each bench.py run prints):
Msamples/s, ms per frame, path-kernel ms, the VALU roofline (frac, lane utilisation, counters'
build and staleness), HBM fraction and parity. usage: python tools/results_table.py <dir>"""
import json
import sys
from pathlib import Path

ORDER = ["b_cornell", "bench_default", "b_cornell_fp32", "b_adaptive", "b_spheres", "b_rain", "b_100k", "b_config5"]
LABEL = {"b_cornell": "Cornell 800² spp256 d16 (config 3, headline)", "bench_default": "headline, default run (CPU leg)",
         "b_cornell_fp32": "Cornell, fp32 mode", "b_adaptive": "Cornell, reference adaptive defaults",
         "b_spheres": "spheres-500 800² spp64 d8 (config 2)", "b_rain": "rain 1920×1080 spp512 d16 (config 4)",
         "b_100k": "spheres-100k 4096² spp16 d100", "b_config5": "spheres-100k 4096² spp1024 d100 (config 5)"}


def line(path: Path):
    js = [x for x in path.read_text().splitlines() if x.startswith("{")]
    return json.loads(js[-1]) if js else None


def main():
    d = Path(sys.argv[1])
    print("| config | Msamples/s | ms / frame | path kernel ms | VALU frac | lane util | HBM frac | parity (px differing rgb / radiance) | counters |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name in ORDER:
        f = d / f"{name}.log"
        if not f.exists():
            continue
        L = line(f)
        if not L:
            continue
        r, p = L.get("roofline") or {}, L.get("parity") or {}
        hbm = (r.get("hbm") or {}).get("frac")
        par = f"{p.get('pixels_differing_rgb')} / {p.get('pixels_differing_radiance')}" if p else "-"
        if p and L.get("dtype") == "f32":
            par += " (fp32: tolerance rule)"
        print(f"| {LABEL[name]} | {L['value']:,.0f} | {L['ms_per_step']:.2f} | {r.get('kernel_ms')} | {r.get('frac')} | "
              f"{r.get('lane_util')} | {hbm} | {par} | {str(r.get('pmc_build'))[:8]}{' STALE' if r.get('pmc_stale') else ''} |")
    cpu = None
    if (d / "bench_default.log").exists():
        cpu = (line(d / "bench_default.log") or {}).get("cpu_baseline")
    if cpu:
        print()
        print(f"CPU (oracle, {cpu.get('kind')}): 1 thread ref {cpu['value']:.2f} Msamples/s; "
              f"1 thread fp32 {cpu.get('fp32', {}).get('value', float('nan')):.2f}; "
              f"{cpu.get('multi_core', {}).get('cores')} threads ref {cpu.get('multi_core', {}).get('value', float('nan')):.1f} "
              f"({cpu.get('multi_core', {}).get('cpu')})")


if __name__ == "__main__":
    main()
