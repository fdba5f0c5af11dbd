#!/usr/bin/env python3
"""Static ISA statistics of the kernel units (CPU only: hipcc cross-compiles gfx950).

Compiles a kernel unit with the library's own flags plus --save-temps into a scratch
directory and, per kernel symbol matching a pattern, counts instructions by class
(f32 add/mul/fma, min3/max3, f64, SALU, branches, ...) and reports the register
header (VGPRs, SGPRs, spills). Static counts are not issue counts - loops execute
some blocks many times - but they show whether an arithmetic change reached the code
(e.g. v_fma_f32 / v_min3_f32 in the slab tests) before a GPU run measures it.

usage: python tools/isa_stats.py [--unit pt_ref.hip] [--out DIR] [-D NAME=V ...] PATTERN...
"""
from __future__ import annotations

import argparse
import collections
import re
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "mcp-raytracer_amd"))
from raytracer_amd import _build  # noqa: E402

CLASSES = [
    ("fma_f32", r"^v_(fma|fmac|fmaak|fmamk)_f32"),
    ("add_f32", r"^v_(add|sub|subrev)_f32"),
    ("mul_f32", r"^v_mul_f32"),
    ("minmax3_f32", r"^v_(min3|max3|med3)_f32"),
    ("minmax_f32", r"^v_(min|max)_f32"),
    ("pk_f32", r"^v_pk_"),
    ("f64", r"^v_\w+_f64"),
    ("cvt", r"^v_cvt_"),
    ("cmp", r"^v_cmpx?_"),
    ("cndmask", r"^v_cndmask"),
    ("valu_other", r"^v_"),
    ("salu", r"^s_(?!waitcnt|branch|cbranch|endpgm|nop|setprio|barrier|load|buffer|store|dcache|memtime|sleep)"),
    ("smem", r"^s_(load|buffer_load)"),
    ("branch", r"^s_(c?branch)"),
    ("lds", r"^ds_"),
    ("vmem", r"^(global|buffer|flat|scratch)_"),
    ("waitcnt", r"^s_waitcnt"),
]


def compile_unit(unit: str, out: Path, defines, extra=()) -> Path:
    out.mkdir(parents=True, exist_ok=True)
    flags = dict((u[0], u[1]) for u in _build._UNITS)[unit]
    cmd = [_build.hipcc(), *_build._COMMON, *flags, *[f"-D{d}" for d in defines], *extra, '-DRT_BUILD_ID="isa"',
           f"--offload-arch={_build.ARCH}", "--offload-device-only", "-save-temps", "-c",
           str(_build.CSRC / unit), "-o", str(out / "unit.o")]
    subprocess.run(cmd, check=True, cwd=out)
    cands = sorted(out.glob("*gfx950*.s"))
    if not cands:
        raise SystemExit(f"no device assembly in {out}")
    return cands[0]


def functions(asm: str):
    """Yield (symbol, body lines, metadata dict) for every kernel in the assembly."""
    cur, body = None, []
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and line.startswith(".Lfunc_end"):
            yield cur, body
            cur = None
            continue
        if cur:
            body.append(line)
    return


def meta(asm: str, sym: str) -> dict:
    out = {}
    m = re.search(re.escape(sym) + r"\n(.*?)\.end_amdhsa_kernel", asm, re.S)
    blk = asm[asm.find(".amdhsa_kernel " + sym):]
    for key in ("next_free_vgpr", "next_free_sgpr", "accum_offset", "private_segment_fixed_size"):
        mm = re.search(r"\.amdhsa_" + key + r"\s+(\d+)", blk)
        if mm:
            out[key] = int(mm.group(1))
    return out


def stats(body):
    c = collections.Counter()
    for line in body:
        s = line.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c["total"] += 1
        for name, pat in CLASSES:
            if re.match(pat, op):
                c[name] += 1
                break
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("patterns", nargs="+")
    ap.add_argument("--unit", default="pt_ref.hip")
    ap.add_argument("--out", default="/tmp/isa")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--flag", dest="flags", action="append", default=[], help="extra compiler flag (repeatable)")
    ap.add_argument("--reuse", action="store_true", help="parse the assembly already in --out")
    a = ap.parse_args()
    if a.reuse:
        s_path = sorted(Path(a.out).glob("*gfx950*.s"))[0]
    else:
        s_path = compile_unit(a.unit, Path(a.out), a.defines, a.flags)
    asm = s_path.read_text()
    demangled = {}
    syms = [sym for sym, _ in functions(asm)]
    if syms:
        dm = subprocess.run(["c++filt"], input="\n".join(syms), text=True,
                            capture_output=True).stdout.splitlines()
        demangled = dict(zip(syms, dm))
    for sym, body in functions(asm):
        name = demangled.get(sym, sym)
        if not any(re.search(p, name) for p in a.patterns):
            continue
        c = stats(body)
        c["scratch"] = sum(1 for line in body if line.strip().startswith("scratch_"))
        md = meta(asm, sym)
        print(name)
        print("  regs:", md)
        print("  " + " ".join(f"{k}={c[k]}" for k in ["total"] + [n for n, _ in CLASSES] + ["scratch"] if c[k]))


if __name__ == "__main__":
    main()
