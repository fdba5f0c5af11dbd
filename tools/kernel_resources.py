#!/usr/bin/env python3
"""Register and scratch footprint of every kernel in the built library (CPU only).

Reads the gfx950 code objects out of librt_amd.so's .hip_fatbin section (one clang offload
bundle per HIP unit), and from each code object's AMDGPU metadata note (msgpack) the kernels'
VGPR / SGPR counts and private-segment (scratch) bytes per lane. A product path kernel that
spills to scratch pays an L2-missing reload inside its loop ("Round 5, kept: no
machine-code loop-invariant motion"), so tests/test_abi.py holds the product kernels at zero.

usage: python tools/kernel_resources.py [path/to/librt_amd.so] [name-regex]
"""
from __future__ import annotations

import re
import struct
import sys
from pathlib import Path

import msgpack

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
NT_AMDGPU_METADATA = 32


def _sections(elf: bytes) -> dict:
    """name -> (offset, size) of an ELF64 little-endian file's sections."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise ValueError("not an ELF64 little-endian object")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    str_off, str_size = hdrs[shstrndx][4], hdrs[shstrndx][5]
    names = elf[str_off:str_off + str_size]
    out = {}
    for h in hdrs:
        name = names[h[0]:names.index(b"\0", h[0])].decode()
        out[name] = (h[4], h[5])
    return out


CCOB_MAGIC = b"CCOB"  # clang's compressed offload bundle (not parsed here)


def code_objects(lib: Path, target: str = "gfx950"):
    """Yield the device code objects for `target` in the library's offload bundles."""
    data = lib.read_bytes()
    off, size = _sections(data)[".hip_fatbin"]
    fat = data[off:off + size]
    if BUNDLE_MAGIC not in fat:
        kind = "compressed (CCOB) bundles" if CCOB_MAGIC in fat else "no offload bundle"
        raise RuntimeError(f"{lib.name}: .hip_fatbin holds {kind}; this reader parses uncompressed "
                           f"{BUNDLE_MAGIC.decode()} bundles only (build without --offload-compress)")
    for m in re.finditer(re.escape(BUNDLE_MAGIC), fat):
        base = m.start()
        n, = struct.unpack_from("<Q", fat, base + len(BUNDLE_MAGIC))
        p = base + len(BUNDLE_MAGIC) + 8
        for _ in range(n):
            e_off, e_size, t_len = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + t_len].decode()
            p += 24 + t_len
            if triple.endswith(target) and e_size:
                yield fat[base + e_off:base + e_off + e_size]


def kernels(code: bytes):
    """Yield the metadata map of every kernel in one code object."""
    off, size = _sections(code)[".note"]
    p, end = off, off + size
    while p < end:
        namesz, descsz, ntype = struct.unpack_from("<III", code, p)
        name_end = p + 12 + ((namesz + 3) & ~3)
        desc = code[name_end:name_end + descsz]
        if ntype == NT_AMDGPU_METADATA and code[p + 12:p + 12 + namesz].rstrip(b"\0") == b"AMDGPU":
            meta = msgpack.unpackb(desc, raw=False, strict_map_key=False)
            yield from meta.get("amdhsa.kernels", [])
        p = name_end + ((descsz + 3) & ~3)


def resources(lib: Path, pattern: str = "") -> list[dict]:
    rx = re.compile(pattern) if pattern else None
    out = []
    for code in code_objects(lib):
        for k in kernels(code):
            name = k.get(".name", "")
            if rx and not rx.search(name):
                continue
            out.append({"name": name, "vgpr": k.get(".vgpr_count"), "agpr": k.get(".agpr_count"),
                        "sgpr": k.get(".sgpr_count"), "scratch": k.get(".private_segment_fixed_size"),
                        "lds": k.get(".group_segment_fixed_size"),
                        "vgpr_spill": k.get(".vgpr_spill_count"), "sgpr_spill": k.get(".sgpr_spill_count")})
    return out


def main():
    root = Path(__file__).resolve().parents[1]
    lib = Path(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1] else root / "mcp-raytracer_amd/raytracer_amd/lib/librt_amd.so"
    pattern = sys.argv[2] if len(sys.argv) > 2 else ""
    for r in resources(lib, pattern):
        print(f"{r['name'][:90]:90s} vgpr {r['vgpr']:>4} sgpr {r['sgpr']:>4} scratch {r['scratch']:>5} "
              f"spills v{r['vgpr_spill']} s{r['sgpr_spill']}")


if __name__ == "__main__":
    main()
