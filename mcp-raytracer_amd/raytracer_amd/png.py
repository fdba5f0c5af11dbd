"""Image files from the raw RGB framebuffer.

The reference hands its Uint8ClampedArray to sharp/libvips
(src/raytracer.ts:101-110). Encoding runs in librt_amd.so (rt_encode_png:
8-bit RGB, filter 0 rows, zlib; rt_encode_ppm: binary P6) right next to the
u8 frame the device wrote; decode_png_rgb is a minimal reader for tests.
"""
from __future__ import annotations

import ctypes as C
import struct
import zlib

from . import _lib


def _call(fn, *args) -> bytes:
    out, n = C.c_void_p(), C.c_size_t()
    _lib.check(fn(*args, C.byref(out), C.byref(n)))
    try:
        return C.string_at(out, n.value)
    finally:
        _lib.load().rt_free(out)


def _buf(rgb, width: int, height: int, channels: int):
    if channels != 3:
        raise ValueError("only RGB is supported")
    raw = bytes(rgb)
    if len(raw) < width * height * 3:
        raise ValueError("pixel buffer too small")
    return raw


def encode_png(rgb, width: int, height: int, channels: int = 3, level: int = 6) -> bytes:
    raw = _buf(rgb, width, height, channels)
    return _call(_lib.load().rt_encode_png, raw, width, height, level)


def encode_ppm(rgb, width: int, height: int, channels: int = 3) -> bytes:
    raw = _buf(rgb, width, height, channels)
    return _call(_lib.load().rt_encode_ppm, raw, width, height)


def decode_png_rgb(png: bytes):
    """Minimal decoder for the files encode_png writes (tests)."""
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(png):
        (n,) = struct.unpack(">I", png[pos:pos + 4])
        tag = png[pos + 4:pos + 8]
        data = png[pos + 8:pos + 8 + n]
        (crc,) = struct.unpack(">I", png[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(tag + data) & 0xFFFFFFFF, tag
        if tag == b"IHDR":
            w, h = struct.unpack(">II", data[:8])
        elif tag == b"IDAT":
            idat += data
        pos += 12 + n
    raw = zlib.decompress(idat)
    stride = w * 3
    out = bytearray()
    for y in range(h):
        row = raw[y * (stride + 1):(y + 1) * (stride + 1)]
        assert row[0] == 0
        out += row[1:]
    return w, h, bytes(out)
