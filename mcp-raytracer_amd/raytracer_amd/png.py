"""PNG encoding of the raw RGB framebuffer.

The reference hands its Uint8ClampedArray to sharp/libvips
(src/raytracer.ts:101-110). That step is outside the hot path; this is a
dependency-free encoder (8-bit RGB, filter 0, zlib) producing an equivalent
PNG of the same pixels.
"""
from __future__ import annotations

import struct
import zlib


def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def encode_png(rgb, width: int, height: int, channels: int = 3) -> bytes:
    if channels != 3:
        raise ValueError("only RGB is supported")
    raw = bytes(rgb)
    if len(raw) < width * height * 3:
        raise ValueError("pixel buffer too small")
    stride = width * 3
    rows = b"".join(b"\x00" + raw[y * stride:(y + 1) * stride] for y in range(height))
    ihdr = struct.pack(">IIBBBBB", width, height, 8, 2, 0, 0, 0)
    return b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", zlib.compress(rows, 6)) + _chunk(b"IEND", b"")


def decode_png_rgb(png: bytes):
    """Minimal decoder for the files encode_png writes (tests)."""
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(png):
        (n,) = struct.unpack(">I", png[pos:pos + 4])
        tag = png[pos + 4:pos + 8]
        data = png[pos + 8:pos + 8 + n]
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
