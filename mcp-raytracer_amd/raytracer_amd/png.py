"""Image files from the raw RGB framebuffer.

The reference hands its Uint8ClampedArray to sharp/libvips
(src/raytracer.ts:101-110). generate_image_buffer encodes the device frame on
the GPU (rt_encode_png_device / rt_camera_render_png: per-row PNG filters,
per-segment dynamic-Huffman deflate blocks, checksums); rt_encode_png (host
zlib, filter 0) and rt_encode_ppm (binary P6) encode host buffers;
decode_png_rgb is a minimal reader for tests.
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


def encode_png_device(rgb_ptr: int, width: int, height: int, stream=None) -> bytes:
    """PNG of a DEVICE u8 RGB frame (a device pointer), encoded on the GPU
    (rt_encode_png_device); queued on `stream` (hipStream_t as int, None = default)."""
    lib = _lib.load()
    return _call(lib.rt_encode_png_device, C.c_void_p(rgb_ptr), width, height, C.c_void_p(stream or 0))


def debug_png_host(rgb, width: int, height: int, channels: int = 3) -> bytes:
    """The device encoder's algorithm run on the host (rt_debug_png_host): the same
    bytes rt_encode_png_device writes for this frame (tests)."""
    raw = _buf(rgb, width, height, channels)
    return _call(_lib.load().rt_debug_png_host, raw, width, height)


def encode_ppm(rgb, width: int, height: int, channels: int = 3) -> bytes:
    raw = _buf(rgb, width, height, channels)
    return _call(_lib.load().rt_encode_ppm, raw, width, height)


def decode_png_rgb(png: bytes):
    """Minimal decoder for the 8-bit RGB files the encoders write (all five filter types; tests)."""
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
    if len(raw) != h * (stride + 1):
        raise ValueError("PNG data length does not match the header")
    out = bytearray(h * stride)
    prev = bytes(stride)
    for y in range(h):
        row = raw[y * (stride + 1):(y + 1) * (stride + 1)]
        ft, cur = row[0], bytearray(row[1:])
        if ft == 1:
            for x in range(3, stride):
                cur[x] = (cur[x] + cur[x - 3]) & 255
        elif ft == 2:
            for x in range(stride):
                cur[x] = (cur[x] + prev[x]) & 255
        elif ft == 3:
            for x in range(stride):
                a = cur[x - 3] if x >= 3 else 0
                cur[x] = (cur[x] + ((a + prev[x]) >> 1)) & 255
        elif ft == 4:
            for x in range(stride):
                a = cur[x - 3] if x >= 3 else 0
                b = prev[x]
                c = prev[x - 3] if x >= 3 else 0
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                cur[x] = (cur[x] + (a if pa <= pb and pa <= pc else b if pb <= pc else c)) & 255
        elif ft != 0:
            raise ValueError(f"bad PNG filter type {ft}")
        out[y * stride:(y + 1) * stride] = cur
        prev = bytes(cur)
    return w, h, bytes(out)
