// Image-file encoders for the framebuffer. The reference hands its
// Uint8ClampedArray to sharp/libvips for PNG (src/raytracer.ts:101-110); this is
// the same step without the libvips dependency: 8-bit RGB PNG (filter 0 rows,
// zlib stream, CRC-32 chunks) and binary PPM (P6), straight from the u8 frame
// the device wrote (writeColorToBuffer, src/camera.ts:455-472).
#include <zlib.h>

#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_amd.h"

namespace {

void put32(std::vector<uint8_t>& o, uint32_t v) {
    o.push_back((uint8_t)(v >> 24));
    o.push_back((uint8_t)(v >> 16));
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

void chunk(std::vector<uint8_t>& o, const char* tag, const uint8_t* data, size_t n) {
    put32(o, (uint32_t)n);
    const size_t at = o.size();
    o.insert(o.end(), tag, tag + 4);
    if (n) o.insert(o.end(), data, data + n);
    const uLong crc = crc32(crc32(0L, Z_NULL, 0), o.data() + at, (uInt)(4 + n));
    put32(o, (uint32_t)crc);
}

int hand_out(const std::vector<uint8_t>& v, uint8_t** out, size_t* out_len) {
    uint8_t* b = (uint8_t*)std::malloc(v.size() ? v.size() : 1);
    if (!b) return RT_ERR_INVALID;
    std::memcpy(b, v.data(), v.size());
    *out = b;
    *out_len = v.size();
    return RT_OK;
}

}  // namespace

int rt_set_error_message(int code, const char* msg);  // rt_api.cpp

extern "C" int rt_encode_png(const uint8_t* rgb, int32_t width, int32_t height, int32_t level, uint8_t** out,
                             size_t* out_len) {
    if (!rgb || !out || !out_len || width <= 0 || height <= 0 || level < 0 || level > 9)
        return rt_set_error_message(RT_ERR_INVALID, "rt_encode_png: bad arguments");
    const size_t stride = (size_t)width * 3;
    std::vector<uint8_t> raw((stride + 1) * (size_t)height);
    for (int32_t y = 0; y < height; ++y) {
        uint8_t* row = raw.data() + (stride + 1) * (size_t)y;
        row[0] = 0;  // filter type None
        std::memcpy(row + 1, rgb + stride * (size_t)y, stride);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), level) != Z_OK)
        return rt_set_error_message(RT_ERR_INVALID, "rt_encode_png: zlib failure");
    std::vector<uint8_t> o;
    o.reserve(zlen + 64);
    const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    o.insert(o.end(), sig, sig + 8);
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)width);
    put32(ihdr, (uint32_t)height);
    const uint8_t rest[5] = {8, 2, 0, 0, 0};  // 8-bit, truecolour, deflate, filter 0, no interlace
    ihdr.insert(ihdr.end(), rest, rest + 5);
    chunk(o, "IHDR", ihdr.data(), ihdr.size());
    chunk(o, "IDAT", z.data(), zlen);
    chunk(o, "IEND", nullptr, 0);
    if (hand_out(o, out, out_len) != RT_OK) return rt_set_error_message(RT_ERR_INVALID, "out of memory");
    return RT_OK;
}

extern "C" int rt_encode_ppm(const uint8_t* rgb, int32_t width, int32_t height, uint8_t** out, size_t* out_len) {
    if (!rgb || !out || !out_len || width <= 0 || height <= 0)
        return rt_set_error_message(RT_ERR_INVALID, "rt_encode_ppm: bad arguments");
    const std::string head = "P6\n" + std::to_string(width) + " " + std::to_string(height) + "\n255\n";
    std::vector<uint8_t> o(head.begin(), head.end());
    o.insert(o.end(), rgb, rgb + (size_t)width * height * 3);
    if (hand_out(o, out, out_len) != RT_OK) return rt_set_error_message(RT_ERR_INVALID, "out of memory");
    return RT_OK;
}
