// PNG of the u8 framebuffer, encoded on the device (png_deflate.hpp), and the
// same encoder run on the host (rt_debug_png_host: the CPU tests' pin of the
// exact bytes). The container (signature, IHDR, IDAT, IEND) and the combination
// of the segments' Adler-32 / CRC-32 values are host steps over a few hundred
// words; the filtering, LZ77 runs, Huffman coding and checksums of the pixel
// data run on the GPU.
#include <hip/hip_runtime.h>
#include <zlib.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rt_amd.h"
#include "png_deflate.hpp"

using rtpng::SegResult;
using rtpng::SegWork;

int rt_set_error_message(int code, const char* msg);  // rt_api.cpp

namespace {

// One thread per row: the row's PNG filter type (libpng's min-sum heuristic).
__global__ __launch_bounds__(256) void png_filter_kernel(const uint8_t* __restrict__ rgb, int w3, int h,
                                                         uint8_t* __restrict__ ftype) {
    const int y = blockIdx.x * blockDim.x + threadIdx.x;
    if (y < h) ftype[y] = (uint8_t)rtpng::choose_filter(rgb, w3, y);
}

// One 64-lane workgroup per segment: the lanes fill the segment's filtered bytes
// (and the CRC table), lane 0 encodes, the lanes copy the compressed bytes out.
__global__ __launch_bounds__(64) void png_deflate_kernel(const uint8_t* __restrict__ rgb,
                                                          const uint8_t* __restrict__ ftype, int w3, int64_t total,
                                                          int n_seg, uint8_t* __restrict__ seg_out,
                                                          SegResult* __restrict__ res) {
    __shared__ SegWork W;
    __shared__ uint32_t crc_table[256];
    __shared__ SegResult r;
    const int k = blockIdx.x;
    if (k >= n_seg) return;
    const int64_t q0 = (int64_t)k * rtpng::kSeg;
    const int n = (int)((total - q0) < rtpng::kSeg ? (total - q0) : rtpng::kSeg);
    for (int t = threadIdx.x; t < 256; t += 64) crc_table[t] = rtpng::crc_table_entry((uint32_t)t);
    for (int i = threadIdx.x; i < n; i += 64) W.f[i] = rtpng::stream_byte(rgb, ftype, w3, q0 + i);
    if (threadIdx.x < 4) {
        const int64_t q = q0 - 4 + threadIdx.x;
        W.hist[threadIdx.x] = q >= 0 ? rtpng::stream_byte(rgb, ftype, w3, q) : 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) r = rtpng::deflate_segment(W, n, q0, k == n_seg - 1, crc_table);
    __syncthreads();
    uint8_t* dst = seg_out + (size_t)k * rtpng::kOutCap;
    for (uint32_t i = threadIdx.x; i < r.len; i += 64) dst[i] = W.out[i];
    if (threadIdx.x == 0) res[k] = r;
}

// One workgroup per segment: its compressed bytes to their place in the stream.
__global__ __launch_bounds__(256) void png_gather_kernel(const uint8_t* __restrict__ seg_out,
                                                         const uint64_t* __restrict__ off,
                                                         const SegResult* __restrict__ res, uint8_t* __restrict__ dst) {
    const int k = blockIdx.x;
    const uint8_t* src = seg_out + (size_t)k * rtpng::kOutCap;
    uint8_t* d = dst + off[k];
    const uint32_t n = res[k].len;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = src[i];
}

void put32(std::vector<uint8_t>& o, uint32_t v) {
    o.push_back((uint8_t)(v >> 24));
    o.push_back((uint8_t)(v >> 16));
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

void put_chunk(std::vector<uint8_t>& o, const char* tag, const uint8_t* data, size_t n) {
    put32(o, (uint32_t)n);
    const size_t at = o.size();
    o.insert(o.end(), tag, tag + 4);
    if (n) o.insert(o.end(), data, data + n);
    put32(o, (uint32_t)crc32(crc32(0L, Z_NULL, 0), o.data() + at, (uInt)(4 + n)));
}

// The PNG file around the concatenated segments: fill(dst) writes the zlen
// compressed bytes of the deflate stream at dst.
template <class Fill>
std::vector<uint8_t> assemble(int32_t w, int32_t h, const std::vector<SegResult>& res, Fill fill) {
    size_t zlen = 0;
    uLong adler = adler32(0L, Z_NULL, 0);
    for (const SegResult& r : res) {
        zlen += r.len;
        adler = adler32_combine(adler, r.adler, (z_off_t)r.raw);
    }
    std::vector<uint8_t> o;
    const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    o.insert(o.end(), sig, sig + 8);
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)w);
    put32(ihdr, (uint32_t)h);
    const uint8_t rest[5] = {8, 2, 0, 0, 0};  // 8-bit, truecolour, deflate, adaptive filtering, no interlace
    ihdr.insert(ihdr.end(), rest, rest + 5);
    put_chunk(o, "IHDR", ihdr.data(), ihdr.size());
    // IDAT: zlib header (deflate, 32K window, no dictionary), the segments, Adler-32
    const size_t idat_len = 2 + zlen + 4;
    if (idat_len > 0x7fffffffu) throw std::runtime_error("PNG IDAT chunk too large");
    put32(o, (uint32_t)idat_len);
    const uint8_t head[6] = {'I', 'D', 'A', 'T', 0x78, 0x01};
    o.insert(o.end(), head, head + 6);
    const size_t zat = o.size();
    o.resize(zat + zlen);
    fill(o.data() + zat);
    uLong crc = crc32(crc32(0L, Z_NULL, 0), head, 6);
    for (const SegResult& r : res) crc = crc32_combine(crc, r.crc, (z_off_t)r.len);
    put32(o, (uint32_t)adler);
    crc = crc32(crc, o.data() + o.size() - 4, 4);
    put32(o, (uint32_t)crc);
    put_chunk(o, "IEND", nullptr, 0);
    return o;
}

int hand_out(const std::vector<uint8_t>& v, uint8_t** out, size_t* out_len) {
    uint8_t* b = (uint8_t*)std::malloc(v.size() ? v.size() : 1);
    if (!b) return rt_set_error_message(RT_ERR_INVALID, "out of memory");
    std::memcpy(b, v.data(), v.size());
    *out = b;
    *out_len = v.size();
    return RT_OK;
}

void hipc(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    explicit DevBuf(size_t n) { hipc(hipMalloc(&p, n * sizeof(T) + 16), "hipMalloc"); }
    ~DevBuf() { if (p) (void)hipFree(p); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
};

}  // namespace

// Encodes the device frame d_rgb (width*height*3 u8) as PNG on the device queue
// `stream`; waits for it and returns the file bytes in host memory.
std::vector<uint8_t> rt_png_encode_device(const uint8_t* d_rgb, int32_t w, int32_t h, hipStream_t stream) {
    const int w3 = w * 3;
    const int64_t total = (int64_t)h * (w3 + 1);
    const int n_seg = (int)((total + rtpng::kSeg - 1) / rtpng::kSeg);
    DevBuf<uint8_t> ftype((size_t)h), seg_out((size_t)n_seg * rtpng::kOutCap);
    DevBuf<SegResult> res((size_t)n_seg);
    hipLaunchKernelGGL(png_filter_kernel, dim3((h + 255) / 256), dim3(256), 0, stream, d_rgb, w3, h, ftype.p);
    hipc(hipGetLastError(), "png_filter_kernel");
    hipLaunchKernelGGL(png_deflate_kernel, dim3(n_seg), dim3(64), 0, stream, d_rgb, ftype.p, w3, total, n_seg,
                       seg_out.p, res.p);
    hipc(hipGetLastError(), "png_deflate_kernel");
    std::vector<SegResult> hr((size_t)n_seg);
    hipc(hipMemcpyAsync(hr.data(), res.p, hr.size() * sizeof(SegResult), hipMemcpyDeviceToHost, stream),
         "hipMemcpyAsync");
    hipc(hipStreamSynchronize(stream), "hipStreamSynchronize");
    std::vector<uint64_t> off((size_t)n_seg);
    uint64_t zlen = 0;
    for (int k = 0; k < n_seg; ++k) {
        if (hr[k].len > (uint32_t)rtpng::kOutCap) throw std::runtime_error("PNG segment overflow");
        off[k] = zlen;
        zlen += hr[k].len;
    }
    DevBuf<uint64_t> d_off((size_t)n_seg);
    DevBuf<uint8_t> d_z((size_t)zlen);
    hipc(hipMemcpyAsync(d_off.p, off.data(), off.size() * sizeof(uint64_t), hipMemcpyHostToDevice, stream),
         "hipMemcpyAsync");
    hipLaunchKernelGGL(png_gather_kernel, dim3(n_seg), dim3(256), 0, stream, seg_out.p, d_off.p, res.p, d_z.p);
    hipc(hipGetLastError(), "png_gather_kernel");
    return assemble(w, h, hr, [&](uint8_t* dst) {
        hipc(hipMemcpyAsync(dst, d_z.p, zlen, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync");
        hipc(hipStreamSynchronize(stream), "hipStreamSynchronize");
    });
}

extern "C" int rt_encode_png_device(const uint8_t* d_rgb, int32_t width, int32_t height, void* stream, uint8_t** out,
                                    size_t* out_len) {
    if (!d_rgb || !out || !out_len || width <= 0 || height <= 0 || width > (1 << 24) / 3)
        return rt_set_error_message(RT_ERR_INVALID, "rt_encode_png_device: bad arguments");
    try {
        return hand_out(rt_png_encode_device(d_rgb, width, height, (hipStream_t)stream), out, out_len);
    } catch (const std::exception& e) {
        return rt_set_error_message(RT_ERR_DEVICE, e.what());
    }
}

extern "C" int rt_debug_png_host(const uint8_t* rgb, int32_t width, int32_t height, uint8_t** out, size_t* out_len) {
    if (!rgb || !out || !out_len || width <= 0 || height <= 0 || width > (1 << 24) / 3)
        return rt_set_error_message(RT_ERR_INVALID, "rt_debug_png_host: bad arguments");
    try {
        const int w3 = width * 3;
        const int64_t total = (int64_t)height * (w3 + 1);
        const int n_seg = (int)((total + rtpng::kSeg - 1) / rtpng::kSeg);
        std::vector<uint8_t> ftype((size_t)height);
        for (int y = 0; y < height; ++y) ftype[y] = (uint8_t)rtpng::choose_filter(rgb, w3, y);
        uint32_t table[256];
        for (uint32_t t = 0; t < 256; ++t) table[t] = rtpng::crc_table_entry(t);
        std::vector<SegResult> res((size_t)n_seg);
        std::vector<uint8_t> z;
        std::unique_ptr<SegWork> W(new SegWork);
        for (int k = 0; k < n_seg; ++k) {
            const int64_t q0 = (int64_t)k * rtpng::kSeg;
            const int n = (int)std::min<int64_t>(total - q0, rtpng::kSeg);
            for (int i = 0; i < n; ++i) W->f[i] = rtpng::stream_byte(rgb, ftype.data(), w3, q0 + i);
            for (int t = 0; t < 4; ++t) {
                const int64_t q = q0 - 4 + t;
                W->hist[t] = q >= 0 ? rtpng::stream_byte(rgb, ftype.data(), w3, q) : 0;
            }
            res[k] = rtpng::deflate_segment(*W, n, q0, k == n_seg - 1, table);
            z.insert(z.end(), W->out, W->out + res[k].len);
        }
        return hand_out(assemble(width, height, res, [&](uint8_t* dst) { std::memcpy(dst, z.data(), z.size()); }),
                        out, out_len);
    } catch (const std::exception& e) {
        return rt_set_error_message(RT_ERR_INVALID, e.what());
    }
}
