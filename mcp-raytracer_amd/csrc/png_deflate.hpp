// PNG encoding of the u8 framebuffer on the device.
//
// The reference hands its finished Uint8ClampedArray to sharp/libvips for the
// PNG (src/raytracer.ts:101-110). Here the frame never leaves HBM before it is
// a PNG: the filtered scanline stream (PNG filter type + filtered bytes per
// row, RFC 2083 §6) is cut into independent kSeg-byte segments; each segment
// is one deflate block (RFC 1951) with its own dynamic Huffman code, ended by
// an empty stored block (a "sync flush") so that the segments' compressed
// bytes simply concatenate into one zlib stream. Every segment also reports
// the Adler-32 of its raw bytes and the CRC-32 of its compressed bytes, which
// the host combines (zlib adler32_combine / crc32_combine) into the zlib
// trailer and the IDAT CRC.
//
// Everything below is __host__ __device__ and sequential per segment: the
// device runs one segment per 64-lane workgroup (lane 0 encodes, the others
// fill the filtered bytes), rt_debug_png_host runs the same functions on the
// CPU so the CPU tests pin the exact bytes the GPU writes.
//
// LZ77: runs only (distance 1 = the previous byte, distance 3 = the previous
// pixel's channel), greedy. After PNG filtering, flat regions (sky, walls lit
// evenly) are runs of zero residuals; elsewhere the residuals are small
// numbers whose entropy the per-segment Huffman code captures.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define PNG_HD __host__ __device__
#else
#define PNG_HD
#endif

namespace rtpng {

constexpr int kSeg = 4096;              // filtered-stream bytes per segment
constexpr int kOutCap = kSeg + 64;      // compressed bytes per segment (stored fallback: kSeg + 5)
constexpr int kLL = 286, kDist = 30, kCL = 19;
constexpr int kMaxLL = 15, kMaxCL = 7;

// Scratch of one segment (LDS on the device: 27 KB).
struct SegWork {
    uint8_t hist[4];            // the 4 stream bytes before the segment (hist[3] = the previous byte)
    uint8_t f[kSeg];            // the segment's filtered bytes
    uint32_t tok[kSeg];         // literal (< 256) or match: bit 31 | dist3 << 16 | length
    uint32_t freq[kLL + kDist + kCL];
    uint8_t len[kLL + kDist + kCL];
    uint16_t code[kLL + kDist + kCL];
    uint16_t srt[kLL], tmp[kLL];  // symbols sorted by frequency
    uint32_t a[kLL];              // Huffman lengths in sorted order
    uint16_t cl_sym[kLL + kDist];  // code-length alphabet stream (symbol | extra << 8)
    uint32_t cnt[129], bl[33], nc[16], c2[16];  // sort buckets, codes per length
    uint8_t out[kOutCap];
};

struct SegResult {
    uint32_t len;    // compressed bytes
    uint32_t crc;    // CRC-32 of those bytes (zlib convention)
    uint32_t adler;  // Adler-32 of the segment's raw filtered bytes
    uint32_t raw;    // raw filtered bytes of the segment
};

PNG_HD inline int paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = p > a ? p - a : a - p;
    const int pb = p > b ? p - b : b - p;
    const int pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

// Filtered byte x (0 <= x < 3W) of row y under filter type ft (RFC 2083 §6.2-6.6).
PNG_HD inline uint8_t filter_byte(const uint8_t* rgb, int w3, int y, int x, int ft) {
    const uint8_t* p = rgb + (int64_t)y * w3;
    const int raw = p[x];
    const int a = x >= 3 ? p[x - 3] : 0;
    const int b = y > 0 ? p[x - w3] : 0;
    const int c = (y > 0 && x >= 3) ? p[x - w3 - 3] : 0;
    int v = raw;
    switch (ft) {
        case 1: v = raw - a; break;
        case 2: v = raw - b; break;
        case 3: v = raw - ((a + b) >> 1); break;
        case 4: v = raw - paeth(a, b, c); break;
        default: break;
    }
    return (uint8_t)v;
}

// libpng's heuristic: the filter with the least sum of |residual| (residuals as
// signed bytes); ties go to the lower type.
PNG_HD inline int choose_filter(const uint8_t* rgb, int w3, int y) {
    uint32_t best = 0xffffffffu;
    int bt = 0;
    for (int ft = 0; ft < 5; ++ft) {
        uint32_t s = 0;
        for (int x = 0; x < w3; ++x) {
            const int v = (int8_t)filter_byte(rgb, w3, y, x, ft);
            s += (uint32_t)(v < 0 ? -v : v);
        }
        if (s < best) {
            best = s;
            bt = ft;
        }
    }
    return bt;
}

// Byte q of the filtered stream (row = filter type byte + 3W filtered bytes).
PNG_HD inline uint8_t stream_byte(const uint8_t* rgb, const uint8_t* ftype, int w3, int64_t q) {
    const int64_t rl = (int64_t)w3 + 1;
    const int y = (int)(q / rl);
    const int c = (int)(q - (int64_t)y * rl);
    return c == 0 ? ftype[y] : filter_byte(rgb, w3, y, c - 1, ftype[y]);
}

PNG_HD inline uint32_t bit_reverse(uint32_t v, int n) {
    uint32_t r = 0;
    for (int i = 0; i < n; ++i) {
        r = (r << 1) | (v & 1u);
        v >>= 1;
    }
    return r;
}

// Match length 3..258 -> length code index k (symbol 257 + k), extra bits e, extra value.
PNG_HD inline void length_code(int L, int& k, int& e, int& ev) {
    const int v = L - 3;
    if (v < 8) {
        k = v; e = 0; ev = 0;
    } else if (v == 255) {
        k = 28; e = 0; ev = 0;
    } else {
        int lg = 31 - __builtin_clz((unsigned)v);  // 3..7
        e = lg - 2;
        k = 4 * e + 4 + ((v >> e) - 4);
        ev = v & ((1 << e) - 1);
    }
}

// Code lengths (<= max_len) for `n` symbols with frequencies freq[0..n) (zero =
// unused) into len[0..n); canonical codes (bit-reversed for the LSB-first
// stream) into code[0..n). Minimum-redundancy lengths by Moffat and
// Katajainen's in-place algorithm over the frequency-sorted symbols, then
// limited to max_len by moving leaves down (Kraft sum kept at exactly 1).
PNG_HD inline void huffman(SegWork& W, const uint32_t* freq, int n, int max_len, uint8_t* len, uint16_t* code) {
    int m = 0;
    for (int s = 0; s < n; ++s) {
        len[s] = 0;
        if (freq[s]) W.tmp[m++] = (uint16_t)s;
    }
    // stable LSD radix sort of the used symbols by frequency (< 2^14: 2 x 7 bits)
    for (int pass = 0; pass < 2; ++pass) {
        uint32_t* cnt = W.cnt;
        for (int b = 0; b <= 128; ++b) cnt[b] = 0;
        for (int i = 0; i < m; ++i) ++cnt[((freq[W.tmp[i]] >> (7 * pass)) & 127) + 1];
        for (int b = 0; b < 128; ++b) cnt[b + 1] += cnt[b];
        for (int i = 0; i < m; ++i) W.srt[cnt[(freq[W.tmp[i]] >> (7 * pass)) & 127]++] = W.tmp[i];
        for (int i = 0; i < m; ++i) W.tmp[i] = W.srt[i];
    }
    uint32_t* A = W.a;
    for (int i = 0; i < m; ++i) A[i] = freq[W.srt[i]];
    if (m == 1) {
        A[0] = 1;
    } else if (m > 1) {
        A[0] += A[1];
        int root = 0, leaf = 2, next;
        for (next = 1; next < m - 1; ++next) {
            if (leaf >= m || A[root] < A[leaf]) { A[next] = A[root]; A[root++] = (uint32_t)next; }
            else A[next] = A[leaf++];
            if (leaf >= m || (root < next && A[root] < A[leaf])) { A[next] += A[root]; A[root++] = (uint32_t)next; }
            else A[next] += A[leaf++];
        }
        A[m - 2] = 0;
        for (next = m - 3; next >= 0; --next) A[next] = A[A[next]] + 1;
        int avbl = 1, used = 0, dpth = 0;
        root = m - 2;
        next = m - 1;
        while (avbl > 0) {
            while (root >= 0 && (int)A[root] == dpth) { ++used; --root; }
            while (avbl > used) { A[next--] = (uint32_t)dpth; --avbl; }
            avbl = 2 * used;
            ++dpth;
            used = 0;
        }
    }
    // count per length, limit to max_len
    uint32_t* bl = W.bl;
    for (int l = 0; l <= 32; ++l) bl[l] = 0;
    for (int i = 0; i < m; ++i) ++bl[A[i] > 32 ? 32 : A[i]];
    if (m > 1) {
        for (int l = max_len + 1; l <= 32; ++l) {
            bl[max_len] += bl[l];
            bl[l] = 0;
        }
        uint32_t total = 0;
        for (int l = max_len; l > 0; --l) total += bl[l] << (max_len - l);
        while (total != (1u << max_len)) {
            --bl[max_len];
            for (int l = max_len - 1; l > 0; --l) {
                if (bl[l]) {
                    --bl[l];
                    bl[l + 1] += 2;
                    break;
                }
            }
            --total;
        }
    }
    // longest codes to the least frequent symbols
    int j = 0;
    for (int l = max_len; l >= 1; --l)
        for (uint32_t c = bl[l]; c > 0; --c) len[W.srt[j++]] = (uint8_t)l;
    // canonical codes (RFC 1951 §3.2.2)
    uint32_t* next_code = W.nc;
    uint32_t* cnt2 = W.c2;
    for (int l = 0; l < 16; ++l) cnt2[l] = 0;
    for (int s = 0; s < n; ++s) ++cnt2[len[s]];
    cnt2[0] = 0;
    uint32_t c = 0;
    for (int l = 1; l < 16; ++l) {
        c = (c + cnt2[l - 1]) << 1;
        next_code[l] = c;
    }
    for (int s = 0; s < n; ++s)
        code[s] = len[s] ? (uint16_t)bit_reverse(next_code[len[s]]++, len[s]) : 0;
}

// The code-length codes' transmission order 16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11,
// 4, 12, 3, 13, 2, 14, 1, 15 (RFC 1951 §3.2.7).
PNG_HD inline int cl_order(int i) {
    if (i < 3) return 16 + i;
    const int j = i - 3;
    if (j == 0) return 0;
    return (j & 1) ? 8 + (j - 1) / 2 : 8 - j / 2;
}

struct BitOut {
    uint8_t* p;
    uint32_t pos = 0;  // bytes written
    uint64_t acc = 0;
    int nb = 0;
    PNG_HD void put(uint32_t bits, int n) {
        acc |= (uint64_t)bits << nb;
        nb += n;
        while (nb >= 8) {
            p[pos++] = (uint8_t)acc;
            acc >>= 8;
            nb -= 8;
        }
    }
    PNG_HD void align() {
        if (nb > 0) put(0, 8 - nb);
    }
    PNG_HD void byte(uint8_t b) { p[pos++] = b; }
};

PNG_HD inline uint32_t crc32_bytes(const uint32_t* table, const uint8_t* p, uint32_t n) {
    uint32_t c = 0xffffffffu;
    for (uint32_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return c ^ 0xffffffffu;
}

PNG_HD inline uint32_t crc_table_entry(uint32_t n) {
    uint32_t c = n;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? 0xedb88320u ^ (c >> 1) : c >> 1;
    return c;
}

PNG_HD inline uint32_t adler32_bytes(const uint8_t* p, uint32_t n) {
    uint32_t a = 1, b = 0;
    for (uint32_t i = 0; i < n; ++i) {
        a += p[i];
        if (a >= 65521u) a -= 65521u;
        b += a;
        if (b >= 65521u) b -= 65521u;
    }
    return (b << 16) | a;
}

// Encodes W.f[0..n) (stream position q0; W.hist holds the 4 bytes before it,
// valid for the q0 of them that exist) into W.out. `final`: the last segment.
PNG_HD inline SegResult deflate_segment(SegWork& W, int n, int64_t q0, bool final, const uint32_t* crc_table) {
    // 1. greedy run tokens
    int nt = 0;
    for (int i = 0; i < kLL + kDist + kCL; ++i) W.freq[i] = 0;
    uint32_t* fll = W.freq;
    uint32_t* fd = W.freq + kLL;
    auto at = [&](int i) -> int { return i >= 0 ? W.f[i] : W.hist[4 + i]; };
    for (int q = 0; q < n;) {
        int L1 = 0, L3 = 0;
        if (q0 + q >= 1)
            while (q + L1 < n && L1 < 258 && at(q + L1) == at(q + L1 - 1)) ++L1;
        if (q0 + q >= 3 && L1 < 258)
            while (q + L3 < n && L3 < 258 && at(q + L3) == at(q + L3 - 3)) ++L3;
        const int L = L1 >= L3 ? L1 : L3;
        if (L >= 3) {
            const bool d3 = L3 > L1;
            W.tok[nt++] = 0x80000000u | (d3 ? 0x10000u : 0u) | (uint32_t)L;
            int k, e, ev;
            length_code(L, k, e, ev);
            ++fll[257 + k];
            ++fd[d3 ? 2 : 0];
            q += L;
        } else {
            W.tok[nt++] = W.f[q];
            ++fll[W.f[q]];
            ++q;
        }
    }
    ++fll[256];  // end of block
    // complete codes: at least two distance codes (1 bit each when otherwise unused)
    if (!fd[0]) fd[0] = 1;
    if (!fd[1]) fd[1] = 1;
    if (fll[0] == 0) {  // at least two literal/length codes
        int used = 0;
        for (int s = 0; s < kLL; ++s) used += fll[s] ? 1 : 0;
        if (used < 2) fll[0] = 1;
    }
    uint8_t* lll = W.len;
    uint8_t* ld = W.len + kLL;
    uint8_t* lcl = W.len + kLL + kDist;
    uint16_t* cll = W.code;
    uint16_t* cd = W.code + kLL;
    uint16_t* ccl = W.code + kLL + kDist;
    huffman(W, fll, kLL, kMaxLL, lll, cll);
    huffman(W, fd, kDist, kMaxLL, ld, cd);
    int hlit = kLL;
    while (hlit > 257 && lll[hlit - 1] == 0) --hlit;
    int hdist = kDist;
    while (hdist > 1 && ld[hdist - 1] == 0) --hdist;
    // 2. the code lengths in the code-length alphabet (RFC 1951 §3.2.7)
    uint32_t* fcl = W.freq + kLL + kDist;
    int ncl = 0;
    {
        const int tot = hlit + hdist;
        auto lv = [&](int i) -> int { return i < hlit ? lll[i] : ld[i - hlit]; };
        for (int i = 0; i < tot;) {
            const int v = lv(i);
            int run = 1;
            while (i + run < tot && lv(i + run) == v) ++run;
            i += run;
            if (v == 0) {
                while (run >= 11) {
                    const int r = run < 138 ? run : 138;
                    W.cl_sym[ncl++] = (uint16_t)(18 | ((r - 11) << 8));
                    ++fcl[18];
                    run -= r;
                }
                if (run >= 3) {
                    W.cl_sym[ncl++] = (uint16_t)(17 | ((run - 3) << 8));
                    ++fcl[17];
                    run = 0;
                }
            } else {
                W.cl_sym[ncl++] = (uint16_t)v;
                ++fcl[v];
                --run;
                while (run >= 3) {
                    const int r = run < 6 ? run : 6;
                    W.cl_sym[ncl++] = (uint16_t)(16 | ((r - 3) << 8));
                    ++fcl[16];
                    run -= r;
                }
            }
            while (run > 0) {
                W.cl_sym[ncl++] = (uint16_t)v;
                ++fcl[v];
                --run;
            }
        }
        int used = 0;
        for (int s = 0; s < kCL; ++s) used += fcl[s] ? 1 : 0;
        if (used < 2) {
            if (!fcl[0]) fcl[0] = 1;
            else fcl[18] = 1;
        }
    }
    huffman(W, fcl, kCL, kMaxCL, lcl, ccl);
    int hclen = kCL;
    while (hclen > 4 && lcl[cl_order(hclen - 1)] == 0) --hclen;
    // 3. size of the dynamic block vs a stored one
    uint64_t bits = 3 + 5 + 5 + 4 + 3 * (uint64_t)hclen;
    for (int i = 0; i < ncl; ++i) {
        const int s = W.cl_sym[i] & 0xff;
        bits += lcl[s] + (s == 16 ? 2 : s == 17 ? 3 : s == 18 ? 7 : 0);
    }
    for (int s = 0; s < kLL; ++s) {
        if (!fll[s] || !lll[s]) continue;
        int e = 0;
        if (s > 256) {
            const int k = s - 257;
            e = (k >= 8 && k < 28) ? (k - 4) / 4 : 0;
        }
        bits += (uint64_t)fll[s] * (lll[s] + e);
    }
    for (int t = 0; t < nt; ++t)
        if (W.tok[t] & 0x80000000u) bits += ld[(W.tok[t] & 0x10000u) ? 2 : 0];
    const uint64_t dyn_bytes = (bits + 7) / 8 + (final ? 0 : 5);  // + the sync flush
    const uint64_t stored_bytes = (uint64_t)n + 5;
    BitOut o;
    o.p = W.out;
    if (stored_bytes <= dyn_bytes) {
        o.put(final ? 1 : 0, 1);
        o.put(0, 2);
        o.align();
        o.byte((uint8_t)n);
        o.byte((uint8_t)(n >> 8));
        o.byte((uint8_t)~n);
        o.byte((uint8_t)(~n >> 8));
        for (int i = 0; i < n; ++i) o.byte(W.f[i]);
    } else {
        o.put(final ? 1 : 0, 1);
        o.put(2, 2);
        o.put((uint32_t)(hlit - 257), 5);
        o.put((uint32_t)(hdist - 1), 5);
        o.put((uint32_t)(hclen - 4), 4);
        for (int i = 0; i < hclen; ++i) o.put(lcl[cl_order(i)], 3);
        for (int i = 0; i < ncl; ++i) {
            const int s = W.cl_sym[i] & 0xff, ev = W.cl_sym[i] >> 8;
            o.put(ccl[s], lcl[s]);
            if (s == 16) o.put((uint32_t)ev, 2);
            else if (s == 17) o.put((uint32_t)ev, 3);
            else if (s == 18) o.put((uint32_t)ev, 7);
        }
        for (int t = 0; t < nt; ++t) {
            const uint32_t tk = W.tok[t];
            if (!(tk & 0x80000000u)) {
                o.put(cll[tk], lll[tk]);
            } else {
                int k, e, ev;
                length_code((int)(tk & 0xffffu), k, e, ev);
                o.put(cll[257 + k], lll[257 + k]);
                if (e) o.put((uint32_t)ev, e);
                const int ds = (tk & 0x10000u) ? 2 : 0;
                o.put(cd[ds], ld[ds]);
            }
        }
        o.put(cll[256], lll[256]);
        if (final) {
            o.align();
        } else {  // sync flush: an empty stored block ends the segment on a byte boundary
            o.put(0, 3);
            o.align();
            o.byte(0);
            o.byte(0);
            o.byte(0xff);
            o.byte(0xff);
        }
    }
    SegResult r;
    r.len = o.pos;
    r.crc = crc32_bytes(crc_table, W.out, o.pos);
    r.adler = adler32_bytes(W.f, (uint32_t)n);
    r.raw = (uint32_t)n;
    return r;
}

}  // namespace rtpng
