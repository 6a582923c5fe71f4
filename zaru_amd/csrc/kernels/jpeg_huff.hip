// jpeg_huff.hip -- baseline JPEG Huffman entropy decoding on the device for
// streams with restart intervals: one thread per interval (T.81 F.2.2.5: every RSTn resets the
// DC predictions and byte-aligns the bit stream, so intervals decode independently -- the
// parallelism the reference's decoders never use, crates/zaru-image/src/jpeg.rs:107-205 and
// TODO.txt:9-12).  The decode is runtime/jpeg.cpp's entropy_decode restated (same tables, same
// lookahead fast paths, same byte stuffing / marker rule), so the coefficients are identical and
// the IDCT / colour stages downstream produce the same bytes as the host path.
#include "../runtime/zr_jpeg.h"

namespace zr {
namespace {

constexpr uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// the host Bits reader over one interval's bytes: 0xFF00 is a stuffed 0xFF, any other 0xFFxx (the
// interval's RSTn / EOI) feeds zero bits from there on.  The bytes come through a window of
// aligned 16-B words: `cur` is consumed, `nxt` only peeked at (a 0xFF at the end of `cur`) and
// `far` is in flight -- issued one word before anything reads it, so no read waits on the load
// just issued (a byte-serial reader is one dependent ~2 us global load per byte).
struct DevBits {
    const uint4 *base;  // the scan data (16-B aligned, >= 32 B of slack past the end)
    int p, n;           // next byte, end of the interval
    uint64_t acc;
    int cnt;
    bool marker;
    int wb;             // byte offset of `cur`
    uint4 cur, nxt, far;
    __device__ void init(const uint8_t *data, int start, int end) {
        base = reinterpret_cast<const uint4 *>(data);
        p = start;
        n = end;
        acc = 0;
        cnt = 0;
        marker = false;
        wb = start & ~15;
        cur = base[wb >> 4];
        nxt = base[(wb >> 4) + 1];
        far = base[(wb >> 4) + 2];
    }
    static __device__ __forceinline__ uint32_t byte_of(const uint4 &w, int o) {
        const int k = o >> 2;
        const uint32_t d = k == 0 ? w.x : k == 1 ? w.y : k == 2 ? w.z : w.w;
        return (d >> ((o & 3) * 8)) & 0xFFu;
    }
    __device__ void fill() {
        while (cnt <= 56) {
            uint32_t b = 0;
            if (!marker && p < n) {
                if (p >= wb + 16) {  // slide the window; the load of the word after it starts now
                    cur = nxt;
                    nxt = far;
                    wb += 16;
                    far = base[(wb >> 4) + 2];
                }
                const int o = p - wb;
                b = byte_of(cur, o);
                if (b == 0xFF) {
                    const uint32_t nx = p + 1 >= n ? 0xD9u : o < 15 ? byte_of(cur, o + 1) : nxt.x & 0xFFu;
                    if (nx == 0x00) {
                        p += 2;
                    } else {
                        marker = true;
                        b = 0;
                    }
                } else {
                    p++;
                }
            }
            acc |= (uint64_t)b << (56 - cnt);
            cnt += 8;
        }
    }
    __device__ uint32_t peek(int k) {
        if (cnt < k) fill();
        return (uint32_t)(acc >> (64 - k));
    }
    __device__ void skip(int k) {
        acc <<= k;
        cnt -= k;
    }
    __device__ int get(int k) {
        if (k == 0) return 0;
        const uint32_t v = peek(k);
        skip(k);
        return (int)v;
    }
};

__device__ __forceinline__ int huff_decode(DevBits &b, const JpegHuffTable &h, bool &bad) {
    const uint32_t l = b.peek(9);
    const uint16_t e = h.look[l];
    if (e) {
        b.skip(e >> 8);
        return e & 0xFF;
    }
    const uint32_t code = b.peek(16);
    for (int len = 10; len <= 16; len++) {
        const int32_t c = (int32_t)(code >> (16 - len));
        if (c <= h.maxcode[len]) {
            b.skip(len);
            return h.vals[(c + h.valoff[len]) & 255];
        }
    }
    bad = true;
    return 0;
}

__device__ __forceinline__ int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

// Every coefficient goes to the thread's block in LDS (natural order through an LDS zig-zag
// table) and the finished block leaves in eight 16-B stores: a zig-zag table in global memory
// puts one dependent global load in front of every coefficient store (~2.5 us per symbol).
__global__ __launch_bounds__(64) void jpeg_huff_kernel(const JpegHuffParams P) {
    __shared__ JpegHuffTable T[8];
    __shared__ uint8_t zz[64];
    __shared__ int4 sblk[64][8];  // one 64-coefficient int16 block per thread
    {  // the tables, 16 B per thread-step
        const uint4 *src = reinterpret_cast<const uint4 *>(P.tables);
        uint4 *dst = reinterpret_cast<uint4 *>(T);
        constexpr int n16 = (int)(8 * sizeof(JpegHuffTable) / 16);
        for (int i = threadIdx.x; i < n16; i += 64) dst[i] = src[i];
        zz[threadIdx.x] = kZigzag[threadIdx.x];
    }
    __syncthreads();
    int4 *const mine = sblk[threadIdx.x];
    int16_t *const co = reinterpret_cast<int16_t *>(mine);
    const int iv = blockIdx.x * 64 + threadIdx.x;
    if (iv >= P.n_iv) return;
    DevBits bits;
    bits.init(P.data, P.iv_off[iv], P.iv_off[iv + 1]);
    int pred[3] = {0, 0, 0};
    bool bad = false;
    const int m0 = iv * P.restart, m1 = min(m0 + P.restart, P.nmcu);
    for (int m = m0; m < m1 && !bad; m++) {
        const int my = m / P.mcux, mx = m - my * P.mcux;
        for (int c = 0; c < P.ncomp; c++) {
            const JpegHuffTable &dc = T[P.td[c]], &ac = T[4 + P.ta[c]];
            for (int v = 0; v < P.cv[c]; v++)
                for (int h = 0; h < P.ch[c]; h++) {
                    const int by = my * P.cv[c] + v, bx = mx * P.ch[c] + h;
                    int4 *const b4 = reinterpret_cast<int4 *>(
                        P.coef + (P.coef_off[c] + (int64_t)by * P.bw[c] + bx) * 64);
#pragma unroll
                    for (int z = 0; z < 8; z++) mine[z] = make_int4(0, 0, 0, 0);
                    const int s = huff_decode(bits, dc, bad);
                    if (s > 11) bad = true;
                    pred[c] += s && s <= 11 ? extend(bits.get(s), s) : 0;
                    co[0] = (int16_t)pred[c];
                    for (int k = 1; k < 64 && !bad;) {
                        const int fa = ac.fast_ac[bits.peek(9)];
                        if (fa) {  // run, size and magnitude in one lookup
                            k += (fa >> 4) & 15;
                            bits.skip(fa & 15);
                            if (k > 63) {
                                bad = true;
                                break;
                            }
                            co[zz[k]] = (int16_t)(fa >> 8);
                            k++;
                            continue;
                        }
                        const int rs = huff_decode(bits, ac, bad);
                        const int r = rs >> 4, sz = rs & 15;
                        if (sz) {
                            k += r;
                            if (k > 63) {
                                bad = true;
                                break;
                            }
                            co[zz[k]] = (int16_t)extend(bits.get(sz), sz);
                            k++;
                        } else {
                            if (r != 15) break;
                            k += 16;
                        }
                    }
#pragma unroll
                    for (int z = 0; z < 8; z++) b4[z] = mine[z];
                }
        }
    }
    if (bad) *P.error = 1;
}

}  // namespace

const char *launch_jpeg_huff(const JpegHuffParams &p, hipStream_t s) {
    hipLaunchKernelGGL(jpeg_huff_kernel, dim3((p.n_iv + 63) / 64), dim3(64), 0, s, p);
    return "jpeg_huff_kernel";
}

}  // namespace zr
