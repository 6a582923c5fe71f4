// jpeg.hip -- the device half of the JPEG frame source: libjpeg-turbo's
// accurate integer IDCT (jidctint.c jpeg_idct_islow), its fancy upsampling (jdsample.c
// h2v1/h2v2_fancy_upsample) and YCbCr -> RGBA (jdcolor.c ycc_rgb_convert tables), restated
// operation for operation in integer arithmetic, so frames come out byte-identical to the
// reference's libjpeg-turbo backend (crates/zaru-image/src/jpeg.rs:164-182).
// Stage 1: one thread per 8x8 block (dequantise, column pass into an int workspace, row pass,
// range limit).  Stage 2: one thread per output pixel (upsample from clamped neighbours -- the
// edge replication libjpeg's context rows and first/last-column cases amount to -- and convert).
#include "../runtime/zr_jpeg.h"

namespace zr {
namespace {

constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373, F1_175 = 9633,
              F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819, F2_562 = 20995, F3_072 = 25172;

template <typename T>
__device__ __forceinline__ T descale(T x, int n) { return (x + ((T)1 << (n - 1))) >> n; }

// IDCT_range_limit(cinfo)[x & RANGE_MASK] (jdmaster.c prepare_range_limit_table)
__device__ __forceinline__ uint32_t idct_limit(int v) {
    const int x = v & 1023;
    return (uint32_t)(x < 128 ? x + 128 : x < 512 ? 255 : x < 896 ? 0 : x - 896);
}

// The shared butterfly of both passes: in[0..7] -> out[0..7] before the final descale.  T = int
// when every input is below 2^15 in magnitude: the islow rows sum to < 7.5 * 2^13 in absolute
// value, so every output is below 2^31 and the wrapping int32 arithmetic gives the exact
// result (intermediates that wrap cancel mod 2^32).  Legal 8-bit streams always take it
// (libjpeg: pass-1 outputs need BITS_IN_JSAMPLE + PASS1_BITS + 3 bits); a block of corrupt
// coefficients falls back to T = long long, libjpeg-turbo's 64-bit JLONG.
template <typename T>
__device__ __forceinline__ void islow_1d(T i0, T i1, T i2, T i3, T i4, T i5, T i6, T i7, T o[8]) {
    T z1 = (i2 + i6) * (T)F0_541;
    const T t2e = z1 + i6 * (T)-F1_847;
    const T t3e = z1 + i2 * (T)F0_765;
    const T t0e = (T)((i0 + i4) * (T)(1 << CONST_BITS));
    const T t1e = (T)((i0 - i4) * (T)(1 << CONST_BITS));
    const T t10 = t0e + t3e, t13 = t0e - t3e, t11 = t1e + t2e, t12 = t1e - t2e;
    T t0 = i7, t1 = i5, t2 = i3, t3 = i1;
    z1 = t0 + t3;
    T z2 = t1 + t2, z3 = t0 + t2, z4 = t1 + t3;
    const T z5 = (z3 + z4) * (T)F1_175;
    t0 = t0 * (T)F0_298;
    t1 = t1 * (T)F2_053;
    t2 = t2 * (T)F3_072;
    t3 = t3 * (T)F1_501;
    z1 = z1 * (T)-F0_899;
    z2 = z2 * (T)-F2_562;
    z3 = z3 * (T)-F1_961;
    z4 = z4 * (T)-F0_390;
    z3 += z5;
    z4 += z5;
    t0 += z1 + z3;
    t1 += z2 + z4;
    t2 += z2 + z3;
    t3 += z1 + z4;
    o[0] = t10 + t3;
    o[7] = t10 - t3;
    o[1] = t11 + t2;
    o[6] = t11 - t2;
    o[2] = t12 + t1;
    o[5] = t12 - t1;
    o[3] = t13 + t0;
    o[4] = t13 - t0;
}

// int32 wrapping multiply/add: done in uint32 so the wrap is defined
struct W32 {
    uint32_t v;
    __device__ W32() = default;
    __device__ constexpr W32(int x) : v((uint32_t)x) {}
    __device__ W32 operator+(W32 o) const { return W32((int)(v + o.v)); }
    __device__ W32 operator-(W32 o) const { return W32((int)(v - o.v)); }
    __device__ W32 operator*(W32 o) const { return W32((int)(v * o.v)); }
    __device__ W32 &operator+=(W32 o) { v += o.v; return *this; }
    __device__ W32 operator>>(int n) const { return W32((int)v >> n); }
    __device__ W32 operator<<(int n) const { return W32((int)(v << n)); }
    __device__ int i() const { return (int)v; }
};

template <typename T>
__device__ __forceinline__ int as_int(T x) { return (int)x; }
template <>
__device__ __forceinline__ int as_int<W32>(W32 x) { return x.i(); }

// pass 1 over the 8 columns of the dequantised block `d` into the workspace
template <typename T>
__device__ __forceinline__ void idct_pass1(const int d[64], int ws[64]) {
#pragma unroll
    for (int x = 0; x < 8; ++x) {
        T o[8];
        islow_1d<T>(T(d[x]), T(d[8 + x]), T(d[16 + x]), T(d[24 + x]), T(d[32 + x]), T(d[40 + x]), T(d[48 + x]),
                    T(d[56 + x]), o);
#pragma unroll
        for (int k = 0; k < 8; ++k) ws[k * 8 + x] = as_int(descale<T>(o[k], CONST_BITS - PASS1_BITS));
    }
}

// pass 2 over row r of the workspace: 8 samples packed little-endian in two words
template <typename T>
__device__ __forceinline__ uint2 idct_pass2(const int *w) {
    T o[8];
    islow_1d<T>(T(w[0]), T(w[1]), T(w[2]), T(w[3]), T(w[4]), T(w[5]), T(w[6]), T(w[7]), o);
    uint32_t b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = idct_limit(as_int(descale<T>(o[k], CONST_BITS + PASS1_BITS + 3)));
    return make_uint2(b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24, b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24);
}

// One thread per block: the 128-B block in eight 16-B loads, everything in registers (the
// quantisation tables in LDS: a per-lane component index into the kernel argument would put
// them in scratch), each output row one 8-B store.
__global__ __launch_bounds__(256) void jpeg_idct_kernel(const JpegParams P) {
    __shared__ uint16_t sq[4][64];
    reinterpret_cast<uint16_t *>(sq)[threadIdx.x] = reinterpret_cast<const uint16_t *>(P.q)[threadIdx.x];
    __syncthreads();
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= P.total_blocks) return;
    int c = 0;
    while (c + 1 < P.ncomp && g >= P.coef_off[c + 1]) ++c;
    const int qs = c == 0 ? P.qsel[0] : c == 1 ? P.qsel[1] : P.qsel[2];
    const int bw = c == 0 ? P.bw[0] : c == 1 ? P.bw[1] : P.bw[2];
    const int64_t coff = c == 0 ? P.coef_off[0] : c == 1 ? P.coef_off[1] : P.coef_off[2];
    const int64_t poff = c == 0 ? P.plane_off[0] : c == 1 ? P.plane_off[1] : P.plane_off[2];
    const int b = g - (int)coff;
    const int by = b / bw, bx = b - by * bw;
    const int4 *in4 = reinterpret_cast<const int4 *>(P.coef + (int64_t)g * 64);
    int d[64];
    int mx = 0;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
        const int4 t = in4[v];
        const int w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const int k = v * 8 + h * 2;
            d[k] = (int)(int16_t)(w[h] & 0xFFFF) * (int)sq[qs][k];  // DEQUANTIZE = coef * quant
            d[k + 1] = (w[h] >> 16) * (int)sq[qs][k + 1];
            mx = max(mx, max(abs(d[k]), abs(d[k + 1])));
        }
    }
    int ws[64];
    if (mx < 32768)
        idct_pass1<W32>(d, ws);
    else
        idct_pass1<long long>(d, ws);
    int mw = 0;
#pragma unroll
    for (int k = 0; k < 64; ++k) mw = max(mw, abs(ws[k]));
    uint8_t *dst = P.planes + poff + (int64_t)(by * 8) * (bw * 8) + bx * 8;
    const int64_t stride = (int64_t)bw * 8;
#pragma unroll
    for (int r = 0; r < 8; ++r)
        *reinterpret_cast<uint2 *>(dst + r * stride) =
            mw < 32768 ? idct_pass2<W32>(ws + r * 8) : idct_pass2<long long>(ws + r * 8);
}

__device__ __forceinline__ int clamp255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

// one 4-B store per pixel when the frame buffer and its row stride allow it (the ABI only asks
// for row_stride >= 4 * width)
__device__ __forceinline__ void put_rgba(uint8_t *o, uint32_t px, const JpegParams &P) {
    if ((((uintptr_t)P.out | (uintptr_t)P.out_stride) & 3) == 0) {
        *reinterpret_cast<uint32_t *>(o) = px;
    } else {
        o[0] = (uint8_t)px;
        o[1] = (uint8_t)(px >> 8);
        o[2] = (uint8_t)(px >> 16);
        o[3] = (uint8_t)(px >> 24);
    }
}

__global__ __launch_bounds__(256) void jpeg_color_kernel(const JpegParams P) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= P.W || y >= P.H) return;
    const uint8_t *yp = P.planes + P.plane_off[0];
    const int ystride = P.bw[0] * 8;
    const int Y = yp[(int64_t)y * ystride + x];
    uint8_t *o = P.out + (int64_t)y * P.out_stride + 4 * x;
    if (P.ncomp == 1) {  // gray -> RGB replication
        put_rgba(o, (uint32_t)Y * 0x010101u | 0xFF000000u, P);
        return;
    }
    const int cstride = P.bw[1] * 8;
    int chroma[2];
    for (int k = 0; k < 2; ++k) {
        const uint8_t *cp = P.planes + P.plane_off[1 + k];
        if (P.hs == 1 && P.vs == 1) {
            chroma[k] = cp[(int64_t)y * cstride + x];
        } else if (P.vs == 1) {  // h2v1_fancy_upsample
            const int j = x >> 1, jn = (x & 1) ? min(j + 1, P.cw - 1) : max(j - 1, 0);
            const int row = y * cstride;
            const int v3 = cp[row + j] * 3, vn = cp[row + jn];
            chroma[k] = (x & 1) ? (v3 + vn + 2) >> 2 : (v3 + vn + 1) >> 2;
        } else {  // h2v2_fancy_upsample: column sums of this and the nearer neighbouring row
            const int i = y >> 1, in = (y & 1) ? min(i + 1, P.ch - 1) : max(i - 1, 0);
            const uint8_t *r0 = cp + (int64_t)i * cstride, *r1 = cp + (int64_t)in * cstride;
            const int j = x >> 1, jn = (x & 1) ? min(j + 1, P.cw - 1) : max(j - 1, 0);
            const int cs = r0[j] * 3 + r1[j], csn = r0[jn] * 3 + r1[jn];
            chroma[k] = (x & 1) ? (cs * 3 + csn + 7) >> 4 : (cs * 3 + csn + 8) >> 4;
        }
    }
    // jdcolor.c build_ycc_rgb_table: SCALEBITS 16, ONE_HALF, FIX(x) = x * 65536 + 0.5
    // (|cb|, |cr| <= 128: every product and sum below fits int32)
    const int cb = chroma[0] - 128, cr = chroma[1] - 128;
    const int r_off = (91881 * cr + 32768) >> 16;
    const int b_off = (116130 * cb + 32768) >> 16;
    const int g_off = (-22554 * cb + 32768 + -46802 * cr) >> 16;
    put_rgba(o, (uint32_t)clamp255(Y + r_off) | (uint32_t)clamp255(Y + g_off) << 8 |
                    (uint32_t)clamp255(Y + b_off) << 16 | 0xFF000000u, P);  // TJPF_RGBA
}

}  // namespace

const char *launch_jpeg(const JpegParams &p, hipStream_t s) {
    hipLaunchKernelGGL(jpeg_idct_kernel, dim3((p.total_blocks + 255) / 256), dim3(256), 0, s, p);
    hipLaunchKernelGGL(jpeg_color_kernel, dim3((p.W + 63) / 64, (p.H + 3) / 4), dim3(256), 0, s, p);
    return "jpeg_idct_kernel+jpeg_color_kernel";
}

}  // namespace zr
