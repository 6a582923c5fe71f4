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
constexpr long long F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373,
                    F1_175 = 9633, F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819,
                    F2_562 = 20995, F3_072 = 25172;

__device__ __forceinline__ long long descale(long long x, int n) { return (x + (1LL << (n - 1))) >> n; }

// IDCT_range_limit(cinfo)[x & RANGE_MASK] (jdmaster.c prepare_range_limit_table)
__device__ __forceinline__ uint8_t idct_limit(long long v) {
    const int x = (int)(v & 1023);
    return (uint8_t)(x < 128 ? x + 128 : x < 512 ? 255 : x < 896 ? 0 : x - 896);
}

// The shared butterfly of both passes: in[0..7] -> out[0..7] before the final descale.
__device__ __forceinline__ void islow_1d(long long i0, long long i1, long long i2, long long i3, long long i4,
                                         long long i5, long long i6, long long i7, long long o[8]) {
    long long z1 = (i2 + i6) * F0_541;
    const long long t2e = z1 + i6 * -F1_847;
    const long long t3e = z1 + i2 * F0_765;
    const long long t0e = (i0 + i4) << CONST_BITS;
    const long long t1e = (i0 - i4) << CONST_BITS;
    const long long t10 = t0e + t3e, t13 = t0e - t3e, t11 = t1e + t2e, t12 = t1e - t2e;
    long long t0 = i7, t1 = i5, t2 = i3, t3 = i1;
    z1 = t0 + t3;
    long long z2 = t1 + t2, z3 = t0 + t2, z4 = t1 + t3;
    const long long z5 = (z3 + z4) * F1_175;
    t0 = t0 * F0_298;
    t1 = t1 * F2_053;
    t2 = t2 * F3_072;
    t3 = t3 * F1_501;
    z1 = z1 * -F0_899;
    z2 = z2 * -F2_562;
    z3 = z3 * -F1_961;
    z4 = z4 * -F0_390;
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

__global__ __launch_bounds__(256) void jpeg_idct_kernel(const JpegParams P) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= P.total_blocks) return;
    int c = 0;
    while (c + 1 < P.ncomp && g >= P.coef_off[c + 1]) ++c;
    const int b = g - (int)P.coef_off[c];
    const int by = b / P.bw[c], bx = b - by * P.bw[c];
    const int16_t *in = P.coef + (int64_t)g * 64;
    const uint16_t *q = P.q[P.qsel[c]];
    int ws[64];
    long long o[8];
    for (int x = 0; x < 8; ++x) {  // pass 1: columns from input (DEQUANTIZE = coef * quant)
        islow_1d((long long)in[x] * q[x], (long long)in[8 + x] * q[8 + x], (long long)in[16 + x] * q[16 + x],
                 (long long)in[24 + x] * q[24 + x], (long long)in[32 + x] * q[32 + x],
                 (long long)in[40 + x] * q[40 + x], (long long)in[48 + x] * q[48 + x],
                 (long long)in[56 + x] * q[56 + x], o);
        for (int k = 0; k < 8; ++k) ws[k * 8 + x] = (int)descale(o[k], CONST_BITS - PASS1_BITS);
    }
    uint8_t *plane = P.planes + P.plane_off[c];
    const int stride = P.bw[c] * 8;
    for (int r = 0; r < 8; ++r) {  // pass 2: rows of the workspace
        const int *w = ws + r * 8;
        islow_1d(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
        uint8_t *dst = plane + (int64_t)(by * 8 + r) * stride + bx * 8;
        for (int k = 0; k < 8; ++k) dst[k] = idct_limit(descale(o[k], CONST_BITS + PASS1_BITS + 3));
    }
}

__device__ __forceinline__ int clamp255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

__global__ __launch_bounds__(256) void jpeg_color_kernel(const JpegParams P) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= P.W || y >= P.H) return;
    const uint8_t *yp = P.planes + P.plane_off[0];
    const int ystride = P.bw[0] * 8;
    const int Y = yp[(int64_t)y * ystride + x];
    uint8_t *o = P.out + (int64_t)y * P.out_stride + 4 * x;
    if (P.ncomp == 1) {  // gray -> RGB replication
        o[0] = o[1] = o[2] = (uint8_t)Y;
        o[3] = 255;
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
    const int cb = chroma[0] - 128, cr = chroma[1] - 128;
    const int r_off = (int)((91881LL * cr + 32768) >> 16);
    const int b_off = (int)((116130LL * cb + 32768) >> 16);
    const int g_off = (int)((-22554LL * cb + 32768 + -46802LL * cr) >> 16);
    o[0] = (uint8_t)clamp255(Y + r_off);
    o[1] = (uint8_t)clamp255(Y + g_off);
    o[2] = (uint8_t)clamp255(Y + b_off);
    o[3] = 255;  // TJPF_RGBA
}

}  // namespace

const char *launch_jpeg(const JpegParams &p, hipStream_t s) {
    hipLaunchKernelGGL(jpeg_idct_kernel, dim3((p.total_blocks + 255) / 256), dim3(256), 0, s, p);
    hipLaunchKernelGGL(jpeg_color_kernel, dim3((p.W + 63) / 64, (p.H + 3) / 4), dim3(256), 0, s, p);
    return "jpeg_idct_kernel+jpeg_color_kernel";
}

}  // namespace zr
