// glibc_math.h -- the four libm functions the reference evaluates on its hot path (Rust's
// f32::{sin, cos, exp, atan2} call the platform libm: glibc on x86_64-linux-gnu), restated so
// device code produces glibc's bits instead of the GPU's own (<= 2 ulp) cosf/sinf/expf/atan2f.
// The same source compiles for the host (g++, tools/libm_exhaustive.cpp) and for gfx950.
//
// Which glibc: 2.35 (this image and the GPU box).  On an x86_64 CPU with FMA + AVX2 (both hosts)
// the IFUNC resolver of sinf / cosf / expf picks the "-fma" multiarch builds: the generic C
// compiled with -mfma, where GCC contracts every `a + b * c` whose product has no other kind of
// use.  atanf / atan2f are not IFUNCs (plain x86_64 builds, no FMA).  ZR_GLIBC_FMA selects the
// contraction (1 = the FMA build, the default; 0 = the baseline build).
//
// Sources restated (glibc 2.35, names as in the tree):
//   sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h (sinf_poly, reduce_fast, reduce_large),
//     sincosf_data.c (__sincosf_table), s_sincosf_data / __inv_pio4
//   sysdeps/ieee754/flt-32/e_expf.c, e_exp2f_data.c (__exp2f_data, EXP2F_TABLE_BITS = 5)
//   sysdeps/ieee754/flt-32/e_atan2f.c, s_atanf.c (fdlibm float versions)
// The tables were cross-checked byte for byte against this image's libm.so.6 .rodata, and every
// function is verified over all 2^32 inputs (atan2f: atanf exhaustively plus random pairs) by
// tools/libm_exhaustive.cpp; tests/test_glibc_math_cpu.py and tests/test_gpu_glibc_math.py
// re-check strided samples on the host and on the GPU.
//
// Callers: kernels/track.hip (LandmarkTracker::track_impl on the device).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define ZR_HD __host__ __device__ __forceinline__
#define ZR_CONST static __constant__
#else
#include <string.h>
#define ZR_HD static inline
#define ZR_CONST static const
#endif

#ifndef ZR_GLIBC_FMA
#define ZR_GLIBC_FMA 1
#endif

namespace zr {
namespace glibc {

#if ZR_GLIBC_FMA
ZR_HD double mla(double a, double b, double c) { return __builtin_fma(a, b, c); }  // c + a*b, one rounding
#else
ZR_HD double mla(double a, double b, double c) { return c + a * b; }
#endif

ZR_HD uint32_t asuint(float f) {
#ifdef __HIPCC__
    return __builtin_bit_cast(uint32_t, f);
#else
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
#endif
}
ZR_HD float asfloat(uint32_t u) {
#ifdef __HIPCC__
    return __builtin_bit_cast(float, u);
#else
    float f;
    memcpy(&f, &u, 4);
    return f;
#endif
}
ZR_HD double asdouble(uint64_t u) {
#ifdef __HIPCC__
    return __builtin_bit_cast(double, u);
#else
    double d;
    memcpy(&d, &u, 8);
    return d;
#endif
}
ZR_HD uint64_t asuint64(double d) {
#ifdef __HIPCC__
    return __builtin_bit_cast(uint64_t, d);
#else
    uint64_t u;
    memcpy(&u, &d, 8);
    return u;
#endif
}

// ---------------------------------------------------------------- sinf / cosf
// __sincosf_table[0..1] (sincosf_data.c): field order c0, c1, s1, c2, s2, c3, s3, c4; table 1 is
// table 0 with the cosine coefficients negated (quadrants 2, 3).
#define ZR_SC_HPI_INV 0x1.45F306DC9C883p+23  // 2/pi * 2^24 (no TOINT_INTRINSICS on x86_64)
#define ZR_SC_HPI 0x1.921FB54442D18p0        // pi/2
#define ZR_SC_C1 (-0x1.ffffffd0c621cp-2)
#define ZR_SC_S1 (-0x1.555545995a603p-3)
#define ZR_SC_C2 0x1.55553e1068f19p-5
#define ZR_SC_S2 0x1.1107605230bc4p-7
#define ZR_SC_C3 (-0x1.6c087e89a359dp-10)
#define ZR_SC_S3 (-0x1.994eb3774cf24p-13)
#define ZR_SC_C4 0x1.99343027bf8c3p-16

// __inv_pio4: 4/pi as overlapping 32-bit windows, entry i = bits [8i-24, 8i+8) of 2/pi's
// fraction (0xa2f9836e 4e441529 fc2757d1 f534ddc0 db629599 3c439041 ...)
ZR_CONST uint32_t kInvPio4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};

ZR_HD uint32_t abstop12(float x) { return (asuint(x) >> 20) & 0x7ff; }

// sincosf.h sinf_poly: n even -> sine polynomial, n odd -> cosine; `neg` selects table 1
ZR_HD float sinf_poly(double x, double x2, int n, bool neg) {
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = mla(x2, ZR_SC_S3, ZR_SC_S2);
        const double x7 = x3 * x2;
        const double s = mla(x3, ZR_SC_S1, x);
        return (float)mla(x7, s1, s);
    }
    const double c0 = neg ? -1.0 : 1.0, c1 = neg ? -ZR_SC_C1 : ZR_SC_C1;
    const double c2k = neg ? -ZR_SC_C2 : ZR_SC_C2, c3 = neg ? -ZR_SC_C3 : ZR_SC_C3;
    const double c4 = neg ? -ZR_SC_C4 : ZR_SC_C4;
    const double x4 = x2 * x2;
    const double c2 = mla(x2, c4, c3);
    const double cc1 = mla(x2, c1, c0);
    const double x6 = x4 * x2;
    const double c = mla(x4, c2k, cc1);
    return (float)mla(x6, c2, c);
}

// reduce_fast, non-TOINT_INTRINSICS form: |x| < 120, quadrant in bits 24..31 of x * 2/pi * 2^24
ZR_HD double reduce_fast(double x, int *np) {
    const double r = x * ZR_SC_HPI_INV;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return mla(-(double)n, ZR_SC_HPI, x);  // x - n * hpi
}

// reduce_large: Payne-Hanek with 4/pi windows, |x| >= 120
ZR_HD double reduce_large(uint32_t xi, int *np) {
    const uint32_t *arr = &kInvPio4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    res0 = (uint32_t)(xi * arr[0]);
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    const double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * 0x1.921FB54442D18p-62;  // pi63 = pi * 2^-63 (sincosf.h)
}

ZR_HD float sinf(float y) {
    double x = y;
    int n;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {  // |y| < pi/4
        const double s = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sinf_poly(x, s, 0, false);
    } else if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast(x, &n);
        const double s = (n & 3) == 0 || (n & 3) == 3 ? 1.0 : -1.0;  // sign[n & 3]
        return sinf_poly(x * s, x * x, n, (n & 2) != 0);
    } else if (abstop12(y) < abstop12(__builtin_inff())) {
        const uint32_t xi = asuint(y);
        const int sign = xi >> 31;
        x = reduce_large(xi, &n);
        const int q = (n + sign) & 3;
        const double s = q == 0 || q == 3 ? 1.0 : -1.0;
        return sinf_poly(x * s, x * x, n, (q & 2) != 0);
    }
    return (y - y) / (y - y);  // __math_invalidf
}

ZR_HD float cosf(float y) {
    double x = y;
    int n;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        const double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sinf_poly(x, x2, 1, false);
    } else if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast(x, &n);
        const double s = (n & 3) == 0 || (n & 3) == 3 ? 1.0 : -1.0;
        return sinf_poly(x * s, x * x, n ^ 1, (n & 2) != 0);
    } else if (abstop12(y) < abstop12(__builtin_inff())) {
        const uint32_t xi = asuint(y);
        const int sign = xi >> 31;
        x = reduce_large(xi, &n);
        const int q = (n + sign) & 3;
        const double s = q == 0 || q == 3 ? 1.0 : -1.0;
        return sinf_poly(x * s, x * x, n ^ 1, (q & 2) != 0);
    }
    return (y - y) / (y - y);
}

// ---------------------------------------------------------------- expf
// __exp2f_data.tab[i] = asuint64(2^(i/32)) - (i << 47)  (verified against libm's .rodata)
ZR_CONST uint64_t kExp2fTab[32] = {
    0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51,
    0x3fef72b83c7d517b, 0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1,
    0x3fef06fe0a31b715, 0x3feef1a7373aa9cb, 0x3feedea64c123422, 0x3feece086061892d,
    0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429, 0x3feea47eb03a5585,
    0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
    0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d,
    0x3feee89f995ad3ad, 0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069,
    0x3fef5818dcfba487, 0x3fef7c97337b9b5f, 0x3fefa4afa2a490da, 0x3fefd0765b6e4540};

ZR_HD float expf(float x) {
    const double xd = (double)x;
    const uint32_t abstop = (asuint(x) >> 20) & 0x7ff;
    if (abstop >= (asuint(88.0f) >> 20)) {  // |x| >= 88 or NaN
        if (asuint(x) == asuint(-__builtin_inff())) return 0.0f;
        if (abstop >= (asuint(__builtin_inff()) >> 20)) return x + x;
        if (x > 0x1.62e42ep6f) return __builtin_inff();  // __math_oflowf
        if (x < -0x1.9fe368p6f) return 0.0f;             // __math_uflowf
    }
    // z = x * N/ln2; kd = round(z) via the 1.5*2^52 shift; GCC contracts both uses of the
    // product (z + SHIFT and z - kd) in the FMA build
    const double invln2n = 0x1.71547652b82fep+5, shift = 0x1.8p+52;
#if ZR_GLIBC_FMA
    double kd = __builtin_fma(invln2n, xd, shift);
    const uint64_t ki = asuint64(kd);
    kd -= shift;
    const double r = __builtin_fma(invln2n, xd, -kd);
#else
    const double z = invln2n * xd;
    double kd = z + shift;
    const uint64_t ki = asuint64(kd);
    kd -= shift;
    const double r = z - kd;
#endif
    uint64_t t = kExp2fTab[ki % 32];
    t += ki << 47;
    const double s = asdouble(t);
    const double zz = mla(0x1.c6af84b912394p-20, r, 0x1.ebfce50fac4f3p-13);  // C0*r + C1
    const double r2 = r * r;
    double y = mla(0x1.62e42ff0c52d6p-6, r, 1.0);  // C2*r + 1
    y = mla(zz, r2, y);
    y = y * s;
    return (float)y;
}

// ---------------------------------------------------------------- atanf / atan2f (fdlibm)
ZR_CONST float kAtanHi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
ZR_CONST float kAtanLo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
ZR_CONST float kAT[11] = {3.3333334327e-01f,  -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                          9.0908870101e-02f,  -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                          4.9768779427e-02f,  -3.6531571299e-02f, 1.6285819933e-02f};

ZR_HD float atanf(float x) {
    const int32_t hx = (int32_t)asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {  // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? kAtanHi[3] + kAtanLo[3] : -kAtanHi[3] - kAtanLo[3];
    }
    if (ix < 0x3ee00000) {              // |x| < 0.4375
        if (ix < 0x31000000) return x;  // |x| < 2^-29
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3f980000) {      // |x| < 1.1875
            if (ix < 0x3f300000) {  // 7/16 <= |x| < 11/16
                id = 0;
                x = (2.0f * x - 1.0f) / (2.0f + x);
            } else {  // 11/16 <= |x| < 19/16
                id = 1;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else if (ix < 0x401c0000) {  // |x| < 2.4375
            id = 2;
            x = (x - 1.5f) / (1.0f + 1.5f * x);
        } else {  // 2.4375 <= |x| < 2^34
            id = 3;
            x = -1.0f / x;
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (kAT[0] + w * (kAT[2] + w * (kAT[4] + w * (kAT[6] + w * (kAT[8] + w * kAT[10])))));
    const float s2 = w * (kAT[1] + w * (kAT[3] + w * (kAT[5] + w * (kAT[7] + w * kAT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = kAtanHi[id] - ((x * (s1 + s2) - kAtanLo[id]) - x);
    return hx < 0 ? -r : r;
}

ZR_HD float atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f;
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)asuint(x), hy = (int32_t)asuint(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;  // NaN
    if (hx == 0x3f800000) return atanf(y);                  // x = 1.0
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);      // 2*sign(x) + sign(y)
    if (iy == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;    // |y/x| > 2^60
    else if (hx < 0 && k < -60) z = 0.0f;     // |y|/x < -2^60
    else z = atanf(__builtin_fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return asfloat(asuint(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

}  // namespace glibc
}  // namespace zr
