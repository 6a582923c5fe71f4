/*
 * jpeg.c -- TEST INFRASTRUCTURE ONLY (see oracle.h): a scalar CPU restatement of the pixel
 * stages of libjpeg-turbo's default decode, the library behind the reference's libjpeg-turbo
 * JPEG backend (crates/zaru-image/src/jpeg.rs:164-182; turbojpeg 0.5.3 / turbojpeg-sys 0.2.3,
 * Cargo.lock:2945-2958).  libjpeg-turbo is third-party and not vendored in /root/reference;
 * this follows its published algorithms:
 *   jidctint.c jpeg_idct_islow   -- accurate integer IDCT (CONST_BITS 13, PASS1_BITS 2)
 *   jdmaster.c prepare_range_limit_table -- post-IDCT range limiting
 *   jdsample.c h2v1_fancy_upsample / h2v2_fancy_upsample, jdmainct.c context rows
 *   jdcolor.c build_ycc_rgb_table / ycc_rgb_convert (SCALEBITS 16), RGBA alpha 0xFF
 * written as libjpeg's row loops (explicit first / last column cases, context-row pointers),
 * independently of the GPU kernels' per-pixel formulation.  Input: the quantised coefficients
 * of zr_jpeg_coefficients (the product's host entropy decoder); pinned against Pillow's
 * libjpeg-turbo decode in tests/test_oracle_jpeg.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define CONST_BITS 13
#define PASS1_BITS 2
typedef long long JLONG;
#define DESCALE(x, n) (((x) + ((JLONG)1 << ((n)-1))) >> (n))

static uint8_t range_limit_idct(JLONG v) {
    int x = (int)(v & 1023);
    return (uint8_t)(x < 128 ? x + 128 : x < 512 ? 255 : x < 896 ? 0 : x - 896);
}

static void idct_islow(const int16_t *coef, const uint16_t *q, uint8_t *out, int stride) {
    int ws[64];
    for (int ctr = 0; ctr < 8; ctr++) {
        const int16_t *in = coef + ctr;
        const uint16_t *qp = q + ctr;
        JLONG z1, z2, z3, z4, z5, tmp0, tmp1, tmp2, tmp3, tmp10, tmp11, tmp12, tmp13;
        z2 = (JLONG)in[16] * qp[16];
        z3 = (JLONG)in[48] * qp[48];
        z1 = (z2 + z3) * 4433;
        tmp2 = z1 + z3 * -15137;
        tmp3 = z1 + z2 * 6270;
        z2 = (JLONG)in[0] * qp[0];
        z3 = (JLONG)in[32] * qp[32];
        tmp0 = (z2 + z3) << CONST_BITS;
        tmp1 = (z2 - z3) << CONST_BITS;
        tmp10 = tmp0 + tmp3;
        tmp13 = tmp0 - tmp3;
        tmp11 = tmp1 + tmp2;
        tmp12 = tmp1 - tmp2;
        tmp0 = (JLONG)in[56] * qp[56];
        tmp1 = (JLONG)in[40] * qp[40];
        tmp2 = (JLONG)in[24] * qp[24];
        tmp3 = (JLONG)in[8] * qp[8];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        z4 = tmp1 + tmp3;
        z5 = (z3 + z4) * 9633;
        tmp0 = tmp0 * 2446;
        tmp1 = tmp1 * 16819;
        tmp2 = tmp2 * 25172;
        tmp3 = tmp3 * 12299;
        z1 = z1 * -7373;
        z2 = z2 * -20995;
        z3 = z3 * -16069;
        z4 = z4 * -3196;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        ws[ctr + 0] = (int)DESCALE(tmp10 + tmp3, CONST_BITS - PASS1_BITS);
        ws[ctr + 56] = (int)DESCALE(tmp10 - tmp3, CONST_BITS - PASS1_BITS);
        ws[ctr + 8] = (int)DESCALE(tmp11 + tmp2, CONST_BITS - PASS1_BITS);
        ws[ctr + 48] = (int)DESCALE(tmp11 - tmp2, CONST_BITS - PASS1_BITS);
        ws[ctr + 16] = (int)DESCALE(tmp12 + tmp1, CONST_BITS - PASS1_BITS);
        ws[ctr + 40] = (int)DESCALE(tmp12 - tmp1, CONST_BITS - PASS1_BITS);
        ws[ctr + 24] = (int)DESCALE(tmp13 + tmp0, CONST_BITS - PASS1_BITS);
        ws[ctr + 32] = (int)DESCALE(tmp13 - tmp0, CONST_BITS - PASS1_BITS);
    }
    for (int ctr = 0; ctr < 8; ctr++) {
        const int *w = ws + ctr * 8;
        uint8_t *o = out + ctr * stride;
        JLONG z1, z2, z3, z4, z5, tmp0, tmp1, tmp2, tmp3, tmp10, tmp11, tmp12, tmp13;
        z2 = w[2];
        z3 = w[6];
        z1 = (z2 + z3) * 4433;
        tmp2 = z1 + z3 * -15137;
        tmp3 = z1 + z2 * 6270;
        z2 = (JLONG)w[0] + ((JLONG)1 << (PASS1_BITS + 2)); /* fudge factor for the final descale */
        z3 = w[4];
        tmp0 = (z2 + z3) << CONST_BITS;
        tmp1 = (z2 - z3) << CONST_BITS;
        tmp10 = tmp0 + tmp3;
        tmp13 = tmp0 - tmp3;
        tmp11 = tmp1 + tmp2;
        tmp12 = tmp1 - tmp2;
        tmp0 = w[7];
        tmp1 = w[5];
        tmp2 = w[3];
        tmp3 = w[1];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        z4 = tmp1 + tmp3;
        z5 = (z3 + z4) * 9633;
        tmp0 = tmp0 * 2446;
        tmp1 = tmp1 * 16819;
        tmp2 = tmp2 * 25172;
        tmp3 = tmp3 * 12299;
        z1 = z1 * -7373;
        z2 = z2 * -20995;
        z3 = z3 * -16069;
        z4 = z4 * -3196;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        const int sh = CONST_BITS + PASS1_BITS + 3;
        o[0] = range_limit_idct((tmp10 + tmp3) >> sh);
        o[7] = range_limit_idct((tmp10 - tmp3) >> sh);
        o[1] = range_limit_idct((tmp11 + tmp2) >> sh);
        o[6] = range_limit_idct((tmp11 - tmp2) >> sh);
        o[2] = range_limit_idct((tmp12 + tmp1) >> sh);
        o[5] = range_limit_idct((tmp12 - tmp1) >> sh);
        o[3] = range_limit_idct((tmp13 + tmp0) >> sh);
        o[4] = range_limit_idct((tmp13 - tmp0) >> sh);
    }
}

static uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

/* one output row pair of h2v2_fancy_upsample for chroma row i (v = 0 upper, 1 lower) */
static void h2v2_row(const uint8_t *in0, const uint8_t *in1, int cw, uint8_t *out) {
    int thiscolsum = in0[0] * 3 + in1[0];
    int nextcolsum = cw > 1 ? in0[1] * 3 + in1[1] : thiscolsum;
    int lastcolsum;
    *out++ = (uint8_t)((thiscolsum * 4 + 8) >> 4);
    *out++ = (uint8_t)((thiscolsum * 3 + nextcolsum + 7) >> 4);
    lastcolsum = thiscolsum;
    thiscolsum = nextcolsum;
    for (int col = 2; col < cw; col++) {
        nextcolsum = in0[col] * 3 + in1[col];
        *out++ = (uint8_t)((thiscolsum * 3 + lastcolsum + 8) >> 4);
        *out++ = (uint8_t)((thiscolsum * 3 + nextcolsum + 7) >> 4);
        lastcolsum = thiscolsum;
        thiscolsum = nextcolsum;
    }
    if (cw > 1) {
        *out++ = (uint8_t)((thiscolsum * 3 + lastcolsum + 8) >> 4);
        *out++ = (uint8_t)((thiscolsum * 4 + 7) >> 4);
    }
}

static void h2v1_row(const uint8_t *in, int cw, uint8_t *out) {
    int invalue = in[0];
    *out++ = (uint8_t)invalue;
    *out++ = (uint8_t)((invalue * 3 + (cw > 1 ? in[1] : invalue) + 2) >> 2);
    for (int col = 1; col < cw - 1; col++) {
        invalue = in[col] * 3;
        *out++ = (uint8_t)((invalue + in[col - 1] + 1) >> 2);
        *out++ = (uint8_t)((invalue + in[col + 1] + 2) >> 2);
    }
    if (cw > 1) {
        invalue = in[cw - 1];
        *out++ = (uint8_t)((invalue * 3 + in[cw - 2] + 1) >> 2);
        *out++ = (uint8_t)invalue;
    }
}

int zo_jpeg_pixels(const int16_t *coef, uint32_t width, uint32_t height, uint32_t ncomp,
                   uint32_t h_samp, uint32_t v_samp, const uint32_t *bw, const uint32_t *bh,
                   const uint32_t *qsel, const uint16_t *quant /* [4][64] */, uint8_t *rgba) {
    uint8_t *planes[3] = {NULL, NULL, NULL};
    size_t boff = 0;
    for (uint32_t c = 0; c < ncomp; c++) {
        planes[c] = (uint8_t *)malloc((size_t)bw[c] * bh[c] * 64);
        if (!planes[c]) return -1;
        const int stride = (int)bw[c] * 8;
        for (uint32_t by = 0; by < bh[c]; by++)
            for (uint32_t bx = 0; bx < bw[c]; bx++)
                idct_islow(coef + (boff + (size_t)by * bw[c] + bx) * 64, quant + 64 * qsel[c],
                           planes[c] + (size_t)by * 8 * stride + bx * 8, stride);
        boff += (size_t)bw[c] * bh[c];
    }
    const int W = (int)width, H = (int)height;
    if (ncomp == 1) {
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                uint8_t *o = rgba + ((size_t)y * W + x) * 4;
                o[0] = o[1] = o[2] = planes[0][(size_t)y * bw[0] * 8 + x];
                o[3] = 255;
            }
        free(planes[0]);
        return 0;
    }
    const int cw = (W + (int)h_samp - 1) / (int)h_samp, ch = (H + (int)v_samp - 1) / (int)v_samp;
    const int cstride = (int)bw[1] * 8;
    uint8_t *up[2];
    up[0] = (uint8_t *)malloc((size_t)2 * cw + 2);
    up[1] = (uint8_t *)malloc((size_t)2 * cw + 2);
    for (int y = 0; y < H; y++) {
        const uint8_t *rows[2];
        for (int k = 0; k < 2; k++) {
            const uint8_t *pl = planes[1 + k];
            if (h_samp == 1 && v_samp == 1) {
                rows[k] = pl + (size_t)y * cstride;
            } else if (v_samp == 1) {
                h2v1_row(pl + (size_t)y * cstride, cw, up[k]);
                rows[k] = up[k];
            } else {
                /* context rows: above row 0 is row 0, below the last is the last (jdmainct.c) */
                const int i = y >> 1;
                const int nb = (y & 1) ? (i + 1 < ch ? i + 1 : ch - 1) : (i > 0 ? i - 1 : 0);
                h2v2_row(pl + (size_t)i * cstride, pl + (size_t)nb * cstride, cw, up[k]);
                rows[k] = up[k];
            }
        }
        for (int x = 0; x < W; x++) {
            const int Y = planes[0][(size_t)y * bw[0] * 8 + x];
            const int cb = rows[0][x] - 128, cr = rows[1][x] - 128;
            /* Cr_r_tab, Cb_b_tab: RIGHT_SHIFT(FIX(k) * x + ONE_HALF, 16); Cb_g_tab carries ONE_HALF */
            const JLONG cr_r = (91881LL * cr + 32768) >> 16, cb_b = (116130LL * cb + 32768) >> 16;
            const JLONG cb_g = -22554LL * cb + 32768, cr_g = -46802LL * cr;
            uint8_t *o = rgba + ((size_t)y * W + x) * 4;
            o[0] = clamp255(Y + (int)cr_r);
            o[1] = clamp255(Y + (int)((cb_g + cr_g) >> 16));
            o[2] = clamp255(Y + (int)cb_b);
            o[3] = 255;
        }
    }
    free(up[0]);
    free(up[1]);
    for (int c = 0; c < 3; c++) free(planes[c]);
    return 0;
}
