// epilogue.h -- the fused BlazeBlock tail shared by every 1x1-conv kernel:
//   out = post( pre(acc + bias) + residual )
// where the residual is the block input (res_mode 1) or its 2x2/2 max-pool (res_mode 2), and
// channels >= r_C of it are zero (the ONNX channel Pad).  The store goes through the output's
// (sN, sC, sP) strides, which is how graph outputs land in the reference's row-major layout.
// Also the C/D fragment row map of v_mfma_f32_32x32x2_f32.
//
// Addressing: every tensor a launch touches is < 2^31 floats (checked by the runtime), so
// offsets are 32-bit and added to uniform base pointers (saddr + voffset addressing, no 64-bit
// VALU address math per element).
#pragma once
#include "../runtime/zr_kernels.h"
#include "act.h"

namespace zr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// row of accumulator register r held by lane half kh (= lane / 32); the column is lane % 32
__device__ __forceinline__ int mfma32_row(int r, int kh) { return (r & 3) + 8 * (r >> 2) + 4 * kh; }

// One 32x32 accumulator tile of one lane: rows mbase + mfma32_row(r, kh), column (n, q).
// Loads (bias, residual, slopes) are all issued before any is used, from clamped addresses:
// the tile pays one memory latency, not sixteen.  epilogue_values leaves the 16 results in v;
// epilogue_tile also stores them.
// Rows r0 .. r0 + NR - 1 of the tile.  RES = false compiles the residual paths out (a kernel
// instance for launches with res_mode 0: the expand convs) -- their clamped loads otherwise
// hold registers in every instance and cost the store-bound GEMMs a wave per SIMD.
template <int NR = 16, bool RES = true>
__device__ __forceinline__ void epilogue_part(const GemmParams &P, const f32x16 &acc, int n, int q,
                                              int mbase, int kh, int r0, float *v) {
    auto chan = [&](int r) {
        const int m = mbase + mfma32_row(r0 + r, kh);
        return m < P.Mpad ? m : 0;
    };
#pragma unroll
    for (int r = 0; r < NR; ++r) v[r] = acc[r0 + r] + P.bias[chan(r)];
    float rv[NR];
    if (!RES) {
    } else if (P.res_mode == 1) {
        const uint32_t rb = (uint32_t)n * (uint32_t)P.r_sN + (uint32_t)q;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int m = mbase + mfma32_row(r0 + r, kh);
            const float x = P.r[rb + (uint32_t)(m < P.r_C ? m : 0) * (uint32_t)P.r_sC];
            rv[r] = m < P.r_C ? x : 0.f;
        }
    } else if (P.res_mode == 2) {
        const int y = q / P.out_W, x = q - y * P.out_W;
        const uint32_t rb = (uint32_t)n * (uint32_t)P.r_sN + (uint32_t)((2 * y) * P.r_W + 2 * x);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int m = mbase + mfma32_row(r0 + r, kh);
            const uint32_t o = rb + (uint32_t)(m < P.r_C ? m : 0) * (uint32_t)P.r_sC;
            const float p = fmaxf(fmaxf(P.r[o], P.r[o + 1]), fmaxf(P.r[o + P.r_W], P.r[o + P.r_W + 1]));
            rv[r] = m < P.r_C ? p : 0.f;
        }
    }
    apply_act_n<NR>(P.pre, v, chan);
    if (RES && P.res_mode != 0) {  // ONNX Add of the (zero-padded) shortcut
#pragma unroll
        for (int r = 0; r < NR; ++r) v[r] += rv[r];
    }
    apply_act_n<NR>(P.post, v, chan);
}

template <bool RES = true>
__device__ __forceinline__ void epilogue_values(const GemmParams &P, const f32x16 &acc, int n, int q,
                                                int mbase, int kh, float v[16]) {
    epilogue_part<16, RES>(P, acc, n, q, mbase, kh, 0, v);
}

template <bool RES = true>
__device__ __forceinline__ void epilogue_tile(const GemmParams &P, const f32x16 &acc, int n, int q,
                                              int mbase, int kh) {
    float v[16];
    epilogue_values<RES>(P, acc, n, q, mbase, kh, v);
    const uint32_t ob = (uint32_t)n * (uint32_t)P.o_sN + (uint32_t)q * (uint32_t)P.o_sP;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = mbase + mfma32_row(r, kh);
        if (m < P.M) P.out[ob + (uint32_t)m * (uint32_t)P.o_sC] = v[r];
    }
}

}  // namespace zr
