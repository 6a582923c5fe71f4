// epilogue.h -- the fused BlazeBlock tail shared by every 1x1-conv kernel:
//   out = post( pre(acc + bias) + residual )
// where the residual is the block input (res_mode 1) or its 2x2/2 max-pool (res_mode 2), and
// channels >= r_C of it are zero (the ONNX channel Pad).  The store goes through the output's
// (sN, sC, sP) strides, which is how graph outputs land in the reference's row-major layout.
// Also the C/D fragment row map of v_mfma_f32_32x32x2_f32.
#pragma once
#include "../runtime/zr_kernels.h"
#include "act.h"

namespace zr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// row of accumulator register r held by lane half kh (= lane / 32); the column is lane % 32
__device__ __forceinline__ int mfma32_row(int r, int kh) { return (r & 3) + 8 * (r >> 2) + 4 * kh; }

// One 32x32 accumulator tile of one lane: rows mbase + mfma32_row(r, kh), column (n, q).
// All residual loads of the tile are issued before any is used (clamped addresses, no branch
// around a load), so the tile pays one memory latency, not sixteen.
__device__ __forceinline__ void epilogue_tile(const GemmParams &P, const f32x16 &acc, int n, int q,
                                              int mbase, int kh) {
    float rv[16];
    if (P.res_mode == 1) {
        const float *rb = P.r + (int64_t)n * P.r_sN + q;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = mbase + mfma32_row(r, kh);
            const float v = rb[(int64_t)(m < P.r_C ? m : 0) * P.r_sC];
            rv[r] = m < P.r_C ? v : 0.f;
        }
    } else if (P.res_mode == 2) {
        const int y = q / P.out_W, x = q - y * P.out_W;
        const float *rb = P.r + (int64_t)n * P.r_sN + (int64_t)(2 * y) * P.r_W + 2 * x;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = mbase + mfma32_row(r, kh);
            const float *s0 = rb + (int64_t)(m < P.r_C ? m : 0) * P.r_sC;
            const float v = fmaxf(fmaxf(s0[0], s0[1]), fmaxf(s0[P.r_W], s0[P.r_W + 1]));
            rv[r] = m < P.r_C ? v : 0.f;
        }
    }
    float *ob = P.out + (int64_t)n * P.o_sN + (int64_t)q * P.o_sP;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = mbase + mfma32_row(r, kh);
        if (m >= P.M) continue;
        float v = apply_act(P.pre, acc[r] + P.bias[m], m);
        if (P.res_mode != 0) v += rv[r];  // ONNX Add of the (zero-padded) shortcut
        ob[(int64_t)m * P.o_sC] = apply_act(P.post, v, m);
    }
}

}  // namespace zr
