// bneck.hip -- FaceMesh V2's bottleneck residual block in one launch: a 1x1
// reduction C -> C/2 (+ bias, PReLU), a 3x3 depthwise over the reduced planes, a 1x1 back to C
// (+ bias), the block input added back and a PReLU.  Reference: the Conv / PRelu / Add nodes of
// face_landmarks_detector.onnx that ORT / tract execute at crates/zaru/src/nn/mod.rs:483-533
// (face/landmark/mediapipe.rs:81-115; the plan's `gemm (ir=1) -> dwpw res=1` pairs, 14 of them at
// 128^2 / 64^2 / 32^2 with C = 16 / 32 / 64; fused here: the 128^2 and 64^2 ones).
//
// Unfused, the reduction writes C/2 planes to HBM and the dwpw launch reads them back and reads
// the block input again for the residual: 4C floats per position against the block's 2C.  Here a
// 256-thread workgroup owns TR = 256 / W output rows of one image:
//   phase A: the reduction of the band's TR + 2 input rows (the depthwise's halo; rows outside
//            the plane are the zero padding) into LDS, one position per thread, C/2 accumulators,
//            the block input read once from HBM (coalesced along the row), weights through the
//            scalar cache;
//   phase B: the dwpw_valu form over the staged planes -- per reduced channel the depthwise from
//            LDS, then the 1x1 accumulated into C registers -- and the epilogue, whose residual
//            read hits the lines phase A just fetched.
// Arithmetic and order are the unfused launches': the reduction is an fmaf chain over the input
// channels in order from +0 then + bias and the activation (the MFMA GEMM's chain, bitwise equal:
// tools/debug/mfma_order.hip), the depthwise bias + fmaf over the taps in (ky, kx) order with
// the padding read as +0, the 1x1 an fmaf chain over the reduced channels, then the shared
// epilogue order (bias, pre, + residual, post).  So fusing changes no output bit
// (tests/test_gpu_forms.py, -bneck).
#include "../runtime/zr_kernels.h"
#include "act.h"

namespace zr {

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int C, int W>
__global__ __launch_bounds__(256) void bneck_kernel(const GemmParams E, const DwPwParams D, int bands) {
    constexpr int MH = C / 2, TR = 256 / W, R = TR + 2, LW = W + 8, PL = R * W;
    static_assert(TR * W == 256 && W % 4 == 0, "bneck layout");
    __shared__ __attribute__((aligned(16))) float sT[MH * R * LW];  // reduced planes, zero columns
    const GemmParams &G = D.g;
    const int cpx = gridDim.x >> 3;  // gridDim.x is a multiple of 8: consecutive bands share an XCD
    const int tile = (blockIdx.x & 7) * cpx + (blockIdx.x >> 3);
    const int nimg = G.ncols / G.P;
    if (tile >= nimg * bands) return;  // whole workgroup, before any barrier
    const int n = tile / bands, oy0 = (tile - n * bands) * TR;
    if (G.nact && n >= *G.nact) return;
    const int tid = threadIdx.x, H = D.in.H;
    const uint32_t xn = (uint32_t)n * (uint32_t)E.x_sN;

    // the zero columns of every staged row (4 left, 4 right)
    for (int i = tid; i < MH * R * 8; i += 256) {
        const int row = i >> 3, e = i & 7;
        sT[row * LW + (e < 4 ? e : W + e)] = 0.f;
    }
    // ---- phase A: t[m][r][x] = pre(sum_k W1[m][k] x[k][iy][x] + b1[m]), rows outside the plane 0
    const __attribute__((address_space(4))) f32x2 *w1 = (const __attribute__((address_space(4))) f32x2 *)E.wt;
    for (int p = tid; p < PL; p += 256) {
        const int r = p / W, x = p - r * W, iy = oy0 - 1 + r;
        float t[MH];
        if (iy >= 0 && iy < H) {
            f32x2 acc[MH / 2];
#pragma unroll
            for (int i = 0; i < MH / 2; ++i) acc[i] = (f32x2)(0.f);
            const float *xp = E.x + xn + (uint32_t)(iy * W + x);
#pragma unroll 8
            for (int k = 0; k < C; ++k) {
                const float xv = xp[(uint32_t)k * (uint32_t)E.x_sC];
#pragma unroll
                for (int i = 0; i < MH / 2; ++i)
                    acc[i] = __builtin_elementwise_fma(w1[(k * E.Mpad) / 2 + i], (f32x2)(xv), acc[i]);
            }
#pragma unroll
            for (int i = 0; i < MH / 2; ++i) {
                t[2 * i] = acc[i].x + ldc(E.bias, 2 * i);
                t[2 * i + 1] = acc[i].y + ldc(E.bias, 2 * i + 1);
            }
            apply_act_n<MH>(E.pre, t, [](int m) { return m; });
        } else {
#pragma unroll
            for (int m = 0; m < MH; ++m) t[m] = 0.f;
        }
#pragma unroll
        for (int m = 0; m < MH; ++m) sT[(m * R + r) * LW + 4 + x] = t[m];
    }
    __syncthreads();

    // ---- phase B: output (oy0 + ty, tx): depthwise from LDS, 1x1 into C accumulators
    const int ty = tid / W, tx = tid - ty * W;
    f32x2 acc[C / 2];
#pragma unroll
    for (int i = 0; i < C / 2; ++i) acc[i] = (f32x2)(0.f);
    const __attribute__((address_space(4))) f32x2 *w2 = (const __attribute__((address_space(4))) f32x2 *)G.wt;
#pragma unroll 2
    for (int ch = 0; ch < MH; ++ch) {
        const float *t0 = sT + (ch * R + ty) * LW + 3 + tx;  // tap (0, 0): row ty, column tx - 1
        float d = ldc(D.dw_b, ch);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) d = __builtin_fmaf(ldc(D.dw_w, ch * 9 + ky * 3 + kx), t0[ky * LW + kx], d);
        d = apply_act(D.dw_act, d, ch);
#pragma unroll
        for (int i = 0; i < C / 2; ++i) acc[i] = __builtin_elementwise_fma(w2[(ch * G.Mpad) / 2 + i], (f32x2)(d), acc[i]);
    }
    const int q = (oy0 + ty) * W + tx;
    float v[C];
#pragma unroll
    for (int i = 0; i < C / 2; ++i) {
        v[2 * i] = acc[i].x + ldc(G.bias, 2 * i);
        v[2 * i + 1] = acc[i].y + ldc(G.bias, 2 * i + 1);
    }
    auto chan = [](int m) { return m; };
    apply_act_n<C>(G.pre, v, chan);
    const uint32_t rb = (uint32_t)n * (uint32_t)G.r_sN + (uint32_t)q;
#pragma unroll
    for (int m = 0; m < C; ++m) v[m] += G.r[rb + (uint32_t)m * (uint32_t)G.r_sC];
    apply_act_n<C>(G.post, v, chan);
    const uint32_t ob = (uint32_t)n * (uint32_t)G.o_sN + (uint32_t)q;
#pragma unroll
    for (int m = 0; m < C; ++m) G.out[ob + (uint32_t)m * (uint32_t)G.o_sC] = v[m];
}

template <int C, int W>
const char *bneck_go(const GemmParams &e, const DwPwParams &d, hipStream_t s) {
    constexpr int TR = 256 / W;
    const int bands = d.in.H / TR, nimg = d.g.ncols / d.g.P;
    const int tiles = nimg * bands;
    hipLaunchKernelGGL((bneck_kernel<C, W>), dim3((tiles + 7) / 8 * 8), dim3(256), 0, s, e, d, bands);
    return kernel_name("bneck_kernel<%d,%d>", C, W);
}

}  // namespace

// The fused form applies to a reduction (1x1, C -> C/2, no residual, CNHW input) whose output only
// the next 3x3 stride-1 depthwise -> 1x1 (C/2 -> C) step reads, with that step's residual the
// reduction's input (res_mode 1, every channel), TF-style 'same' padding over a square plane of
// width 128 or 64 (the band holds whole rows), and plain CNHW outputs.
const char *launch_bneck(const GemmParams &e, const DwPwParams &d, hipStream_t s) {
    const int C = e.K, W = d.in.W;
    if (!form_on(FORM_BNECK) || e.KK != 1 || e.res_mode != 0 || e.post.kind != ACT_NONE || e.M * 2 != C ||
        e.M != d.g.K || d.g.M != C || e.out != d.in.p || e.nact != d.g.nact || d.k != 3 || d.stride != 1 ||
        d.pad_t != 1 || d.pad_l != 1 || d.in.H != W || d.OW != W || d.g.P != W * W || e.P != W * W ||
        e.x_sN != e.P || d.in.sN != (int64_t)e.P || d.g.ncols % d.g.P != 0 || e.ncols != d.g.ncols ||
        d.g.o_sP != 1 || d.g.o_sN != d.g.P || d.g.res_mode != 1 || d.g.r != e.x || d.g.r_sN != e.x_sN ||
        d.g.r_sC != e.x_sC || d.g.r_C != C || e.Mpad % 2 != 0 || d.g.Mpad % 2 != 0 ||
        ((uintptr_t)e.wt | (uintptr_t)d.g.wt) % 8 != 0)
        return nullptr;
    if (C == 16 && W == 128) return bneck_go<16, 128>(e, d, s);
    if (C == 32 && W == 64) return bneck_go<32, 64>(e, d, s);
    // (C = 64 at 32^2 measured slower than the two launches: 68-71 vs 52 us at 171 images -- the
    // VALU reduction of 64 channels and 3 waves per SIMD cost more than the saved round trip;
    // profiles/r06_layers/face_landmarks_detector_171_bneck_vs_unfused.txt)
    return nullptr;
}

}  // namespace zr
