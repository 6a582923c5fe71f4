// chain.hip -- a run of low-resolution layers fused into one launch, one workgroup per image,
// every activation in LDS (see ChainParams in zr_kernels.h).
//
// Why: below ~16x16 positions the BlazeBlocks of BlazeFace (16^2 / 8^2, 48-96 channels) and
// FaceMesh (12^2 / 6^2 / 3^2, 128 channels) are tiny GEMMs (M, K <= 128, N <= 256 per image)
// whose per-layer launches spend their time on HBM round trips of activations, barriers and
// tails rather than on arithmetic.  Here an image's whole tensor (<= 128 x 256 f32) stays in
// LDS from layer to layer; HBM sees the entry tensor once and the tensors consumed outside the
// chain once.
//
// Per layer (8 waves, 512 threads):
//   CHAIN_DWPW: per chunk of 16 input channels, every wave computes the depthwise 3x3 outputs of
//     two channels (one channel per wave at a time: the depthwise weights are uniform, scalar
//     loads) from the LDS input into a D buffer [16][positions]; double-buffered, one barrier per
//     chunk.  The 1x1 conv then runs as v_mfma_f32_16x16x4_f32 with B fragments from D and A
//     fragments (the transposed 1x1 weights, [Cin][Mpad]) from the L2-resident weight buffer,
//     prefetched one chunk ahead.
//   CHAIN_PW: the B fragments come straight from the LDS input.
//   Waves own MTW x NTW accumulator tiles of 16x16: wave w takes M group w % MS and N tiles
//   w / MS + (8 / MS) * j.
//   Epilogue (after a barrier: every read of the input is done): bias, activation, residual
//   (+channel pad, +2x2 max-pool), activation -- the order of epilogue.h -- into the output's
//   LDS region (stride-1 layers may overwrite their own input: each element's residual is read
//   by the lane that writes it) and/or a global destination.
// Arithmetic order: the depthwise sum starts at the bias and adds taps in (ky, kx) order with
// fmaf, out-of-image taps as fmaf(w, 0, a); the 1x1 accumulates from 0 in channel order (the
// MFMA is an exact k-ordered fmaf chain) and adds the bias after -- exactly the other dwpw and
// gemm kernels' order, so a chained model is bit-identical to the unchained plan.
// Reference: the Conv/PRelu/Add/Pad/MaxPool nodes ORT/tract run at crates/zaru/src/nn/mod.rs:
// 483-533 for face/detection.rs (BlazeFace) and face/landmark/mediapipe.rs (FaceMesh).
#include <algorithm>

#include "../runtime/zr_kernels.h"
#include "act.h"

namespace zr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int CT = 512, CW = 8, KC = 16;  // threads, waves, input channels per chunk
constexpr int NTWM = 4, MTWM = 4;         // max N / M tiles per wave

__device__ __forceinline__ float act_of(const float *W, const ChainAct &a, float v, int c) {
    switch (a.kind) {
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_CLIP: return fminf(fmaxf(v, a.lo), a.hi);
    case ACT_PRELU: return v < 0.f ? v * ldc(W, a.slope_off + c) : v;
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
    }
}

// depthwise 3x3 outputs of input channels kc .. kc+15 into D buffer `d` ([16][ds])
__device__ __forceinline__ void dw_chunk(const ChainParams &A, const ChainOp &op, const float *lds_in,
                                         float *d, int kc, int wave, int lane) {
    const float *W = A.weights;
    const int NP = op.NT * 16;
    for (int cc = wave; cc < KC; cc += CW) {
        const int c = kc + cc;
        float *drow = d + cc * op.ds;
        if (c >= op.Cin) {
            for (int q = lane; q < NP; q += 64) drow[q] = 0.f;
            continue;
        }
        const float *x = lds_in + c * op.P;
        float w[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) w[t] = ldc(W, op.dw_w_off + c * 9 + t);
        const float b = ldc(W, op.dw_b_off + c);
        const int H = op.P / op.W;
#pragma unroll
        for (int pass = 0; pass < 4; ++pass) {
            const int q = lane + 64 * pass;
            if (q >= NP) break;
            float v = 0.f;
            if (q < op.OP) {
                const int oy = q / op.OW, ox = q - oy * op.OW;
                const int iy0 = oy * op.stride - op.pad_t, ix0 = ox * op.stride - op.pad_l;
                float a = b;
#pragma unroll
                for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                    for (int kx = 0; kx < 3; ++kx) {
                        const int iy = iy0 + ky, ix = ix0 + kx;
                        const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < op.W;
                        const float t = x[ok ? iy * op.W + ix : 0];
                        a = __builtin_fmaf(w[ky * 3 + kx], ok ? t : 0.f, a);
                    }
                v = act_of(W, op.dw_act, a, c);
            }
            drow[q] = v;
        }
    }
}

__device__ void run_op(const ChainParams &A, const ChainOp &op, float *lds, int n, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
    const float *W = A.weights;
    const int ms = wave % op.MS, ng = wave / op.MS, NG = CW / op.MS;
    const int kl = lane >> 4, cl = lane & 15;  // MFMA 16x16x4: A[cl][kl], B[kl][cl]
    const bool dwpw = op.kind == CHAIN_DWPW;
    float *dbuf = lds + A.d_off;
    const float *x = lds + op.in_off;

    f32x4 acc[NTWM][MTWM];
#pragma unroll
    for (int j = 0; j < NTWM; ++j)
#pragma unroll
        for (int t = 0; t < MTWM; ++t) acc[j][t] = (f32x4)(0.f);

    // A fragments of one chunk: [k-step][M tile]
    auto load_a = [&](int kc, float (&a)[4][MTWM]) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < MTWM; ++t) {
                const int k = kc + 4 * s + kl, m = (ms * op.MTW + t) * 16 + cl;
                const bool ok = t < op.MTW && k < op.Cin && m < op.Mpad;
                const float v = ldc(W, op.w_off + (ok ? k * op.Mpad + m : 0));
                a[s][t] = ok ? v : 0.f;
            }
    };

    const int nchunks = (op.Cin + KC - 1) / KC;
    float an[4][MTWM];
    load_a(0, an);
    if (dwpw) {
        dw_chunk(A, op, x, dbuf, 0, wave, lane);
        __syncthreads();
    }
    for (int ch = 0; ch < nchunks; ++ch) {
        const int kc = ch * KC;
        float a[4][MTWM];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < MTWM; ++t) a[s][t] = an[s][t];
        if (ch + 1 < nchunks) {
            load_a(kc + KC, an);
            if (dwpw) dw_chunk(A, op, x, dbuf + ((ch + 1) & 1) * A.d_buf, kc + KC, wave, lane);
        }
        const float *d = dbuf + (ch & 1) * A.d_buf;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            float b[NTWM];
#pragma unroll
            for (int j = 0; j < NTWM; ++j) {
                const int nt = ng + NG * j;
                const int col = nt * 16 + cl;
                if (dwpw) {
                    b[j] = (j < op.NTW && nt < op.NT) ? d[(4 * s + kl) * op.ds + col] : 0.f;
                } else {
                    const int k = kc + 4 * s + kl;
                    const bool ok = j < op.NTW && nt < op.NT && k < op.Cin && col < op.P;
                    const float v = x[ok ? k * op.P + col : 0];
                    b[j] = ok ? v : 0.f;
                }
            }
#pragma unroll
            for (int j = 0; j < NTWM; ++j) {
                if (j >= op.NTW || ng + NG * j >= op.NT) continue;
#pragma unroll
                for (int t = 0; t < MTWM; ++t)
                    if (t < op.MTW) acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][t], b[j], acc[j][t], 0, 0, 0);
            }
        }
        __syncthreads();  // chunk ch+1's depthwise is in place; chunk ch's readers are done
    }

    // epilogue: y = post( pre(acc + bias) + residual ), rows (l >> 4) * 4 + r, column l & 15
    const ChainOut go = op.gout >= 0 ? A.gout[op.gout] : ChainOut{};
    const float *res = lds + (op.res_off >= 0 ? op.res_off : 0);
#pragma unroll
    for (int j = 0; j < NTWM; ++j) {
        const int nt = ng + NG * j;
        if (j >= op.NTW || nt >= op.NT) continue;
        const int q = nt * 16 + cl;
        const bool qok = q < op.OP;
        const int oy = q / op.OW, ox = q - oy * op.OW;
#pragma unroll
        for (int t = 0; t < MTWM; ++t) {
            if (t >= op.MTW) continue;
            const int m0 = (ms * op.MTW + t) * 16 + kl * 4;
            float v[4], rv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + r;
                v[r] = acc[j][t][r] + ldc(W, op.b_off + (m < op.Mpad ? m : 0));
                rv[r] = 0.f;
                if (op.res_mode == 1) {
                    const float x1 = res[(m < op.r_C && qok) ? m * op.res_P + q : 0];
                    rv[r] = (m < op.r_C && qok) ? x1 : 0.f;
                } else if (op.res_mode == 2) {
                    const int o = (m < op.r_C && qok) ? m * op.res_P + (2 * oy) * op.res_W + 2 * ox : 0;
                    const float p = fmaxf(fmaxf(res[o], res[o + 1]), fmaxf(res[o + op.res_W], res[o + op.res_W + 1]));
                    rv[r] = (m < op.r_C && qok) ? p : 0.f;
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + r;
                const int mc = m < op.Mpad ? m : 0;
                float y = act_of(W, op.pre, v[r], mc);
                if (op.res_mode != 0) y += rv[r];
                y = act_of(W, op.post, y, mc);
                if (qok && m < op.Cout) {
                    if (op.out_off >= 0) lds[op.out_off + m * op.OP + q] = y;
                    if (op.gout >= 0) go.p[(int64_t)n * go.sN + (int64_t)m * go.sC + (int64_t)q * go.sP] = y;
                }
            }
        }
    }
}

__global__ __launch_bounds__(CT) void chain_kernel(const ChainParams A) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int n = blockIdx.x, tid = threadIdx.x;
    // the entry tensor of this image: e_C channel runs of e_P contiguous floats (e_P % 4 == 0)
    {
        const float *src = A.entry + (int64_t)n * A.e_sN;
        const int total = A.e_C * A.e_P;
        for (int i = 4 * tid; i < total; i += 4 * CT) {
            const int c = i / A.e_P, p = i - c * A.e_P;
            *(float4 *)(lds + A.e_off + i) = *(const float4 *)(src + (int64_t)c * A.e_sC + p);
        }
    }
    __syncthreads();
    constexpr int WORDS = sizeof(ChainOp) / 4;
    const __attribute__((address_space(4))) int *tab =
        (const __attribute__((address_space(4))) int *)(A.weights + A.ops_off);
    for (int o = 0; o < A.nops; ++o) {
        ChainOp op;  // uniform: scalar loads of the op's table words
        int *w = (int *)&op;
#pragma unroll
        for (int i = 0; i < WORDS; ++i) w[i] = tab[o * WORDS + i];
        run_op(A, op, lds, n, tid);
        __syncthreads();  // this layer's outputs are visible to the next
    }
}

}  // namespace

const char *launch_chain(const ChainParams &p, hipStream_t s) {
    hipLaunchKernelGGL(chain_kernel, dim3(p.N), dim3(CT), sizeof(float) * (size_t)p.lds_floats, s, p);
    return "chain_kernel";
}

}  // namespace zr
