// ir.hip -- the MobileNetV2 inverted residual (expand 1x1 -> depthwise KxK -> project 1x1, with
// the block's residual) in one launch, so the expanded tensor (4-6x the block's channels, the
// hand landmark network's 64 x 112^2 / 96 x 56^2 / 144 x 28^2 planes) never reaches HBM.
// Reference: the Conv nodes of hand_landmark_lite.onnx executed by ORT/tract at
// crates/zaru/src/nn/mod.rs:483-533 (hand/landmark.rs:251-322).
//
// One workgroup per TH x TW output tile of one image, one thread per output position.  Per
// chunk of VF expanded channels:
//   1. each thread computes the expanded values of its share of the tile's input footprint
//      ((TH-1)*S+K rows x (TW-1)*S+K columns) from the block input it holds in registers (all
//      Cx channels of its footprint positions, loaded once per tile), the expand weights
//      coming through the scalar cache; zero outside the plane (the depthwise's padding);
//   2. one barrier publishes the chunk (double-buffered LDS);
//   3. each thread runs the depthwise of its output position over the chunk from LDS and
//      accumulates the projection into CO registers (packed FMA).
// Epilogue: bias, activation, residual (+channel pad, +2x2 max-pool), activation, one store per
// channel.  Arithmetic and order are those of the unfused launches -- the expand as an fmaf
// chain over its K in order (= the f32 MFMA), + bias, activation; the depthwise and projection
// as dwpw_valu_kernel -- so fusing changes no output bit (tests/test_gpu_forms.py "ir").
// Opt-in (ZARU_HIP_FORMS=+ir): the VALU expand makes it a wash on the hand pipeline.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "../runtime/zr_kernels.h"
#include "act.h"

namespace zr {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int IR_VF = 4;     // expanded channels per chunk
constexpr int IR_EPT = 5;    // footprint positions per thread (at most; stride 1 tiles need 2)
constexpr int IR_XMAX = 24;  // block-input channels held in registers

template <int K, int S, int CO, int CX>
__global__ __launch_bounds__(256) void ir_kernel(const IrParams P) {
    constexpr int EPT = S == 1 ? 2 : IR_EPT;
    // LDS: [2][VF][EH][EW] expanded chunks | expand weights [Ce][CX] (transposed) + bias [Ce] |
    // depthwise weights [Ce][K*K] + bias [Ce] | projection weights [Ce][CO]
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const GemmParams &E = P.e;   // expand: x = block input, M = Ce, K = Cx
    const GemmParams &G = P.d.g; // project: K = Ce, M = Cout
    const int TH = P.th, TW = P.tw, EH = (TH - 1) * S + K, EW = (TW - 1) * S + K, NE = EH * EW;
    const int tid = threadIdx.x, n = blockIdx.y;
    const int ty0 = (blockIdx.x / P.tiles_x) * TH, tx0 = (blockIdx.x % P.tiles_x) * TW;
    const int H = P.d.in.H, W = P.d.in.W, OW = P.d.OW, OH = G.P / P.d.OW;
    const int ey0 = ty0 * S - P.d.pad_t, ex0 = tx0 * S - P.d.pad_l;  // footprint origin in the plane
    const int Ce = G.K, Cep = (Ce + IR_VF - 1) / IR_VF * IR_VF;
    constexpr int KK = K * K;
    float *sE = lds, *sW1 = sE + 2 * IR_VF * NE, *sB1 = sW1 + Cep * CX, *sDW = sB1 + Cep, *sDB = sDW + Cep * KK,
          *sW2 = sDB + Cep;

    // the layer's parameters, once per workgroup (zero past Ce / Cx)
    for (int i = tid; i < Cep * CX; i += 256) {
        const int c = i / CX, k = i - c * CX;
        sW1[i] = c < Ce && k < E.K ? E.wt[k * E.Mpad + c] : 0.f;
    }
    for (int i = tid; i < Cep * KK; i += 256) sDW[i] = i < Ce * KK ? P.d.dw_w[i] : 0.f;
    for (int i = tid; i < Cep; i += 256) {
        sB1[i] = i < Ce ? E.bias[i] : 0.f;
        sDB[i] = i < Ce ? P.d.dw_b[i] : 0.f;
    }
    for (int i = tid; i < Cep * CO; i += 256) {
        const int c = i / CO, m = i - c * CO;
        sW2[i] = c < Ce && m < G.Mpad ? G.wt[(size_t)c * G.Mpad + m] : 0.f;
    }

    // this thread's footprint positions and the block input there (all CX channels)
    float x[EPT][CX];
    bool inb[EPT];
    int epos[EPT];
    const float *xb = E.x + (int64_t)n * E.x_sN;
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
        const int e = tid + 256 * u;
        const int r = e / EW, c = e - r * EW;
        const int iy = ey0 + r, ix = ex0 + c;
        inb[u] = e < NE && iy >= 0 && iy < H && ix >= 0 && ix < W;
        epos[u] = e < NE ? e : -1;
        const int off = inb[u] ? iy * W + ix : 0;
#pragma unroll
        for (int k = 0; k < CX; ++k) {
            const float v = xb[(int64_t)(k < E.K ? k : 0) * E.x_sC + off];
            x[u][k] = inb[u] && k < E.K ? v : 0.f;
        }
    }
    __syncthreads();  // parameters staged

    // output position of this thread
    const int ty = tid / TW, tx = tid - ty * TW;
    const int oy = ty0 + ty, ox = tx0 + tx;
    const bool active = tid < TH * TW && oy < OH && ox < OW;
    const int tb = (ty * S) * EW + tx * S;  // footprint index of tap (0, 0)
    const int Kx = E.K;

    f32x2 acc[CO / 2];
#pragma unroll
    for (int i = 0; i < CO / 2; ++i) acc[i] = (f32x2)(0.f);

    for (int c0 = 0, it = 0; c0 < Ce; c0 += IR_VF, ++it) {
        float *buf = sE + (it & 1) * IR_VF * NE;
        // 1. expanded values of this chunk at this thread's footprint positions: an fmaf chain over
        // k in order from 0 (= the f32 MFMA of the unfused expand), + bias, activations
#pragma unroll
        for (int cc = 0; cc < IR_VF; ++cc) {
            const int c = c0 + cc;
            const float4 *w4 = reinterpret_cast<const float4 *>(sW1 + c * CX);
            float w[CX];
#pragma unroll
            for (int k4 = 0; k4 < CX / 4; ++k4) {
                const float4 q = w4[k4];
                w[4 * k4] = q.x;
                w[4 * k4 + 1] = q.y;
                w[4 * k4 + 2] = q.z;
                w[4 * k4 + 3] = q.w;
            }
            float a[EPT];
#pragma unroll
            for (int u = 0; u < EPT; ++u) a[u] = 0.f;
#pragma unroll
            for (int k = 0; k < CX; ++k) {
                if (k < Kx) {
#pragma unroll
                    for (int u = 0; u < EPT; ++u) a[u] = __builtin_fmaf(w[k], x[u][k], a[u]);
                }
            }
            const float b = sB1[c];
#pragma unroll
            for (int u = 0; u < EPT; ++u) a[u] = a[u] + b;
            const int cl = min(c, Ce - 1);
            apply_act_n<EPT>(E.pre, a, [&](int) { return cl; });
            apply_act_n<EPT>(E.post, a, [&](int) { return cl; });
#pragma unroll
            for (int u = 0; u < EPT; ++u)
                if (epos[u] >= 0) buf[cc * NE + epos[u]] = inb[u] ? a[u] : 0.f;
        }
        __syncthreads();  // the chunk is published; the other buffer's readers are done
        // 2. depthwise of this output position over the chunk, into the projection
        if (active) {
            float dv[IR_VF];
#pragma unroll
            for (int cc = 0; cc < IR_VF; ++cc) {
                const int ch = c0 + cc;
                const float *t0 = buf + cc * NE + tb;
                const float *w = sDW + ch * KK;
                float d = sDB[ch];
#pragma unroll
                for (int ky = 0; ky < K; ++ky)
#pragma unroll
                    for (int kx = 0; kx < K; ++kx) d = __builtin_fmaf(w[ky * K + kx], t0[ky * EW + kx], d);
                dv[cc] = d;
            }
            apply_act_n<IR_VF>(P.d.dw_act, dv, [&](int cc) { return min(c0 + cc, Ce - 1); });
#pragma unroll
            for (int cc = 0; cc < IR_VF; ++cc) {
                if (c0 + cc >= Ce) continue;
                const f32x2 *w2 = reinterpret_cast<const f32x2 *>(sW2 + (c0 + cc) * CO);
#pragma unroll
                for (int i = 0; i < CO / 2; ++i) acc[i] = __builtin_elementwise_fma(w2[i], (f32x2)(dv[cc]), acc[i]);
            }
        }
    }

    if (!active) return;
    const int q = oy * OW + ox;
    float v[CO];
#pragma unroll
    for (int i = 0; i < CO / 2; ++i) {
        v[2 * i] = acc[i].x + G.bias[2 * i];
        v[2 * i + 1] = acc[i].y + G.bias[2 * i + 1];
    }
    float rv[CO];
    if (G.res_mode == 1) {
        const uint32_t rb = (uint32_t)n * (uint32_t)G.r_sN + (uint32_t)q;
#pragma unroll
        for (int m = 0; m < CO; ++m) {
            const float r = G.r[rb + (uint32_t)(m < G.r_C ? m : 0) * (uint32_t)G.r_sC];
            rv[m] = m < G.r_C ? r : 0.f;
        }
    } else if (G.res_mode == 2) {
        const uint32_t rb = (uint32_t)n * (uint32_t)G.r_sN + (uint32_t)((2 * oy) * G.r_W + 2 * ox);
#pragma unroll
        for (int m = 0; m < CO; ++m) {
            const uint32_t o = rb + (uint32_t)(m < G.r_C ? m : 0) * (uint32_t)G.r_sC;
            const float p = fmaxf(fmaxf(G.r[o], G.r[o + 1]), fmaxf(G.r[o + G.r_W], G.r[o + G.r_W + 1]));
            rv[m] = m < G.r_C ? p : 0.f;
        }
    }
    auto chan = [](int m) { return m; };
    apply_act_n<CO>(G.pre, v, chan);
    if (G.res_mode != 0) {
#pragma unroll
        for (int m = 0; m < CO; ++m) v[m] += rv[m];
    }
    apply_act_n<CO>(G.post, v, chan);
    const uint32_t ob = (uint32_t)n * (uint32_t)G.o_sN + (uint32_t)q * (uint32_t)G.o_sP;
#pragma unroll
    for (int m = 0; m < CO; ++m)
        if (m < G.M) G.out[ob + (uint32_t)m * (uint32_t)G.o_sC] = v[m];
}

namespace {

template <int K, int S, int CO, int CX>
const char *ir_go(IrParams p, hipStream_t s) {
    const int EH = (p.th - 1) * S + K, EW = (p.tw - 1) * S + K;
    const int Cep = (p.d.g.K + IR_VF - 1) / IR_VF * IR_VF;
    const size_t lds = sizeof(float) * (2 * IR_VF * (size_t)EH * EW + (size_t)Cep * (CX + 1 + K * K + 1 + CO));
    hipLaunchKernelGGL((ir_kernel<K, S, CO, CX>), dim3(p.tiles_x * p.tiles_y, p.d.g.ncols / p.d.g.P), dim3(256),
                       lds, s, p);
    return kernel_name("ir_kernel<%d,%d,%d,%d>", K, S, CO, CX);
}

template <int K, int S, int CO>
const char *ir_cx(const IrParams &p, hipStream_t s) {
    if (p.e.K <= 16) return ir_go<K, S, CO, 16>(p, s);
    return ir_go<K, S, CO, 24>(p, s);
}

template <int K, int S>
const char *ir_co(const IrParams &p, hipStream_t s) {
    if (p.d.g.M <= 16) return ir_cx<K, S, 16>(p, s);
    if (p.d.g.M <= 24) return ir_cx<K, S, 24>(p, s);
    return ir_cx<K, S, 48>(p, s);
}

}  // namespace

static bool ir_everywhere() {  // ZARU_HIP_IR_ALL=1: fuse every eligible block (A/B runs)
    static const bool v = [] {
        const char *e = std::getenv("ZARU_HIP_IR_ALL");
        return e && e[0] == '1';
    }();
    return v;
}

// The fused block applies when the expand is a plain 1x1 over a CNHW input of <= 32 channels
// with no residual, the projection has <= 48 outputs, the depthwise is 3x3 / 5x5 at stride 1 / 2,
// and a tile's footprint fits IR_EPT positions per thread (host-chosen tile, below).
const char *launch_ir(IrParams p, hipStream_t s) {
    const GemmParams &e = p.e, &g = p.d.g;
    const int k = p.d.k, st = p.d.stride;
    if (!form_on(FORM_IR) || e.KK != 1 || e.res_mode != 0 || e.K > IR_XMAX || e.K < 1 || g.M > 48 ||
        (k != 3 && k != 5) || (st != 1 && st != 2) || e.M != g.K || g.P <= 0 || g.ncols % g.P != 0 ||
        e.x_sN != (int64_t)p.d.in.H * p.d.in.W || e.P != (int64_t)p.d.in.H * p.d.in.W ||
        p.d.g.ncols / g.P > 65535)
        return nullptr;
    // Measured (hand landmark, 1024 ROIs): the expand runs on the VALU here but on the
    // f32 MFMA unfused, so fusing wins only where the expanded tensor's HBM round trip dominates --
    // the 112^2 block (64 x 112^2, 2.00 vs 2.19 ms); at 56^2 / 28^2 it loses (1.47 vs 0.97 ms).
    if ((int64_t)p.d.in.H * p.d.in.W < 112 * 112 && !ir_everywhere()) return nullptr;
    // tile: the TH x TW (<= 256 threads) with the least expand work (footprint positions) plus
    // idle-thread cost per useful output
    const int OW = p.d.OW, OH = g.P / OW;
    double best = 1e30;
    for (int tw = 1; tw <= std::min(OW, 256); ++tw)
        for (int th = 1; th <= std::min(256 / tw, OH); ++th) {
            if (th * tw < 128) continue;
            const int eh = (th - 1) * st + k, ew = (tw - 1) * st + k;
            if (eh * ew > 256 * (st == 1 ? 2 : IR_EPT)) continue;
            const int tx = (OW + tw - 1) / tw, ty = (OH + th - 1) / th;
            const double cost = ((double)eh * ew + 0.5 * 256.0) * tx * ty / ((double)OW * OH);
            if (cost < best) {
                best = cost;
                p.th = th;
                p.tw = tw;
                p.tiles_x = tx;
                p.tiles_y = ty;
            }
        }
    if (best >= 1e30) return nullptr;
    if (k == 3) return st == 1 ? ir_co<3, 1>(p, s) : ir_co<3, 2>(p, s);
    return st == 1 ? ir_co<5, 1>(p, s) : ir_co<5, 2>(p, s);
}

}  // namespace zr
