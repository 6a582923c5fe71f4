// ir.hip -- the MobileNetV2 inverted residual of the hand landmark network's high-resolution
// blocks (expand 1x1 -> depthwise KxK -> project 1x1, + the block's residual) in one launch, so
// the expanded tensor (64 x 112^2 / 96 x 56^2 floats per image, 4-6x the block's own channels)
// never reaches HBM.  Reference: the Conv / Clip / Add nodes of hand_landmark_lite.onnx that ORT /
// tract execute at crates/zaru/src/nn/mod.rs:483-533 (hand/landmark.rs:251-322; SURVEY.md
// Appendix A).
//
// A workgroup owns an 8 x 32 tile of outputs of one image (one thread per output).  Per chunk of 16
// expanded channels:
//   1. expand on f32 MFMA (v_mfma_f32_16x16x4f32): the chunk's 16 channels x the tile's input
//      footprint ((8-1)S+K x (32-1)S+K positions, 16-position column tiles dealt to the 4 waves),
//      the block input (16 channels) held in registers for the whole launch, the chunk's expand
//      weights as the A operand; + bias, activation; positions outside the plane are stored as 0
//      (the depthwise's zero padding) into LDS.  Each column tile's 4-MFMA chain is issued before
//      the previous tile's epilogue, so the VALU epilogue covers the chain's latency;
//   2. each thread's depthwise over the chunk from LDS, accumulated into the projection (packed
//      FMA, the weights through the scalar cache).
// Epilogue: bias, activation, residual (direct or 2x2 max-pool), activation, one store per channel.
// The residual is the block input, already in registers for the expand: it is staged once
// through LDS before the first chunk, so no second HBM read of it.  The expand and depthwise
// activations must be Relu / Clip / none (the hand network's Clip(0, 6)), applied as bounds.
//
// Arithmetic and order are the unfused launches': the expand is the f32 MFMA chain over k in
// order (16x16x4 and 32x32x2 sum each output's products in k order like an fmaf chain --
// tools/debug/mfma_order.hip, profiles/r04_mfma_order_probe.json) then + bias and the activations
// (gemm_tiled_kernel's epilogue); the depthwise and projection are dwpw_valu_kernel's.  So fusing
// changes no output bit (tests/test_gpu_forms.py, -ir).  The round-3 form of this fusion computed
// the expand on the VALU and measured a wash; the MFMA expand is the difference.
#include <algorithm>

#include "../runtime/zr_kernels.h"
#include "act.h"

namespace zr {

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int IR_TH = 8, IR_TW = 32;  // output tile, one thread per output
constexpr int IR_CEC = 16;            // expanded channels per chunk (the MFMA's 16 rows)
constexpr int IR_CX = 16;
#ifndef IR_DWU
#define IR_DWU 2
#endif             // block-input channels (the MFMA's K: four 16x16x4 steps)

template <int K, int S> constexpr int ir_fp() { return ((IR_TH - 1) * S + K) * ((IR_TW - 1) * S + K); }
// LDS row of the expanded footprint: at stride 2 the even and odd columns are stored as two
// half rows, so the depthwise's stride-2 taps of adjacent threads hit adjacent banks
template <int K, int S> constexpr int ir_lrow() {
    return S == 2 ? 2 * (((IR_TW - 1) * S + K + 1) / 2) : (IR_TW - 1) * S + K;
}
template <int K, int S> constexpr int ir_npw() { return ((ir_fp<K, S>() + 15) / 16 + 3) / 4; }


// E: the expand GEMM (x = block input, K = 16, M = Ce); D: the depthwise + projection step
// (D.g.K = Ce, D.g.M = Cout <= CO, residual = the block input or its 2x2 max-pool)
template <int K, int S, int CO>
__global__ __launch_bounds__(256) void ir_kernel(const GemmParams E, const DwPwParams D, int tiles_x) {
    constexpr int PL = S == 1 ? K / 2 : K / 2 - 1;  // TF-style pads (host-checked)
    constexpr int FH = (IR_TH - 1) * S + K, FW = (IR_TW - 1) * S + K, FP = FH * FW;
    constexpr int NPT = (FP + 15) / 16, NPW = ir_npw<K, S>();
    constexpr int LR = ir_lrow<K, S>(), LH = LR / 2, LP = FH * LR;  // LDS row, half row, plane
    extern __shared__ __attribute__((aligned(16))) float sE[];  // [IR_CEC][FH][LR]
    const GemmParams &G = D.g;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int col = lane & 15, kq = lane >> 4;
    const int n = blockIdx.y;
    if (G.nact && n >= *G.nact) return;  // (whole workgroup, before any barrier)
    const int ty0 = (blockIdx.x / tiles_x) * IR_TH, tx0 = (blockIdx.x % tiles_x) * IR_TW;
    const int H = D.in.H, W = D.in.W, OW = D.OW, OH = G.P / D.OW, Ce = E.M;
    const int fy0 = ty0 * S - PL, fx0 = tx0 * S - PL;  // footprint origin in the input plane

    // the block input at this lane's footprint positions (B operands: k = 4 s + kq), for every chunk
    float xr[NPW][4];
    uint32_t inb = 0;  // bit i: footprint column tile i of this wave, this lane's position in the plane
    const float *xb = E.x + (size_t)(uint32_t)n * (uint32_t)E.x_sN;
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
        const int p = (wave * NPW + i) * 16 + col;
        const int r = p / FW, c = p - r * FW;
        const int iy = fy0 + r, ix = fx0 + c;
        const bool ok = p < FP && iy >= 0 && iy < H && ix >= 0 && ix < W;
        inb |= (ok ? 1u : 0u) << i;
        const uint32_t off = ok ? (uint32_t)(iy * W + ix) : 0u;
#pragma unroll
        for (int s = 0; s < 4; ++s) xr[i][s] = xb[(uint32_t)(4 * s + kq) * (uint32_t)E.x_sC + off];
    }

    // this thread's output
    const int ty = tid / IR_TW, tx = tid - ty * IR_TW;
    const int oy = ty0 + ty, ox = tx0 + tx;
    const bool active = oy < OH && ox < OW;
    const int tb = (ty * S) * LR + tx;  // LDS index of tap (0, 0) (stride 2: the even half row)
    f32x2 acc[CO / 2];
#pragma unroll
    for (int i = 0; i < CO / 2; ++i) acc[i] = (f32x2)(0.f);

    // the block's residual (its input at this output, or the 2x2 max-pool of it) from the footprint
    // already in registers: staged once through LDS, so the epilogue reads no HBM for it
    float rx[IR_CX];
    if (G.res_mode != 0) {
#pragma unroll
        for (int i = 0; i < NPW; ++i) {
            const int p = (wave * NPW + i) * 16 + col;
            const int pr = p / FW, pc = p - pr * FW;
            const int lp = pr * LR + (S == 2 ? (pc & 1) * LH + (pc >> 1) : pc);
            if (p < FP) {
#pragma unroll
                for (int s = 0; s < 4; ++s) sE[(4 * s + kq) * LP + lp] = xr[i][s];
            }
        }
        __syncthreads();
        if (active) {
            if (S == 1) {  // res_mode 1 (host-checked): the centre tap
                const int l = (ty + PL) * LR + tx + PL;
#pragma unroll
                for (int m = 0; m < IR_CX; ++m) rx[m] = sE[m * LP + l];
            } else {  // res_mode 2, PL = 0: footprint (2ty + dy, 2tx + dx), the odd column in the odd half row
                const int l = 2 * ty * LR + tx;
#pragma unroll
                for (int m = 0; m < IR_CX; ++m) {
                    const float *e = sE + m * LP + l;
                    rx[m] = fmaxf(fmaxf(e[0], e[LH]), fmaxf(e[LR], e[LR + LH]));
                }
            }
        }
        __syncthreads();  // before the first chunk overwrites the staged input
    }

    const Bounds eb = bounds(E.pre), db = bounds(D.dw_act);  // (E.post: none, host-checked)
    // expand operands of a chunk: A[m][k] = W1[c0 + m][k] from the transposed [Kpad][Mpad]
    // weights, and the biases (c0 < Ce: host-checked Ce % 16 == 0; clamped past the end).  Loaded
    // a chunk ahead: loaded in the chunk that uses them, every chunk waited a memory latency.
    auto load_ab = [&](int c0, float (&aa)[4], float (&bb)[4]) {
        c0 = c0 < Ce ? c0 : Ce - IR_CEC;
#pragma unroll
        for (int s = 0; s < 4; ++s) aa[s] = E.wt[(uint32_t)(4 * s + kq) * (uint32_t)E.Mpad + (uint32_t)(c0 + col)];
#pragma unroll
        for (int r = 0; r < 4; ++r) bb[r] = E.bias[c0 + 4 * kq + r];
    };
    float a[4], bias[4];
    load_ab(0, a, bias);
    for (int c0 = 0; c0 < Ce; c0 += IR_CEC) {
        // 1. expand
        float an[4], bn[4];
        load_ab(c0 + IR_CEC, an, bn);
        // each column tile's MFMA chain is issued before the previous tile's epilogue, so the
        // epilogue's VALU work covers the chain's latency
        auto chain = [&](int i) {
            f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 4; ++s) d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], xr[i][s], d, 0, 0, 0);
            return d;
        };
        // gemm_tiled_kernel's epilogue (RES = false): + bias, pre act, post act
        auto epi = [&](int i, const f32x4 &d) {
            const int p = (wave * NPW + i) * 16 + col;
            const bool live = (inb >> i) & 1u;
            const int pr = p / FW, pc = p - pr * FW;
            const int lp = pr * LR + (S == 2 ? (pc & 1) * LH + (pc >> 1) : pc);
            if (p < FP) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = clamp(eb, d[r] + bias[r]);
                    sE[(4 * kq + r) * LP + lp] = live ? v : 0.f;
                }
            }
        };
        f32x4 dc = chain(0);  // (tile 0 of every wave is inside the footprint: 3 NPW < NPT)
#pragma unroll
        for (int i = 0; i < NPW; ++i) {
            f32x4 dn = dc;
            if (i + 1 < NPW) dn = chain(i + 1);
            if (wave * NPW + i < NPT) epi(i, dc);  // (wave-uniform)
            dc = dn;
        }
        __syncthreads();  // the chunk is in LDS
        // 2. depthwise + projection (dwpw_valu_kernel's arithmetic)
        if (active) {
#pragma unroll IR_DWU
            for (int cc = 0; cc < IR_CEC; ++cc) {
                const int ch = c0 + cc;
                const float *t0 = sE + cc * LP + tb;
                const float *w = D.dw_w + ch * (K * K);
                float dd = ldc(D.dw_b, ch);
#pragma unroll
                for (int ky = 0; ky < K; ++ky)
#pragma unroll
                    for (int kx = 0; kx < K; ++kx) {
                        const int lx = S == 2 ? (kx & 1) * LH + (kx >> 1) : kx;
                        dd = __builtin_fmaf(ldc(w, ky * K + kx), t0[ky * LR + lx], dd);
                    }
                dd = clamp(db, dd);
                const __attribute__((address_space(4))) f32x2 *w2 =
                    (const __attribute__((address_space(4))) f32x2 *)(G.wt + (size_t)ch * G.Mpad);  // [Kpad][Mpad]
#pragma unroll
                for (int i = 0; i < CO / 2; ++i) acc[i] = __builtin_elementwise_fma(w2[i], (f32x2)(dd), acc[i]);
            }
        }
        __syncthreads();  // the chunk's readers are done
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            a[s] = an[s];
            bias[s] = bn[s];
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
#pragma unroll
    for (int m = 0; m < CO; ++m) rv[m] = m < IR_CX && m < G.r_C ? rx[m < IR_CX ? m : 0] : 0.f;
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

template <int K, int S, int CO>
const char *ir_go(const GemmParams &e, const DwPwParams &d, hipStream_t s) {
    constexpr int LP = ((IR_TH - 1) * S + K) * ir_lrow<K, S>();
    const size_t lds = sizeof(float) * IR_CEC * LP;
    static const bool attr = [] {
        if (hipFuncSetAttribute((const void *)ir_kernel<K, S, CO>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) == hipSuccess)
            return true;
        (void)hipGetLastError();  // handled: the pair then runs unfused
        return false;
    }();
    if (!attr) return nullptr;
    const int OH = d.g.P / d.OW, tiles_x = (d.OW + IR_TW - 1) / IR_TW, tiles_y = (OH + IR_TH - 1) / IR_TH;
    const int N = d.g.ncols / d.g.P;
    hipLaunchKernelGGL((ir_kernel<K, S, CO>), dim3(tiles_x * tiles_y, N), dim3(256), lds, s, e, d, tiles_x);
    return kernel_name("ir_kernel<%d,%d,%d>", K, S, CO);
}

}  // namespace

// The fused form applies to an expand (1x1, 16 input channels, no residual, CNHW input) whose
// output only the next depthwise -> 1x1 step reads (plan.cpp mark_inverted_residuals), with the
// models' TF-style pads, W = OW * S, <= 32 output channels and the 3x3 s1 / s2 and 5x5 s2 shapes of
// the hand network's 112^2 and 56^2 blocks.
const char *launch_ir(const GemmParams &e, const DwPwParams &d, hipStream_t s) {
    if (!form_on(FORM_IR) || e.K != IR_CX || e.KK != 1 || e.res_mode != 0 || e.x_sN != e.P || e.M != d.g.K ||
        e.out != d.in.p || d.in.sN != (int64_t)d.in.H * d.in.W || d.g.M > 32 || d.g.o_sP != 1 ||
        d.in.W != d.OW * d.stride || d.g.ncols % d.g.P != 0 || e.ncols != d.in.H * d.in.W * (d.g.ncols / d.g.P) ||
        e.nact != d.g.nact || e.M % IR_CEC != 0)
        return nullptr;
    // the activations the kernel applies as bounds (the hand network's Clip(0, 6))
    for (const Act *a : {&e.pre, &d.dw_act})
        if (a->kind != ACT_NONE && a->kind != ACT_RELU && a->kind != ACT_CLIP) return nullptr;
    if (e.post.kind != ACT_NONE) return nullptr;
    const int pl = d.stride == 1 ? d.k / 2 : d.k / 2 - 1;
    if (d.pad_t != pl || d.pad_l != pl) return nullptr;
    // the residual is the block input itself (staged from the expand's registers)
    if (d.g.res_mode != 0 && (d.g.r != e.x || d.g.r_C > IR_CX || d.g.r_sC != e.x_sC || d.g.r_sN != e.x_sN))
        return nullptr;
    if (d.g.res_mode == 1 && d.stride != 1) return nullptr;
    // the max-pool shortcut is read at footprint (2ty, 2tx): input (2ty, 2tx) only when the
    // footprint starts at the input's origin, i.e. the depthwise pad is 0 (3x3 s2); a 5x5 s2 block
    // with a pooled shortcut (pad 1) runs unfused
    if (d.g.res_mode == 2 && (d.stride != 2 || pl != 0 || d.g.r_W != d.in.W)) return nullptr;
    const bool co16 = d.g.M <= 16;
    if (d.k == 3 && d.stride == 1) return co16 ? ir_go<3, 1, 16>(e, d, s) : ir_go<3, 1, 32>(e, d, s);
    if (d.k == 3 && d.stride == 2) return co16 ? ir_go<3, 2, 16>(e, d, s) : ir_go<3, 2, 32>(e, d, s);
    // 5x5 s2 (56^2 -> 28^2): one workgroup per CU (83 KB of LDS), still 328 vs 352 us unfused at
    // 341 ROIs (profiles/r05_layers/hand_landmark_lite_341_ir5_vs_unfused.txt)
    if (d.k == 5 && d.stride == 2) return co16 ? ir_go<5, 2, 16>(e, d, s) : ir_go<5, 2, 32>(e, d, s);
    return nullptr;
}

}  // namespace zr
