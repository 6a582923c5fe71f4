// chain.hip -- a run of low-resolution layers fused into one launch, one workgroup per image,
// every activation in LDS (see ChainParams in zr_kernels.h).
//
// Why: below ~16x16 positions the BlazeBlocks of BlazeFace (16^2 / 8^2, 48-96 channels) and
// FaceMesh (12^2 / 6^2 / 3^2, 128 channels) are tiny GEMMs (M, K <= 128, N <= 256 per image)
// whose per-layer launches spend their time on HBM round trips of activations, barriers and
// tails rather than on arithmetic.  Here an image's tensors stay in LDS from layer to layer; HBM
// sees the entry tensor once and the tensors consumed outside the chain once.
//
// Roles (512 threads): waves 0-3 are consumers, waves 4-7 producers.  Per chunk of 16 input
// channels of a depthwise 3x3 -> 1x1 layer, the producers compute the depthwise outputs of
// chunk c+1 into one D buffer ([16][positions]) while the consumers run chunk c's 1x1 conv as
// v_mfma_f32_16x16x4_f32 from the other (B fragments from D, A fragments = the transposed 1x1
// weights, zero-padded to 16-row chunks, from the L2-resident weight buffer, loaded a chunk
// ahead); one barrier per chunk.  So the depthwise VALU work and the matrix work overlap on
// every SIMD instead of taking turns.  A plain 1x1 layer reads its B fragments from the input.
// LDS planes keep a one-cell zero border, so a depthwise tap is one ds_read, no bounds test.
// Consumer wave w owns MTW x NTW 16x16 accumulator tiles: M group w % MS, N tiles
// w / MS + (4 / MS) * j.  Epilogue in two phases around a barrier: (1) bias, activation,
// residual (+channel pad, +2x2 max-pool), activation -- the order of epilogue.h -- in registers;
// (2) stores into the output's LDS planes and/or a global destination, so a layer may overwrite
// the input it consumes, at any stride.
// Arithmetic order: the depthwise sum starts at the bias and adds the taps in (ky, kx) order
// with fmaf (a tap in the zero border adds fmaf(w, 0, a)); the 1x1 accumulates from 0 in channel
// order (the MFMA is an exact k-ordered fmaf chain) and adds the bias after -- exactly the other
// dwpw and gemm kernels' order, so a chained model is bit-identical to the unchained plan.
// Reference: the Conv/PRelu/Add/Pad/MaxPool nodes ORT/tract run at crates/zaru/src/nn/mod.rs:
// 483-533 for face/detection.rs (BlazeFace) and face/landmark/mediapipe.rs (FaceMesh).
#include <algorithm>

#include "../runtime/zr_kernels.h"
#include "act.h"

namespace zr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int CT = 1024, KC = 16, NCW = CHAIN_CONSUMER_WAVES;  // threads, channels per chunk, consumer waves
typedef const __attribute__((address_space(4))) ChainOp cop;

// Workgroup barrier for LDS hand-offs only: this wave's LDS accesses complete, then s_barrier.
// (__syncthreads() would also drain every outstanding global load -- the 1x1 weights loaded a
// chunk ahead -- at each of the ~100 barriers of a chain.)  Global results are only stored,
// never re-read inside the kernel.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Per-layer parameters staged in LDS (the producers' depthwise weights and the epilogue's bias
// and slopes become LDS reads), double-buffered across layers:
//   [0, Mpad) bias | [Mpad, 2 Mpad) pre slope | [2 Mpad, 3 Mpad) post slope |
//   [3 Mpad + 12 c, +12) depthwise channel c: 9 weights, bias, PReLU slope, 0
constexpr int PRM_PER_THREAD = 2;  // 3 * 128 + 12 * 128 parameters at most over 1024 threads

__device__ __forceinline__ int param_src(cop *op, int i) {
    const int Mpad = op->Mpad;
    if (i < Mpad) return op->b_off + i;
    if (i < 2 * Mpad) return op->pre.kind == ACT_PRELU ? op->pre.slope_off + i - Mpad : -1;
    if (i < 3 * Mpad) return op->post.kind == ACT_PRELU ? op->post.slope_off + i - 2 * Mpad : -1;
    const int c = (i - 3 * Mpad) / 12, e = i - 3 * Mpad - 12 * c;
    if (e < 9) return op->dw_w_off + 9 * c + e;
    if (e == 9) return op->dw_b_off + c;
    if (e == 10) return op->dw_act.kind == ACT_PRELU ? op->dw_act.slope_off + c : -1;
    return -1;
}

__device__ __forceinline__ int param_count(cop *op) {
    return 3 * op->Mpad + (op->kind == CHAIN_DWPW ? 12 * op->Cin : 0);
}

// issue the global loads of a layer's parameters (they land while the current layer runs) ...
__device__ __forceinline__ void fetch_params(const float *W, cop *op, float (&pv)[PRM_PER_THREAD], int tid) {
    const int total = param_count(op);
#pragma unroll
    for (int u = 0; u < PRM_PER_THREAD; ++u) {
        const int i = tid + CT * u;
        const int src = i < total ? param_src(op, i) : -1;
        const float v = ldc(W, src >= 0 ? src : 0);
        // a layer without PRelu gets slope 1 (the epilogue's activation is branch-free)
        const bool slope = i >= op->Mpad && i < 3 * op->Mpad;
        pv[u] = src >= 0 ? v : (slope ? 1.f : 0.f);
    }
}

// ... and store them into the layer's LDS parameter buffer
__device__ __forceinline__ void commit_params(cop *op, const float (&pv)[PRM_PER_THREAD], float *prm, int tid) {
    const int total = param_count(op);
#pragma unroll
    for (int u = 0; u < PRM_PER_THREAD; ++u)
        if (tid + CT * u < total) prm[tid + CT * u] = pv[u];
}

// Producer role of a depthwise layer (512 threads, 8 waves): for planes of <= 64 positions wave
// w takes channels w and w + 8 of a chunk with one position per lane; for larger planes (<= 256)
// two threads share a position, 8 channels each.
struct Prod {
    int q, c0, cstep, base;
    bool on;
};

__device__ __forceinline__ Prod producer_of(cop *op, int t) {
    Prod p;
    const int NP = op->NT * 16;
    if (NP <= 64) {  // 8 waves x 2 channels, a position per lane
        p.q = t & 63;
        p.c0 = t >> 6;
        p.cstep = 8;
    } else {  // 2 threads per position, 8 channels each
        p.q = t & 255;
        p.c0 = t >> 8;
        p.cstep = 2;
    }
    p.on = p.q < NP;
    const int q = p.q < op->OP ? p.q : 0;
    const int oy = q / op->OW, ox = q - oy * op->OW;
    p.base = (oy * op->stride - op->pad_t + 1) * op->in_wp + (ox * op->stride - op->pad_l + 1);
    return p;
}

// depthwise outputs of channels kc .. kc+15 into D buffer `d` ([16][ds]); zero rows for
// channels >= Cin and zero columns for q >= OP.  Two channels at a time: their weight records
// (LDS, broadcast 16-byte reads) and 18 taps are all requested before the first is used.
__device__ __forceinline__ void produce(cop *op, const Prod &p, const float *x, const float *prm, float *d, int kc) {
    if (!p.on) return;
    const int Cin = op->Cin, OP = op->OP, in_ps = op->in_ps, wp = op->in_wp, ds = op->ds;
    const int act = op->dw_act.kind;
    const float lo = op->dw_act.lo, hi = op->dw_act.hi;
    const float4 *rec = (const float4 *)(prm + 3 * op->Mpad);  // channel c: rec[3c .. 3c+2]
    const bool qok = p.q < OP;
    const int nc = KC / p.cstep;  // channels per thread: 8 or 2
    for (int g = 0; g < nc; g += 2) {
        float4 w[2][3];
        float t[2][9];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = p.c0 + (g + i) * p.cstep, ch = kc + c;
            const int cs = ch < Cin ? ch : 0;
            w[i][0] = rec[3 * cs], w[i][1] = rec[3 * cs + 1], w[i][2] = rec[3 * cs + 2];
            const float *r0 = x + cs * in_ps + p.base, *r1 = r0 + wp, *r2 = r1 + wp;
            t[i][0] = r0[0], t[i][1] = r0[1], t[i][2] = r0[2];
            t[i][3] = r1[0], t[i][4] = r1[1], t[i][5] = r1[2];
            t[i][6] = r2[0], t[i][7] = r2[1], t[i][8] = r2[2];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = p.c0 + (g + i) * p.cstep, ch = kc + c;
            const float wk[12] = {w[i][0].x, w[i][0].y, w[i][0].z, w[i][0].w, w[i][1].x, w[i][1].y,
                                  w[i][1].z, w[i][1].w, w[i][2].x, w[i][2].y, w[i][2].z, w[i][2].w};
            float a = wk[9];  // bias
#pragma unroll
            for (int k = 0; k < 9; ++k) a = __builtin_fmaf(wk[k], t[i][k], a);
            switch (act) {
            case ACT_RELU: a = fmaxf(a, 0.f); break;
            case ACT_CLIP: a = fminf(fmaxf(a, lo), hi); break;
            case ACT_PRELU: a = a < 0.f ? a * wk[10] : a; break;
            case ACT_SIGMOID: a = 1.f / (1.f + expf(-a)); break;
            default: break;
            }
            d[c * ds + p.q] = (qok && ch < Cin) ? a : 0.f;
        }
    }
}

// re-zero the border cells of an output tensor whose region held another tensor
__device__ __forceinline__ void zero_border(cop *op, float *lds, int t, int nt) {
    const int wp = op->out_wp, hp = op->out_ps / op->out_wp, per = 2 * wp + 2 * (hp - 2);
    float *o = lds + op->out_off;
    for (int i = t; i < op->Cout * per; i += nt) {
        const int c = i / per, e = i - c * per;
        int cell;
        if (e < wp) cell = e;
        else if (e < 2 * wp) cell = (hp - 1) * wp + (e - wp);
        else {
            const int r = (e - 2 * wp) >> 1;
            cell = (r + 1) * wp + ((e & 1) ? wp - 1 : 0);
        }
        o[c * op->out_ps + cell] = 0.f;
    }
}

// The producer waves' side of one layer (not templated: one copy of this code).  It passes the
// same barriers as the consumers' side: per depthwise chunk, then the epilogue's phase 1.
__device__ __forceinline__ void produce_layer(const ChainParams &A, cop *op, float *lds, const float *prm, int tid) {
    const int t = tid - NCW * 64;
    if (op->kind == CHAIN_DWPW) {
        const int nchunks = (op->Cin + KC - 1) / KC;
        float *dbuf = lds + A.d_off;
        const float *x = lds + op->in_off;
        const Prod p = producer_of(op, t);
        produce(op, p, x, prm, dbuf, 0);
        lds_barrier();
        for (int ch = 0; ch < nchunks; ++ch) {
            if (ch + 1 < nchunks) produce(op, p, x, prm, dbuf + ((ch + 1) & 1) * A.d_buf, (ch + 1) * KC);
            lds_barrier();
        }
    }
    lds_barrier();  // the consumers' epilogue phase 1 is done
    if (op->zero_border) zero_border(op, lds, t, CT - NCW * 64);
}

// The consumer waves' side of one layer, holding MTW x NTW 16x16 accumulator tiles
// (compile-time: the tiles stay in registers and no guard sits between the MFMAs).
template <int MTW, int NTW>
__device__ __forceinline__ void run_layer(const ChainParams &A, cop *op, float *lds, const float *prm, int n,
                                          int tid) {
    const int wave = tid >> 6;
    const bool dwpw = op->kind == CHAIN_DWPW;
    const int Cin = op->Cin, nchunks = (Cin + KC - 1) / KC;
    float *dbuf = lds + A.d_off;
    const float *x = lds + op->in_off;
    f32x4 acc[NTW][MTW];
    const int lane = tid & 63, kl = lane >> 4, cl = lane & 15;  // MFMA 16x16x4: A[cl][kl], B[kl][cl]
    const int MS = op->MS, ms = wave % MS, ng = wave / MS, NG = NCW / MS, NT = op->NT;  // consumer tiling
    const int OP = op->OP, OW = op->OW;

    // ---------------- consumers
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int t = 0; t < MTW; ++t) acc[j][t] = (f32x4)(0.f);
    int col[NTW];  // owned N tiles (a tile >= NT is computed on zeros and never stored)
#pragma unroll
    for (int j = 0; j < NTW; ++j) col[j] = (ng + NG * j) * 16 + cl;
    const int Mpad = op->Mpad;
    // A fragments: transposed 1x1 weights [Kpad16][Mpad], row k, column (ms*MTW + t)*16 + cl, in
    // a ring of 4 k-steps: the fragments of step s + 4 are requested as step s consumes its own,
    // so a weight load has four k-steps of MFMAs (and the chunk barrier) to land
    const float *wa = A.weights + op->w_off + kl * Mpad + ms * MTW * 16 + cl;
    const int nsteps = nchunks * 4;
    float ring[4][MTW];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < MTW; ++t) ring[s][t] = s < nsteps ? ldc(wa, 4 * s * Mpad + t * 16) : 0.f;
    if (dwpw) {
        const int ds = op->ds;
        lds_barrier();  // chunk 0's depthwise is in place
        for (int ch = 0; ch < nchunks; ++ch) {
            const float *d = dbuf + (ch & 1) * A.d_buf + kl * ds;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                float a[MTW];
#pragma unroll
                for (int t = 0; t < MTW; ++t) a[t] = ring[s][t];
                const int nk = ch * 4 + s + 4 < nsteps ? ch * 4 + s + 4 : nsteps - 1;
#pragma unroll
                for (int t = 0; t < MTW; ++t) ring[s][t] = ldc(wa, 4 * nk * Mpad + t * 16);
                float b[NTW];
#pragma unroll
                for (int j = 0; j < NTW; ++j) b[j] = d[4 * s * ds + col[j]];  // padding columns hold zeros
#pragma unroll
                for (int j = 0; j < NTW; ++j)
#pragma unroll
                    for (int t = 0; t < MTW; ++t)
                        acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[j], acc[j][t], 0, 0, 0);
            }
            lds_barrier();  // chunk ch+1's depthwise is in place; chunk ch's readers are done
        }
    } else {
        // plain 1x1: B fragments straight from the bordered input planes
        const int in_ps = op->in_ps, wp = op->in_wp;
        int pos[NTW];
        bool qok[NTW];
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int q = col[j] < OP ? col[j] : 0;
            const int oy = q / OW, ox = q - oy * OW;
            pos[j] = (oy + 1) * wp + ox + 1;
            qok[j] = col[j] < OP;
        }
        for (int ch = 0; ch < nchunks; ++ch) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int st = ch * 4 + s;
                float a[MTW];
#pragma unroll
                for (int t = 0; t < MTW; ++t) a[t] = ring[s][t];
                const int nk = st + 4 < nsteps ? st + 4 : nsteps - 1;
#pragma unroll
                for (int t = 0; t < MTW; ++t) ring[s][t] = ldc(wa, 4 * nk * Mpad + t * 16);
                const int k = 4 * st + kl;
                float b[NTW];
#pragma unroll
                for (int j = 0; j < NTW; ++j) {
                    const bool ok = k < Cin && qok[j];
                    const float v = x[ok ? k * in_ps + pos[j] : 0];
                    b[j] = ok ? v : 0.f;
                }
#pragma unroll
                for (int j = 0; j < NTW; ++j)
#pragma unroll
                    for (int t = 0; t < MTW; ++t)
                        acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[j], acc[j][t], 0, 0, 0);
            }
        }
    }

    // Epilogue, one 16x16 tile (4 rows x 1 column per lane) at a time with 4-wide arithmetic
    // and one address computation per tile: (1) y = post( pre(acc + bias) + residual ) back into
    // the accumulators; barrier (every read of the input / residual is done); (2) stores.
    // Activations are branch-free: y = v < 0 ? v * slope : v, then clamped to [lo, hi] -- Relu
    // is slope 1, lo 0 (= fmaxf(v, 0)); PRelu the staged slope; Clip slope 1, [lo, hi]; none
    // slope 1, (-inf, inf).  Staged slopes are 1 where a layer has no PRelu.
    const int Cout = op->Cout;
    const int res_mode = op->res_mode, r_C = op->r_C, res_ps = op->res_ps, res_wp = op->res_wp;
    const float *res = lds + (res_mode ? op->res_off : 0);
    const int prek = op->pre.kind, postk = op->post.kind;
    const float plo = prek == ACT_RELU ? 0.f : prek == ACT_CLIP ? op->pre.lo : -__builtin_huge_valf();
    const float phi = prek == ACT_CLIP ? op->pre.hi : __builtin_huge_valf();
    const float qlo = postk == ACT_RELU ? 0.f : postk == ACT_CLIP ? op->post.lo : -__builtin_huge_valf();
    const float qhi = postk == ACT_CLIP ? op->post.hi : __builtin_huge_valf();
    auto act4 = [](f32x4 v, f32x4 sl, float lo, float hi) {
        f32x4 y;
#pragma unroll
        for (int r = 0; r < 4; ++r) y[r] = fminf(fmaxf(v[r] < 0.f ? v[r] * sl[r] : v[r], lo), hi);
        return y;
    };
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int q = col[j] < OP ? col[j] : 0;
        const int oy = q / OW, ox = q - oy * OW;
        const int rcell = res_mode == 2 ? (2 * oy + 1) * res_wp + 2 * ox + 1 : (oy + 1) * res_wp + ox + 1;
#pragma unroll
        for (int t = 0; t < MTW; ++t) {
            const int m0 = (ms * MTW + t) * 16 + kl * 4;
            const f32x4 bias = *(const f32x4 *)(prm + m0);
            f32x4 v = act4(acc[j][t] + bias, *(const f32x4 *)(prm + Mpad + m0), plo, phi);
            if (res_mode) {
                const float *rp = res + m0 * res_ps + rcell;
                f32x4 rv;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float x0 = rp[r * res_ps];
                    if (res_mode == 2)
                        x0 = fmaxf(fmaxf(x0, rp[r * res_ps + 1]), fmaxf(rp[r * res_ps + res_wp], rp[r * res_ps + res_wp + 1]));
                    rv[r] = m0 + r < r_C ? x0 : 0.f;
                }
                v += rv;
            }
            acc[j][t] = act4(v, *(const f32x4 *)(prm + 2 * Mpad + m0), qlo, qhi);
        }
    }
    lds_barrier();  // every read of the input / residual is done: the output may overwrite them
    // phase 2: stores (the LDS planes of the output, and/or its global destination)
    const int out_off = op->out_off, out_ps = op->out_ps, out_wp = op->out_wp, gout = op->gout;
    if (out_off >= 0) {
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int q = col[j];
            if (ng + NG * j >= NT || q >= OP) continue;
            const int oy = q / OW, ox = q - oy * OW;
            float *op0 = lds + out_off + (oy + 1) * out_wp + ox + 1;
#pragma unroll
            for (int t = 0; t < MTW; ++t) {
                const int m0 = (ms * MTW + t) * 16 + kl * 4;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (m0 + r < Cout) op0[(m0 + r) * out_ps] = acc[j][t][r];
            }
        }
    }
    if (gout >= 0) {
        const ChainOut go = A.gout[gout];
        float *gbase = go.p + (int64_t)n * go.sN;  // per-image offsets are < 2^31
        const int sC = (int)go.sC, sP = (int)go.sP;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int q = col[j];
            if (ng + NG * j >= NT || q >= OP) continue;
#pragma unroll
            for (int t = 0; t < MTW; ++t) {
                const int m0 = (ms * MTW + t) * 16 + kl * 4;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (m0 + r < Cout) gbase[(uint32_t)((m0 + r) * sC + q * sP)] = acc[j][t][r];
            }
        }
    }
}

__global__ __launch_bounds__(CT) void chain_kernel(const ChainParams A) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int n = blockIdx.x, tid = threadIdx.x;
    cop *ops = (cop *)(A.weights + A.ops_off);
    // the entry tensor of this image into bordered planes, and the first layer's parameters
    {
        const float *src = A.entry + (int64_t)n * A.e_sN;
        const int wp = A.e_W + 2, hp = A.e_H + 2, ps = wp * hp, total = A.e_C * ps;
        for (int i = tid; i < total; i += CT) {
            const int c = i / ps, cell = i - c * ps, yb = cell / wp, xb = cell - yb * wp;
            const bool in = yb >= 1 && yb <= A.e_H && xb >= 1 && xb <= A.e_W;
            const float v = src[in ? (int64_t)c * A.e_sC + (yb - 1) * A.e_W + (xb - 1) : 0];
            lds[A.e_off + i] = in ? v : 0.f;
        }
        float pv[PRM_PER_THREAD];
        fetch_params(A.weights, ops, pv, tid);
        commit_params(ops, pv, lds + A.p_off, tid);
    }
    lds_barrier();
    for (int o = 0; o < A.nops; ++o) {
        cop *op = ops + o;
        const float *prm = lds + A.p_off + (o & 1) * A.p_buf;
        // the next layer's parameters: loaded now, stored into the other buffer after this layer
        float pv[PRM_PER_THREAD];
        if (o + 1 < A.nops) fetch_params(A.weights, op + 1, pv, tid);
        if (tid >= NCW * 64) produce_layer(A, op, lds, prm, tid);
        else switch (op->MTW * 16 + op->NTW) {
#define ZR_CHAIN_CASE(M, N) \
    case M * 16 + N: run_layer<M, N>(A, op, lds, prm, n, tid); break;
            ZR_CHAIN_CASE(1, 1) ZR_CHAIN_CASE(1, 2) ZR_CHAIN_CASE(1, 3) ZR_CHAIN_CASE(1, 9)
            ZR_CHAIN_CASE(2, 1) ZR_CHAIN_CASE(2, 2) ZR_CHAIN_CASE(3, 1) ZR_CHAIN_CASE(3, 2)
            ZR_CHAIN_CASE(3, 4) ZR_CHAIN_CASE(4, 1) ZR_CHAIN_CASE(4, 2)
#undef ZR_CHAIN_CASE
        default: break;
        }
        if (o + 1 < A.nops) commit_params(op + 1, pv, lds + A.p_off + ((o + 1) & 1) * A.p_buf, tid);
        lds_barrier();  // this layer's outputs and the next layer's parameters are visible
    }
}

}  // namespace

const char *launch_chain(const ChainParams &p, hipStream_t s) {
    hipLaunchKernelGGL(chain_kernel, dim3(p.N), dim3(CT), sizeof(float) * (size_t)p.lds_floats, s, p);
    return "chain_kernel";
}

}  // namespace zr
