// fused.hip -- the two kernels that cut the plan's HBM traffic the most:
//   * stem_kernel: the dense KxK stride-S stem conv (Cin = 3, the first layer of all four
//     models) with every output channel of a pixel in registers and the weights read through
//     the scalar cache.  With PRE it samples its input straight from the RGBA frames through
//     the per-image views (K1 fused in front), so the f32 input tensor never exists.
//   * dwpw_kernel: a depthwise KxK conv feeding a 1x1 conv (the BlazeBlock / inverted-residual
//     tail) in one launch; the depthwise output of a column tile lives only in LDS.
// Reference: the Conv nodes of the four ONNX graphs that ORT/tract execute at
// crates/zaru/src/nn/mod.rs:483-533, and the image->tensor map at nn/mod.rs:54-73.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "../runtime/zr_kernels.h"
#include "act.h"
#include "epilogue.h"
#include "lds_dma.h"
#include "sample.h"

namespace zr {


typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ stem
constexpr int STH = 8, STW = 32;  // output tile: 8 rows x 32 columns, one pixel per thread

template <int K, int S, int CO, bool PRE>
__global__ __launch_bounds__(256) void stem_kernel(const StemParams P) {
    constexpr int RIN = (STH - 1) * S + K, WIN = (STW - 1) * S + K;
    __shared__ float patch[3][RIN][WIN];
    const int tiles_x = (P.OW + STW - 1) / STW;
    const int ty0 = (blockIdx.x / tiles_x) * STH, tx0 = (blockIdx.x % tiles_x) * STW;
    const int n = blockIdx.y;
    if (P.nact && n >= *P.nact) return;  // (whole workgroup, before any barrier)
    const int iy0 = ty0 * S - P.pad_t, ix0 = tx0 * S - P.pad_l;
    if constexpr (PRE) {
        // all of this thread's pixel gathers are issued before the first is used
        constexpr int NP = (RIN * WIN + 255) / 256;
        const ViewDesc d = P.pre.views[n];
        const FrameDesc f = frame_of(P.pre, d);
        uint32_t px[NP];
        bool pad[NP];
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int i = threadIdx.x + 256 * u;
            const int r = i / WIN, x = i - r * WIN;
            const int iy = iy0 + r, ix = ix0 + x;
            // outside the network input: the ONNX zero padding of the f32 tensor
            pad[u] = !(i < RIN * WIN && iy >= 0 && iy < P.IH && ix >= 0 && ix < P.IW);
            px[u] = load_pixel(f, pad[u] ? -1 : sample_offset(d, f, ix, iy, P.IW, P.IH));
        }
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int i = threadIdx.x + 256 * u;
            if (i >= RIN * WIN) break;
            const int r = i / WIN, x = i - r * WIN;
            patch[0][r][x] = pad[u] ? 0.f : color_map(px[u], 0, P.pre.adjust, P.pre.lo);
            patch[1][r][x] = pad[u] ? 0.f : color_map(px[u], 1, P.pre.adjust, P.pre.lo);
            patch[2][r][x] = pad[u] ? 0.f : color_map(px[u], 2, P.pre.adjust, P.pre.lo);
        }
    } else {
        const float *src = P.in.p + (int64_t)n * P.in.sN;
        for (int i = threadIdx.x; i < 3 * RIN * WIN; i += 256) {
            const int c = i / (RIN * WIN), rem = i - c * (RIN * WIN);
            const int r = rem / WIN, x = rem - r * WIN;
            const int iy = iy0 + r, ix = ix0 + x;
            (&patch[0][0][0])[i] = (iy >= 0 && iy < P.IH && ix >= 0 && ix < P.IW)
                                       ? src[(int64_t)c * P.in.sC + (int64_t)iy * P.IW + ix]
                                       : 0.f;
        }
    }
    __syncthreads();
    const int ly = threadIdx.x / STW, lx = threadIdx.x - ly * STW;
    f32x2 acc[CO / 2];
#pragma unroll
    for (int o = 0; o < CO / 2; ++o) acc[o] = (f32x2)(0.f);
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const float v = patch[c][ly * S + ky][lx * S + kx];
                // weights [3][K][K][32]: uniform, so scalar loads feeding v_pk_fma_f32
                const f32x2 *w2 = (const f32x2 *)(P.w + ((c * K + ky) * K + kx) * 32);
#pragma unroll
                for (int o = 0; o < CO / 2; ++o) acc[o] = __builtin_elementwise_fma(w2[o], (f32x2)(v), acc[o]);
            }
    const int oy = ty0 + ly, ox = tx0 + lx;
    if (oy >= P.OH || ox >= P.OW) return;
    float vo[CO];
#pragma unroll
    for (int o = 0; o < CO / 2; ++o) {
        vo[2 * o] = acc[o].x + P.bias[2 * o];
        vo[2 * o + 1] = acc[o].y + P.bias[2 * o + 1];
    }
    apply_act_n<CO>(P.act, vo, [](int o) { return o; });
    float *dst = P.out + (int64_t)n * P.o_sN + (int64_t)oy * P.OW + ox;
#pragma unroll
    for (int o = 0; o < CO; ++o)
        if (o < P.Cout) dst[(int64_t)o * P.o_sC] = vo[o];
}

bool stem_supported(int cin, int k, int stride, int cout) {
    return cin == 3 && (k == 3 || k == 5) && (stride == 1 || stride == 2) && cout >= 1 && cout <= 32;
}

template <int K, int S, int CO>
static const char *stem_go(const StemParams &p, bool pre, hipStream_t s) {
    const int tiles = ((p.OH + STH - 1) / STH) * ((p.OW + STW - 1) / STW);
    dim3 grid(tiles, p.N);
    if (pre) hipLaunchKernelGGL((stem_kernel<K, S, CO, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((stem_kernel<K, S, CO, false>), grid, dim3(256), 0, s, p);
    return kernel_name("stem_kernel<%d,%d,%d,%s>", K, S, CO, pre ? "true" : "false");
}

template <int K, int S>
static const char *stem_co(const StemParams &p, bool pre, hipStream_t s) {
    if (p.Cout <= 16) return stem_go<K, S, 16>(p, pre, s);
    if (p.Cout <= 24) return stem_go<K, S, 24>(p, pre, s);
    return stem_go<K, S, 32>(p, pre, s);
}

const char *launch_stem(const StemParams &p, bool pre, hipStream_t s) {
    if (p.k == 3) return p.stride == 1 ? stem_co<3, 1>(p, pre, s) : stem_co<3, 2>(p, pre, s);
    return p.stride == 1 ? stem_co<5, 1>(p, pre, s) : stem_co<5, 2>(p, pre, s);
}

// ------------------------------------------------------------------ depthwise -> 1x1
// The few-channel high-resolution BlazeBlocks run as VALU kernels (below); the many-channel
// low-resolution ones as f32 MFMA kernels (dwpw_mfma.hip).

// VALU form for the high-resolution layers with few channels (Cin * Cout <= 2048: the
// BlazeBlocks at 96^2 .. 32^2), where the MFMA tile would be mostly padding and the
// per-lane tap loads cost more memory instructions than the bytes they bring.  One thread per
// output position, 256 positions of one image per workgroup:
//   1. per chunk of VFKC input channels, the input rows the tile needs are staged in LDS with
//      16-byte row loads (zero columns/rows where the ONNX padding is);
//   2. each thread computes its depthwise value per channel from LDS (one ds_read + FMA per
//      tap) and accumulates the 1x1 conv into CO registers with v_pk_fma_f32, the weights
//      coming through the scalar cache (they are uniform across the workgroup);
//   3. epilogue per output channel: bias, activation, residual (+pad/+pool), activation, one
//      coalesced store per channel.
constexpr int VTQ = 256, VFKC = 8;

// DB: the staging goes global -> LDS by LDS-DMA (global_load_lds_dwordx4) into two buffers, the
// next chunk's copy in flight while the current chunk is computed (one barrier per chunk).  The
// staged image is slot-linear (slot = 16 B; row stride lw = 4 * srow floats), exactly the
// lane-linear order one DMA wave-instruction writes; zero slots (padding) read zr_zero4.
template <int K, int S, int CO, bool DB, int VF>
__global__ __launch_bounds__(256) void dwpw_valu_kernel(const DwPwParams P, int tpi, int ntiles, int bufsz, int lw) {
    extern __shared__ __attribute__((aligned(16))) float sIn[];  // [VF * rows][lw]
    const GemmParams &G = P.g;
    const int cpx = gridDim.x >> 3;  // gridDim.x is a multiple of 8
    const int tile = (blockIdx.x & 7) * cpx + (blockIdx.x >> 3);
    if (tile >= ntiles) return;  // whole workgroup, before any barrier
    const int tid = threadIdx.x;
    const int n = tile / tpi, q0 = (tile - n * tpi) * VTQ;
    if (G.nact && n >= *G.nact) return;
    const int Pq = G.P, H = P.in.H, W = P.in.W, Cin = G.K, OW = P.OW;
    const int oy_a = q0 / OW, oy_b = min(q0 + VTQ - 1, Pq - 1) / OW;
    const int iy_a = oy_a * S - P.pad_t;
    const int R = (oy_b - oy_a) * S + K;  // VF * R * lw <= bufsz (floats per LDS buffer)
    const int q = min(q0 + tid, Pq - 1);
    const int oy = q / OW, ox = q - oy * OW;
    // LDS row layout: 4 zero floats, the W input values, >= 4 zero floats (lw % 4 == 0)
    const int lb = (oy * S - P.pad_t - iy_a) * lw + 4 - P.pad_l + ox * S;  // tap (0, 0)
    const uint32_t nbase = (uint32_t)n * (uint32_t)P.in.sN;
    const int srow = (W >> 2) + 2;  // float4 slots per staged row
    const float inv_srow = 1.f / (float)srow, inv_R = 1.f / (float)R;

    f32x2 acc[CO / 2];
#pragma unroll
    for (int i = 0; i < CO / 2; ++i) acc[i] = (f32x2)(0.f);

    const int total = VF * R * srow;
    // The slot -> (channel, row, column) decomposition is the same for every chunk: for the
    // (at most 4 * DMAX) DMA wave-instructions of a buffer it is computed once, as the slot's
    // offset from the chunk's first channel plane (-1: a zero slot) and its channel.
    constexpr int DMAX = DB ? 6 : 1;
    const int nwi = (total + 63) >> 6, lane = tid & 63, wave = tid >> 6;
    const bool pre_off = nwi <= 4 * DMAX;
    int goff[DMAX], gch[DMAX];
    if constexpr (DB) {
#pragma unroll
        for (int m = 0; m < DMAX; ++m) {
            const int sl = (wave + 4 * m) * 64 + lane;
            const int cr = qdiv(sl, srow, inv_srow), sx = sl - cr * srow;
            const int c = qdiv(cr, R, inv_R), r = cr - c * R;
            const int iy = iy_a + r, xv = sx - 1;
            const bool ok = sl < total && iy >= 0 && iy < H && xv >= 0 && 4 * xv < W;
            goff[m] = ok ? (int)((uint32_t)c * (uint32_t)P.in.sC + nbase + (uint32_t)(iy * W + 4 * xv)) : -1;
            gch[m] = c;
        }
    }
    auto stage_dma = [&](int kc, float *dst) {
        if (pre_off) {
            const float *base = P.in.p + (size_t)(uint32_t)kc * (uint32_t)P.in.sC;
            const int cl = Cin - kc;
#pragma unroll
            for (int m = 0; m < DMAX; ++m) {
                const int wi = wave + 4 * m;
                if (wi < nwi) {
                    const bool ok = goff[m] >= 0 && gch[m] < cl;
                    const float *src = ok ? base + (uint32_t)goff[m] : (const float *)&zr_zero4;
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                                     (__attribute__((address_space(3))) void *)(dst + wi * 256), 16, 0, 0);
                }
            }
            return;
        }
        for (int wi = wave; wi < nwi; wi += 4) {
            const int sl = wi * 64 + lane;
            const int cr = qdiv(sl, srow, inv_srow), sx = sl - cr * srow;
            const int c = qdiv(cr, R, inv_R), r = cr - c * R;
            const int iy = iy_a + r, ch = kc + c, xv = sx - 1;
            const bool ok = sl < total && iy >= 0 && iy < H && ch < Cin && xv >= 0 && 4 * xv < W;
            const float *src = ok ? P.in.p + (size_t)(uint32_t)ch * (uint32_t)P.in.sC + nbase + (uint32_t)(iy * W + 4 * xv)
                                  : (const float *)&zr_zero4;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(dst + wi * 256), 16, 0, 0);
        }
    };
    if constexpr (DB) stage_dma(0, sIn);

    for (int kc = 0, it = 0; kc < Cin; kc += VF, ++it) {
        const float *buf = sIn;
        if constexpr (DB) {
            buf = sIn + (it & 1) * bufsz;
            __syncthreads();  // vmcnt(0) + barrier: chunk kc has landed, chunk kc - VF's readers are done
            if (kc + VF < Cin) stage_dma(kc + VF, sIn + ((it + 1) & 1) * bufsz);
        } else
        for (int base = 0; base < total; base += 1024) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int sl = min(base + tid + 256 * u, total - 1);
                const int cr = qdiv(sl, srow, inv_srow), sx = sl - cr * srow;
                const int c = qdiv(cr, R, inv_R), r = cr - c * R;
                const int iy = iy_a + r, ch = kc + c, xv = sx - 1;
                const bool ok = iy >= 0 && iy < H && ch < Cin && xv >= 0 && 4 * xv < W;
                const float *src = P.in.p + (size_t)(uint32_t)(ch < Cin ? ch : Cin - 1) * (uint32_t)P.in.sC;
                const float4 x = *(const float4 *)(src + nbase + (uint32_t)(ok ? iy * W + 4 * xv : 0));
                v[u] = ok ? x : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int sl = base + tid + 256 * u;
                if (sl < total) {
                    const int cr = qdiv(sl, srow, inv_srow), sx = sl - cr * srow;
                    *(float4 *)(sIn + cr * lw + 4 * sx) = v[u];
                }
            }
        }
        if constexpr (!DB) __syncthreads();
#pragma unroll 2
        for (int c = 0; c < VF; ++c) {
            const int ch = kc + c;
            if (ch >= Cin) break;
            const float *t0 = buf + c * R * lw + lb;
            const float *w = P.dw_w + ch * (K * K);
            float d = ldc(P.dw_b, ch);
#pragma unroll
            for (int ky = 0; ky < K; ++ky)
#pragma unroll
                for (int kx = 0; kx < K; ++kx) d = __builtin_fmaf(ldc(w, ky * K + kx), t0[ky * lw + kx], d);
            d = apply_act(P.dw_act, d, ch);
            const __attribute__((address_space(4))) f32x2 *w2 =
                (const __attribute__((address_space(4))) f32x2 *)(G.wt + (size_t)ch * G.Mpad);  // [Kpad][Mpad]
#pragma unroll
            for (int i = 0; i < CO / 2; ++i) acc[i] = __builtin_elementwise_fma(w2[i], (f32x2)(d), acc[i]);
        }
        if constexpr (!DB) __syncthreads();
    }

    if (q0 + tid >= Pq) return;
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
            const float x = G.r[rb + (uint32_t)(m < G.r_C ? m : 0) * (uint32_t)G.r_sC];
            rv[m] = m < G.r_C ? x : 0.f;
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

// The BlazeBlock case of the DB VALU form (form "vres"): the residual is the block input, i.e.
// the depthwise input the chunks already stage -- at stride 1 its value at a position is the
// centre tap (pad, pad), at stride 2 its 2x2 max-pool is the max of taps (pad..pad+1)^2 (TF-style
// pads, even planes).  So the residual is captured from the taps in registers while the
// depthwise runs, and the epilogue has no loads left: a tile's lifetime loses one HBM round trip
// and the launch a third of its reads.  Needs Cin <= CO (each input channel's residual lands in
// its own register) and no depthwise activation; the chunk loop is unrolled so every register
// index is static.  Same arithmetic, same order as dwpw_valu_kernel.
// WL: the layer's weights are staged in LDS (see below) -- for launches of few tiles, where each
// CU's scalar cache is cold for every channel; otherwise they come through the scalar cache.
template <int K, int S, int CO, int VF, int RES, bool WL>
__global__ __launch_bounds__(256) void dwpw_vres_kernel(const DwPwParams P, int tpi, int ntiles, int bufsz, int lw) {
    extern __shared__ __attribute__((aligned(16))) float sIn[];  // two buffers of [VF * rows][lw]
    constexpr int NCH = (CO + VF - 1) / VF, PL = DwPad<K, S>::L, DMAX = 6, VT = VTQ, NW = 4;
    const GemmParams &G = P.g;
    const int cpx = gridDim.x >> 3;  // gridDim.x is a multiple of 8
    const int tile = (blockIdx.x & 7) * cpx + (blockIdx.x >> 3);
    if (tile >= ntiles) return;  // whole workgroup, before any barrier
    const int tid = threadIdx.x;
    const int n = tile / tpi, q0 = (tile - n * tpi) * VT;
    if (G.nact && n >= *G.nact) return;
    const int Pq = G.P, H = P.in.H, W = P.in.W, Cin = G.K, OW = P.OW, r_C = G.r_C;
    const int oy_a = q0 / OW, oy_b = min(q0 + VT - 1, Pq - 1) / OW;
    const int iy_a = oy_a * S - P.pad_t;
    const int R = (oy_b - oy_a) * S + K;
    const int q = min(q0 + tid, Pq - 1);
    const int oy = q / OW, ox = q - oy * OW;
    const int lb = (oy * S - P.pad_t - iy_a) * lw + 4 - P.pad_l + ox * S;  // tap (0, 0)
    const uint32_t nbase = (uint32_t)n * (uint32_t)P.in.sN;
    const int srow = (W >> 2) + 2;
    const float inv_srow = 1.f / (float)srow, inv_R = 1.f / (float)R;

    f32x2 acc[CO / 2];
    float rv[CO];
#pragma unroll
    for (int i = 0; i < CO / 2; ++i) acc[i] = (f32x2)(0.f);
#pragma unroll
    for (int m = 0; m < CO; ++m) rv[m] = 0.f;

    const int total = VF * R * srow;
    const int nwi = (total + 63) >> 6, lane = tid & 63, wave = tid >> 6;
    const bool pre_off = nwi <= NW * DMAX;
    int goff[DMAX], gch[DMAX];
#pragma unroll
    for (int m = 0; m < DMAX; ++m) {
        const int sl = (wave + NW * m) * 64 + lane;
        const int cr = qdiv(sl, srow, inv_srow), sx = sl - cr * srow;
        const int c = qdiv(cr, R, inv_R), r = cr - c * R;
        const int iy = iy_a + r, xv = sx - 1;
        const bool ok = sl < total && iy >= 0 && iy < H && xv >= 0 && 4 * xv < W;
        goff[m] = ok ? (int)((uint32_t)c * (uint32_t)P.in.sC + nbase + (uint32_t)(iy * W + 4 * xv)) : -1;
        gch[m] = c;
    }
    auto stage_dma = [&](int kc, float *dst) {
        if (pre_off) {
            const float *base = P.in.p + (size_t)(uint32_t)kc * (uint32_t)P.in.sC;
            const int cl = Cin - kc;
#pragma unroll
            for (int m = 0; m < DMAX; ++m) {
                const int wi = wave + NW * m;
                if (wi < nwi) {
                    const bool ok = goff[m] >= 0 && gch[m] < cl;
                    const float *src = ok ? base + (uint32_t)goff[m] : (const float *)&zr_zero4;
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                                     (__attribute__((address_space(3))) void *)(dst + wi * 256), 16, 0, 0);
                }
            }
            return;
        }
        for (int wi = wave; wi < nwi; wi += NW) {
            const int sl = wi * 64 + lane;
            const int cr = qdiv(sl, srow, inv_srow), sx = sl - cr * srow;
            const int c = qdiv(cr, R, inv_R), r = cr - c * R;
            const int iy = iy_a + r, ch = kc + c, xv = sx - 1;
            const bool ok = sl < total && iy >= 0 && iy < H && ch < Cin && xv >= 0 && 4 * xv < W;
            const float *src = ok ? P.in.p + (size_t)(uint32_t)ch * (uint32_t)P.in.sC + nbase + (uint32_t)(iy * W + 4 * xv)
                                  : (const float *)&zr_zero4;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(dst + wi * 256), 16, 0, 0);
        }
    };
    // the layer's weights into LDS once, behind the two stage buffers: 1x1 [Cin][CO], depthwise
    // records [Cin][RS] (K*K weights, bias, zeros).  The loop then reads only LDS (in-order
    // returns, so the compiler can run loads ahead under lgkmcnt(N)); scalar loads there would
    // share lgkmcnt and, returning out of order, force lgkmcnt(0) per channel.
    constexpr int RS = (K * K + 1 + 3) / 4 * 4;
    float *sW = sIn + 2 * bufsz, *sD = sW + Cin * CO;
    if constexpr (WL) {
    for (int i = tid; i < Cin * CO; i += 64 * NW) {
        const int k = i / CO, m = i - k * CO;
        sW[i] = G.wt[(size_t)k * G.Mpad + m];
    }
    for (int i = tid; i < Cin * RS; i += 64 * NW) {
        const int c = i / RS, e = i - c * RS;
        sD[i] = e < K * K ? P.dw_w[c * K * K + e] : e == K * K ? P.dw_b[c] : 0.f;
    }
    }
    stage_dma(0, sIn);

#pragma unroll
    for (int j = 0; j < NCH; ++j) {
        const int kc = j * VF;
        if (kc >= Cin) break;
        const float *buf = sIn + (j & 1) * bufsz;
        // every wave's DMA of chunk j has landed (explicit: the barrier alone does not promise
        // it), then chunk j - 1's readers are done with the other buffer
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (kc + VF < Cin) stage_dma(kc + VF, sIn + ((j + 1) & 1) * bufsz);
        // one channel: depthwise from the staged taps, residual capture, 1x1 accumulation
        auto chan = [&](int c, int ch) {
            const float *t0 = buf + c * R * lw + lb;
            float t[K * K], wk[RS];
#pragma unroll
            for (int ky = 0; ky < K; ++ky)
#pragma unroll
                for (int kx = 0; kx < K; ++kx) t[ky * K + kx] = t0[ky * lw + kx];
            if constexpr (WL) {
#pragma unroll
                for (int e = 0; e < RS; e += 4) *(f32x4 *)(wk + e) = *(const f32x4 *)(sD + ch * RS + e);  // broadcast
            } else {
#pragma unroll
                for (int e = 0; e < K * K; ++e) wk[e] = ldc(P.dw_w, ch * K * K + e);
                wk[K * K] = ldc(P.dw_b, ch);
            }
            float d = wk[K * K];
#pragma unroll
            for (int k = 0; k < K * K; ++k) d = __builtin_fmaf(wk[k], t[k], d);
            float r = t[PL * K + PL];
            if constexpr (RES == 2)
                r = fmaxf(fmaxf(r, t[PL * K + PL + 1]), fmaxf(t[(PL + 1) * K + PL], t[(PL + 1) * K + PL + 1]));
            rv[ch] = ch < r_C ? r : 0.f;
            if constexpr (WL) {
                const f32x4 *w4 = (const f32x4 *)(sW + ch * CO);  // broadcast
#pragma unroll
                for (int i = 0; i < CO / 4; ++i) {
                    const f32x4 w = w4[i];
                    acc[2 * i] = __builtin_elementwise_fma(f32x2{w.x, w.y}, (f32x2)(d), acc[2 * i]);
                    acc[2 * i + 1] = __builtin_elementwise_fma(f32x2{w.z, w.w}, (f32x2)(d), acc[2 * i + 1]);
                }
            } else {
                const __attribute__((address_space(4))) f32x2 *w2 =
                    (const __attribute__((address_space(4))) f32x2 *)(G.wt + (size_t)ch * G.Mpad);  // [Kpad][Mpad]
#pragma unroll
                for (int i = 0; i < CO / 2; ++i) acc[i] = __builtin_elementwise_fma(w2[i], (f32x2)(d), acc[i]);
            }
        };
#pragma unroll
        for (int c = 0; c < VF; ++c) {
            // (a per-channel exit measured faster than straight-line whole chunks: the scheduler
            // then keeps fewer loads in flight but the occupancy and the scalar cache hold up)
            if (kc + c >= Cin || kc + c >= CO) break;
            chan(c, kc + c);
        }
    }

    if (q0 + tid >= Pq) return;
    float v[CO];
#pragma unroll
    for (int i = 0; i < CO / 2; ++i) {
        v[2 * i] = acc[i].x + G.bias[2 * i];
        v[2 * i + 1] = acc[i].y + G.bias[2 * i + 1];
    }
    auto chan = [](int m) { return m; };
    apply_act_n<CO>(G.pre, v, chan);
#pragma unroll
    for (int m = 0; m < CO; ++m) v[m] += rv[m];
    apply_act_n<CO>(G.post, v, chan);
    const uint32_t ob = (uint32_t)n * (uint32_t)G.o_sN + (uint32_t)q * (uint32_t)G.o_sP;
#pragma unroll
    for (int m = 0; m < CO; ++m)
        if (m < G.M) G.out[ob + (uint32_t)m * (uint32_t)G.o_sC] = v[m];
}

bool dwpw_supported(int k, int stride) { return (k == 3 || k == 5) && (stride == 1 || stride == 2); }

namespace {


// The vres form's case (see dwpw_vres_kernel): 1 = residual is the centre tap, 2 = its 2x2
// max-pool from the taps, 0 = not applicable.
static int vres_mode(const DwPwParams &p, int S, int CO) {
    const GemmParams &g = p.g;
    if (!form_on(FORM_VRES) || g.res_mode == 0 || g.r != p.in.p || g.r_sN != p.in.sN || g.r_sC != p.in.sC ||
        g.K > CO || g.r_C > g.K || p.dw_act.kind != ACT_NONE)
        return 0;
    const int pl = S == 1 ? p.k / 2 : p.k / 2 - 1;
    if (p.pad_t != pl || p.pad_l != pl || pl < 0) return 0;
    const int OH = g.P / p.OW;
    if (g.res_mode == 1 && S == 1 && p.OW == p.in.W && OH == p.in.H) return 1;
    if (g.res_mode == 2 && S == 2 && g.r_W == p.in.W && p.in.H % 2 == 0 && p.in.W % 2 == 0 &&
        2 * p.OW == p.in.W && 2 * OH == p.in.H && pl + 1 < p.k)
        return 2;
    return 0;
}

template <int K, int S, int CO>
const char *dwpw_vres_go(const DwPwParams &p, hipStream_t s) {
    const int P = p.g.P, N = p.g.ncols / P, vt = VTQ;
    const int tpi = (P + vt - 1) / vt, ntiles = tpi * N;
    int rmax = 0;
    for (int t = 0; t < tpi; t++) {
        const int q0 = t * vt, a = q0 / p.OW, b = std::min(q0 + vt - 1, P - 1) / p.OW;
        rmax = std::max(rmax, (b - a) * S + K);
    }
    const int lw = p.in.W + 8;
    auto buf_of = [&](int vf) { return (vf * rmax * lw + 255) / 256 * 256; };  // whole 1 KiB DMA rows
    // 8-channel chunks for 32 channels where two buffers fit 64 KiB (as measured for
    // dwpw_valu_kernel), else 4
    const bool vf8 = 2 * sizeof(float) * (size_t)buf_of(VFKC) <= 64 * 1024 && CO == 32;
    const int vf = vf8 ? VFKC : 4, bufsz = buf_of(vf);
    dim3 grid((ntiles + 7) / 8 * 8);
    constexpr int mode = S;  // vres_mode: centre tap at stride 1, 2x2 pool at stride 2
    const bool wl = ntiles < 2048;  // measured: LDS weights win below ~8 tiles per CU, lose above
    const size_t lds = sizeof(float) * (2 * (size_t)bufsz + (wl ? (size_t)p.g.K * (CO + (K * K + 4) / 4 * 4) : 0));
    if (wl) {
        if (vf8) hipLaunchKernelGGL((dwpw_vres_kernel<K, S, CO, VFKC, mode, true>), grid, dim3(256), lds, s, p, tpi, ntiles, bufsz, lw);
        else hipLaunchKernelGGL((dwpw_vres_kernel<K, S, CO, 4, mode, true>), grid, dim3(256), lds, s, p, tpi, ntiles, bufsz, lw);
    } else {
        if (vf8) hipLaunchKernelGGL((dwpw_vres_kernel<K, S, CO, VFKC, mode, false>), grid, dim3(256), lds, s, p, tpi, ntiles, bufsz, lw);
        else hipLaunchKernelGGL((dwpw_vres_kernel<K, S, CO, 4, mode, false>), grid, dim3(256), lds, s, p, tpi, ntiles, bufsz, lw);
    }
    return kernel_name("dwpw_vres_kernel<%d,%d,%d,%d,%d,%s>", K, S, CO, vf, mode, wl ? "true" : "false");
}

template <int K, int S, int CO>
const char *dwpw_valu_go(const DwPwParams &p, hipStream_t s) {
    const int P = p.g.P, tpi = (P + VTQ - 1) / VTQ, ntiles = tpi * (p.g.ncols / P);
    int rmax = 0;
    for (int t = 0; t < tpi; t++) {
        const int q0 = t * VTQ, a = q0 / p.OW, b = std::min(q0 + VTQ - 1, P - 1) / p.OW;
        rmax = std::max(rmax, (b - a) * S + K);
    }
    const int lw = p.in.W + 8;
    // Double-buffered LDS-DMA staging (form valu_db).  Measured per CO: 32 channels: 8-channel
    // chunks while two buffers fit 64 KiB (the 131 VGPRs hold a CU to 3 workgroups anyway), else
    // 4-channel chunks; 16 channels: 4-channel chunks, so two buffers cost no more LDS (and
    // occupancy) than one 8-channel buffer; 48 channels: at stride 2, and at stride 1 in the
    // vres form (the residual-loading form is slower there).
    auto buf_of = [&](int vf) { return (vf * rmax * lw + 255) / 256 * 256; };  // whole 1 KiB DMA rows
    const bool fit8 = 2 * sizeof(float) * (size_t)buf_of(VFKC) <= 64 * 1024;
    const int vres = vres_mode(p, S, CO);
    const bool db = form_on(FORM_VALU_DB) && (CO == 16 || CO == 32 || (CO == 48 && (S == 2 || vres))) &&
                    2 * sizeof(float) * (size_t)buf_of(4) <= 64 * 1024;
    // 16 channels from >= 32 inputs at >= 96-wide planes (BlazeFace full range's 96^2 32 -> 8):
    // 8-channel chunks too, half the DMA round trips per tile (122 / 119 -> 117 / 114 us at 171
    // images; the hand network's 112^2 24 -> 16 lost 240 -> 282 us, its larger buffers halving the
    // workgroups per CU: profiles/r06_layers/*_valu16vf8_vs_4.txt).  ZARU_HIP_VALU16_VF8=0: 4.
    static const bool v16 = [] {
        const char *e = std::getenv("ZARU_HIP_VALU16_VF8");
        return !e || std::strtol(e, nullptr, 10) != 0;
    }();
    const bool small = db && !((CO == 32 || (CO == 16 && v16 && p.in.W >= 96 && p.g.K >= 32)) && fit8);
    const int vf = small ? 4 : VFKC;
    const int bufsz = buf_of(vf);
    dim3 grid((ntiles + 7) / 8 * 8);
    if (db && vres) return dwpw_vres_go<K, S, CO>(p, s);
    if (db) {
        const size_t lds = 2 * sizeof(float) * (size_t)bufsz;
        if (small)
            hipLaunchKernelGGL((dwpw_valu_kernel<K, S, CO, true, 4>), grid, dim3(256), lds, s, p, tpi, ntiles, bufsz, lw);
        else
            hipLaunchKernelGGL((dwpw_valu_kernel<K, S, CO, true, VFKC>), grid, dim3(256), lds, s, p, tpi, ntiles, bufsz, lw);
    } else {
        const size_t lds = sizeof(float) * (size_t)VFKC * rmax * lw;
        hipLaunchKernelGGL((dwpw_valu_kernel<K, S, CO, false, VFKC>), grid, dim3(256), lds, s, p, tpi, ntiles, bufsz, lw);
    }
    const int vfe = db ? vf : VFKC;
    return kernel_name("dwpw_valu_kernel<%d,%d,%d,%s,%d>", K, S, CO, db ? "true" : "false", vfe);
}

template <int K, int S>
const char *dwpw_valu_co(const DwPwParams &p, hipStream_t s) {
    if (p.g.M <= 16) return dwpw_valu_go<K, S, 16>(p, s);
    if (p.g.M <= 32) return dwpw_valu_go<K, S, 32>(p, s);
    if (p.g.M <= 48) return dwpw_valu_go<K, S, 48>(p, s);
    return dwpw_valu_go<K, S, 64>(p, s);
}

}  // namespace

// The VALU form applies to (see dwpw_valu_kernel): >= 256 positions per image, W % 4 == 0
// (16-byte row loads), Cout <= 48, Cin * Cout <= 2048, staged rows within 64 KiB.
static bool valu_form(const DwPwParams &p) {
    if (!form_on(FORM_VALU) || p.g.P < VTQ || p.in.W % 4 != 0 || p.in.W > 248 || p.g.M > 48 || p.g.K * p.g.M > 2048)
        return false;
    if (p.g.ncols % p.g.P != 0) return false;
    const int rows = (VTQ / p.OW + 2) * p.stride + p.k;
    return sizeof(float) * (size_t)VFKC * rows * (p.in.W + 8) <= 64 * 1024;
}

// High-resolution planes with few channels take the VALU form; the rest an MFMA form
// (launch_dwpw_mfma, dwpw_mfma.hip).
const char *launch_dwpw(const DwPwParams &p, hipStream_t s) {
    if (valu_form(p)) {
        if (p.k == 3) return p.stride == 1 ? dwpw_valu_co<3, 1>(p, s) : dwpw_valu_co<3, 2>(p, s);
        return p.stride == 1 ? dwpw_valu_co<5, 1>(p, s) : dwpw_valu_co<5, 2>(p, s);
    }
    return launch_dwpw_mfma(p, s);
}

const char *launch_dwpw_group(const DwPwParams *p, int n, hipStream_t s) {
    for (int i = 0; i < n; ++i)
        if (valu_form(p[i])) return nullptr;
    return launch_dwpw_mfma_group(p, n, s);
}

}  // namespace zr
