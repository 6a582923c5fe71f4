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
// A workgroup (4 waves) owns a BM x BN output tile: BN consecutive columns j = n*P + q of the
// 1x1 conv's output and BM of its output channels.  The waves are laid out WM along M and
// 4/WM along N; each wave holds MTW x NTW 32x32 accumulator tiles.  Per chunk of FKC input
// channels:
//   1. the workgroup computes the depthwise outputs of the chunk for its BN columns into LDS
//      (taps straight from L1/L2, where neighbouring columns share them; every tap of the
//      chunk is issued before the first is used; clamped addresses + a validity mask, never a
//      branch around a load);
//   2. the chunk of the transposed 1x1 weights goes to LDS;
//   3. every wave runs v_mfma_f32_32x32x2_f32 over the chunk.
// The epilogue is epilogue_tile: bias, activation, residual (+pad/+pool), activation.
// The layout is chosen per layer (launch_dwpw) so that a launch has enough workgroups to fill
// 256 CUs without splitting M (which would recompute the depthwise part): wide column tiles
// for the few-channel high-resolution layers, tall channel tiles for the 128/256-channel
// low-resolution ones.  Column tiles are dealt to XCDs in contiguous runs, so halo rows and the
// residual re-read are L2 hits on the XCD that just fetched them.
// V4: the depthwise part computes 4 horizontally adjacent outputs per thread from one input
// window per row (float4 loads plus pad_l scalars) instead of K*K lane-private taps per
// output: ~4x fewer memory instructions.  Needs OW % 4 == 0, W % 4 == 0 and the models'
// TF-style pads (K3: 1 for stride 1, 0 for stride 2; K5: 2 / 1) -- see v4_ok().
template <int K, int S> struct DwPad { static constexpr int L = S == 1 ? K / 2 : K / 2 - 1; };

template <int K, int S, int WM, int MTW, int NTW, bool V4>
__global__ __launch_bounds__(256) void dwpw_kernel(const DwPwParams P, int nct) {
    constexpr int WN = 4 / WM;
    constexpr int BN = WN * NTW * 32, BM = WM * MTW * 32;
    constexpr int KK = K * K;
    constexpr int FKC = K == 3 ? 16 : 8;  // input channels per chunk
    constexpr int CPAR = 256 / BN;        // channels whose depthwise runs side by side
    constexpr int PER = FKC / CPAR;       // depthwise outputs per thread per chunk
    static_assert(PER >= 1 && FKC % CPAR == 0, "tile/chunk mismatch");
    // V4 layout: Q column quads x CS channel slots; CPT channels per thread
    constexpr int Q = BN / 4, CS = 256 / Q, CPT = FKC > CS ? FKC / CS : 1;
    constexpr int PL = DwPad<K, S>::L;
    constexpr int NV = (3 * S + K - PL + 3) / 4;  // float4 loads per window row
    constexpr int WL = PL + 4 * NV;               // window floats per row
    __shared__ __attribute__((aligned(16))) float sD[FKC][BN];
    __shared__ float sW[FKC][BM];
    const GemmParams &G = P.g;

    const int cpx = gridDim.x >> 3;  // gridDim.x is a multiple of 8
    const int tile = (blockIdx.x & 7) * cpx + (blockIdx.x >> 3);
    if (tile >= nct) return;  // whole workgroup, before any barrier
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kh = lane >> 5, col = lane & 31;
    const int wm = wave % WM, wn = wave / WM;
    const int j0 = tile * BN, m0 = blockIdx.y * BM;
    const int Cin = G.K;

    // depthwise role: column dj of the tile, channels dc, dc + CPAR, ... of each chunk
    const int dj = tid % BN;
    int dc = tid / BN;
    if constexpr (BN >= 64) dc = __builtin_amdgcn_readfirstlane(dc);  // one channel per wave
    const int jd = min(j0 + dj, G.ncols - 1);
    const int n = jd / G.P, q = jd - n * G.P;
    const int oy = q / P.OW, ox = q - oy * P.OW;
    const int iy0 = oy * S - P.pad_t, ix0 = ox * S - P.pad_l;
    const int H = P.in.H, W = P.in.W;
    // tap byte offsets from a channel plane's base, image included (32-bit: see epilogue.h)
    const uint32_t nbase = (uint32_t)n * (uint32_t)P.in.sN;
    uint32_t off[KK];
    uint32_t mask = 0;
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
            const int iy = iy0 + ky, ix = ix0 + kx;
            const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
            off[ky * K + kx] = (nbase + (ok ? (uint32_t)(iy * W + ix) : 0u)) * 4u;  // bytes
            mask |= (ok ? 1u : 0u) << (ky * K + kx);
        }

    // V4 role: column quad qd (positions j4 .. j4+3 of one image row), channel slot cs
    const int qd = tid % Q, cs = tid / Q;
    const int j4 = min(j0 + 4 * qd, G.ncols - 4);
    const int n4 = j4 / G.P, q4 = j4 - n4 * G.P;
    const int oy4 = q4 / P.OW, ox4 = q4 - oy4 * P.OW;
    const int a4 = ox4 * S;  // 16-byte aligned window start (W % 4 == 0, ox4 % 4 == 0)
    const uint32_t nbase4 = (uint32_t)n4 * (uint32_t)P.in.sN;

    f32x16 acc[MTW][NTW];
#pragma unroll
    for (int t = 0; t < MTW; ++t)
#pragma unroll
        for (int u = 0; u < NTW; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;

    // Software pipeline over the channel chunks: the taps and 1x1 weights of chunk k+1 are
    // loaded into registers while the waves run chunk k's MFMAs, so the global-load latency of
    // every chunk after the first hides behind matrix work.
    constexpr int WPT = (FKC * BM + 255) / 256;  // 1x1 weights staged per thread per chunk
    float tap[V4 ? 1 : PER][V4 ? 1 : KK], win[V4 ? CPT : 1][V4 ? K : 1][V4 ? WL : 1], wreg[WPT];
    auto load_chunk = [&](int kc) {
        if constexpr (V4) {
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int c = kc + cs + CS * i;
                const float *pl = P.in.p + (size_t)(uint32_t)(c < Cin ? c : Cin - 1) * (uint32_t)P.in.sC + nbase4;
#pragma unroll
                for (int ky = 0; ky < K; ++ky) {
                    const int iy = oy4 * S - P.pad_t + ky;
                    const bool rok = iy >= 0 && iy < H;
                    const uint32_t rb = (uint32_t)(rok ? iy : 0) * (uint32_t)W;
#pragma unroll
                    for (int e = 0; e < PL; ++e) {  // left of the aligned part
                        const int x = a4 - PL + e;
                        const float v = pl[rb + (uint32_t)(x >= 0 ? x : 0)];
                        win[i][ky][e] = rok && x >= 0 ? v : 0.f;
                    }
#pragma unroll
                    for (int v4 = 0; v4 < NV; ++v4) {
                        const int x = a4 + 4 * v4;
                        const bool ok = rok && x < W;
                        const float4 v = *(const float4 *)(pl + rb + (uint32_t)(ok ? x : 0));
                        win[i][ky][PL + 4 * v4 + 0] = ok ? v.x : 0.f;
                        win[i][ky][PL + 4 * v4 + 1] = ok ? v.y : 0.f;
                        win[i][ky][PL + 4 * v4 + 2] = ok ? v.z : 0.f;
                        win[i][ky][PL + 4 * v4 + 3] = ok ? v.w : 0.f;
                    }
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int c = kc + dc + CPAR * i;
                const char *pl = (const char *)(P.in.p + (size_t)(uint32_t)(c < Cin ? c : Cin - 1) * (uint32_t)P.in.sC);
#pragma unroll
                for (int t = 0; t < KK; ++t) tap[i][t] = *(const float *)(pl + off[t]);
            }
        }
#pragma unroll
        for (int u = 0; u < WPT; ++u) {
            const int i = min(tid + 256 * u, FKC * BM - 1);
            const int r = i / BM, cc = i - r * BM;
            const int k = kc + r, m = m0 + cc;
            const float x = G.wt[(int64_t)(k < Cin ? k : Cin - 1) * G.Mpad + (m < G.Mpad ? m : 0)];
            wreg[u] = (k < Cin && m < G.Mpad) ? x : 0.f;
        }
    };
    load_chunk(0);
    for (int kc = 0; kc < Cin; kc += FKC) {
        if constexpr (V4) {
            float dv[CPT * 4];
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int c = kc + cs + CS * i;
                const int cl = c < Cin ? c : Cin - 1;
                const float *w = P.dw_w + cl * KK;
                const float b = P.dw_b[cl];
#pragma unroll
                for (int o = 0; o < 4; ++o) {
                    float a = b;
#pragma unroll
                    for (int ky = 0; ky < K; ++ky)
#pragma unroll
                        for (int kx = 0; kx < K; ++kx) a = __builtin_fmaf(w[ky * K + kx], win[i][ky][o * S + kx], a);
                    dv[4 * i + o] = a;
                }
            }
            apply_act_n<CPT * 4>(P.dw_act, dv, [&](int e) {
                const int c = kc + cs + CS * (e >> 2);
                return c < Cin ? c : Cin - 1;
            });
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int c = cs + CS * i;
                if (c < FKC) {
                    const bool ok = kc + c < Cin;
                    *(float4 *)&sD[c][4 * qd] = make_float4(ok ? dv[4 * i] : 0.f, ok ? dv[4 * i + 1] : 0.f,
                                                            ok ? dv[4 * i + 2] : 0.f, ok ? dv[4 * i + 3] : 0.f);
                }
            }
        } else {
            float dv[PER];
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int c = kc + dc + CPAR * i;
                const int cl = c < Cin ? c : Cin - 1;
                const float *w = P.dw_w + cl * KK;
                float a = P.dw_b[cl];
#pragma unroll
                for (int t = 0; t < KK; ++t) a = __builtin_fmaf(w[t], ((mask >> t) & 1u) ? tap[i][t] : 0.f, a);
                dv[i] = a;
            }
            apply_act_n<PER>(P.dw_act, dv, [&](int i) {
                const int c = kc + dc + CPAR * i;
                return c < Cin ? c : Cin - 1;
            });
#pragma unroll
            for (int i = 0; i < PER; ++i) sD[dc + CPAR * i][dj] = kc + dc + CPAR * i < Cin ? dv[i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < WPT; ++u) {
            const int i = tid + 256 * u;
            if (i < FKC * BM) (&sW[0][0])[i] = wreg[u];
        }
        __syncthreads();
        if (kc + FKC < Cin) load_chunk(kc + FKC);
#pragma unroll
        for (int s = 0; s < FKC / 2; ++s) {
            float a[MTW], b[NTW];
#pragma unroll
            for (int t = 0; t < MTW; ++t) a[t] = sW[2 * s + kh][(wm * MTW + t) * 32 + col];
#pragma unroll
            for (int u = 0; u < NTW; ++u) b[u] = sD[2 * s + kh][(wn * NTW + u) * 32 + col];
#pragma unroll
            for (int t = 0; t < MTW; ++t)
#pragma unroll
                for (int u = 0; u < NTW; ++u)
                    acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[u], acc[t][u], 0, 0, 0);
        }
        __syncthreads();
    }

#pragma unroll
    for (int u = 0; u < NTW; ++u) {
        const int j = j0 + (wn * NTW + u) * 32 + col;
        if (j >= G.ncols) continue;
        const int on = j / G.P, oq = j - on * G.P;
#pragma unroll
        for (int t = 0; t < MTW; ++t) epilogue_tile(G, acc[t][u], on, oq, m0 + (wm * MTW + t) * 32, kh);
    }
}

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

// a / b for 0 <= a < 2^22 through the f32 reciprocal, corrected to the exact quotient
__device__ __forceinline__ int qdiv(int a, int b, float inv_b) {
    int q = (int)((float)a * inv_b);
    const int r = a - q * b;
    q += r >= b ? 1 : 0;
    q -= r < 0 ? 1 : 0;
    return q;
}

__device__ const float4 zr_zero4 = {0.f, 0.f, 0.f, 0.f};  // LDS-DMA source of the zero slots

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

// LDS-DMA form of the MFMA dwpw for the stride-1 low-resolution layers (24^2 ... 6^2 planes
// with 64-256 channels), whose register-staged form waits on memory most of the time.  Per
// chunk of DFKC input channels one buffer receives, by global_load_lds_dwordx4 (no VGPRs, no
// staging instructions beyond the address math), the contiguous CNHW run of input each channel
// needs for the tile's BN columns (images are contiguous inside a channel: the run from the
// first needed row of the first image to the last needed row of the last one), the chunk's
// rows of the transposed 1x1 weights, and its depthwise weights and biases.  Two buffers: the
// next chunk's copy is in flight while this chunk's depthwise (from LDS) and MFMAs run; the
// barrier that publishes the depthwise tile to the MFMAs is a bare s_barrier, so it does not
// drain that copy.
// (MTW == 1: 4 waves per SIMD fit in 128 registers without spills; the hint moves the
// accumulators out of AGPRs -- 119 VGPRs instead of 119 + 16, i.e. 4 waves instead of 3 when
// the LDS plan leaves room for a fourth workgroup)
template <int K, int S, int WM, int MTW, int DFKC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MTW == 1 ? 4 : 1)))
void dwpw_dma_kernel(const DwPwParams P, int nct, int runmax, int bufsz) {
    constexpr int WN = 4 / WM, BN = WN * 32, BM = WM * MTW * 32, KK = K * K;
    constexpr int CPAR = 256 / BN, PER = DFKC / CPAR;
    constexpr int KKP = (DFKC * KK + 3) / 4 * 4;
    // [guard: 256 words] [2 x bufsz] [sD: DFKC x BN]; masked taps of the first run may index up
    // to pad_t * W + pad_l words before it, into the guard rather than out of the allocation
    extern __shared__ __attribute__((aligned(16))) float lds_all[];
    float *smem = lds_all + 256;
    float *sD = smem + 2 * bufsz;
    const GemmParams &G = P.g;

    const int cpx = gridDim.x >> 3;  // gridDim.x is a multiple of 8
    const int tile = (blockIdx.x & 7) * cpx + (blockIdx.x >> 3);
    if (tile >= nct) return;  // whole workgroup, before any barrier
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kh = lane >> 5, col = lane & 31;
    const int wm = wave % WM, wn = wave / WM;
    const int j0 = tile * BN, m0 = blockIdx.y * BM;
    const int Cin = G.K, H = P.in.H, W = P.in.W, Pin = H * W, OW = P.OW, Pq = G.P;
    const int pt = P.pad_t, pl = P.pad_l;

    // the input run of this tile (floats from a channel's base; 16-byte aligned ends)
    const int ja = j0, jb = min(j0 + BN, G.ncols) - 1;
    const int na = ja / Pq, qa = ja - na * Pq, nb = jb / Pq, qb = jb - nb * Pq;
    const int ya = max(qa / OW * S - pt, 0), yb = min(qb / OW * S - pt + K - 1, H - 1);
    const int s0 = (na * Pin + ya * W) & ~3;
    const int e0 = (nb * Pin + (yb + 1) * W + 3) & ~3;
    const int run4 = (e0 - s0) >> 2;  // <= runmax / 4

    // slot regions of a buffer (16-byte slots)
    const int rq = runmax >> 2;
    const int r1 = DFKC * rq, r2 = r1 + DFKC * (BM / 4), r3 = r2 + KKP / 4, r4 = r3 + DFKC / 4;
    const float inv_rq = 1.f / (float)rq;
    const int nwi = bufsz >> 8;  // 64-slot DMA wave-instructions per buffer
    auto stage = [&](int kc, float *dst) {
        for (int wi = wave; wi < nwi; wi += 4) {
            const int sl = wi * 64 + lane;
            const float *src = (const float *)&zr_zero4;
            if (sl < r1) {
                const int c = qdiv(sl, rq, inv_rq), i = sl - c * rq;
                if (kc + c < Cin && i < run4)
                    src = P.in.p + (size_t)(uint32_t)(kc + c) * (uint32_t)P.in.sC + (uint32_t)(s0 + 4 * i);
            } else if (sl < r2) {
                const int r = (sl - r1) / (BM / 4), i = sl - r1 - r * (BM / 4);
                if (kc + r < G.Kpad && m0 + 4 * i < G.Mpad)
                    src = G.wt + (size_t)(uint32_t)(kc + r) * (uint32_t)G.Mpad + (uint32_t)(m0 + 4 * i);
            } else if (sl < r3) {
                const int i = sl - r2;
                if (kc * KK + 4 * i < Cin * KK) src = P.dw_w + kc * KK + 4 * i;
            } else if (sl < r4) {
                const int i = sl - r3;
                if (kc + 4 * i < Cin) src = P.dw_b + kc + 4 * i;
            }
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(dst + wi * 256), 16, 0, 0);
        }
    };

    // depthwise role: column dj, channels dc, dc + CPAR, ... of each chunk
    const int dj = tid % BN;
    int dc = tid / BN;
    if constexpr (BN >= 64) dc = __builtin_amdgcn_readfirstlane(dc);  // one channel per wave
    const int jd = min(j0 + dj, G.ncols - 1);
    const int n = jd / Pq, q = jd - n * Pq;
    const int oy = q / OW, ox = q - oy * OW;
    const int iy0 = oy * S - pt, ix0 = ox * S - pl;
    const int tb = n * Pin + iy0 * W + ix0 - s0;  // run index of tap (0, 0) (may be < 0 when masked)
    uint32_t mask = 0;
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
            const int iy = iy0 + ky, ix = ix0 + kx;
            mask |= (iy >= 0 && iy < H && ix >= 0 && ix < W ? 1u : 0u) << (ky * K + kx);
        }

    f32x16 acc[MTW];
#pragma unroll
    for (int t = 0; t < MTW; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    stage(0, smem);
    for (int kc = 0, it = 0; kc < Cin; kc += DFKC, ++it) {
        const float *buf = smem + (it & 1) * bufsz;
        __syncthreads();  // vmcnt(0) + barrier: this chunk has landed; last chunk's readers are done
        if (kc + DFKC < Cin) stage(kc + DFKC, smem + ((it + 1) & 1) * bufsz);
        const float *sIn = buf, *sW = buf + DFKC * runmax, *sDW = sW + DFKC * BM, *sDB = sDW + KKP;
        float dv[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int c = dc + CPAR * i;
            const float *t0 = sIn + c * runmax + tb;
            const float *w = sDW + c * KK;
            float a = sDB[c];
#pragma unroll
            for (int ky = 0; ky < K; ++ky)
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const int t = ky * K + kx;
                    const float x = t0[ky * W + kx];
                    a = __builtin_fmaf(w[t], ((mask >> t) & 1u) ? x : 0.f, a);
                }
            dv[i] = a;
        }
        apply_act_n<PER>(P.dw_act, dv, [&](int i) {
            const int c = kc + dc + CPAR * i;
            return c < Cin ? c : Cin - 1;
        });
#pragma unroll
        for (int i = 0; i < PER; ++i) sD[(dc + CPAR * i) * BN + dj] = kc + dc + CPAR * i < Cin ? dv[i] : 0.f;
        // publish sD without draining the next chunk's DMA (a __syncthreads would wait vmcnt(0))
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int s = 0; s < DFKC / 2; ++s) {
            float a[MTW];
#pragma unroll
            for (int t = 0; t < MTW; ++t) a[t] = sW[(2 * s + kh) * BM + (wm * MTW + t) * 32 + col];
            const float b = sD[(2 * s + kh) * BN + wn * 32 + col];
#pragma unroll
            for (int t = 0; t < MTW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b, acc[t], 0, 0, 0);
        }
    }

    const int j = j0 + wn * 32 + col;
    if (j >= G.ncols) return;
    const int on = j / Pq, oq = j - on * Pq;
#pragma unroll
    for (int t = 0; t < MTW; ++t) epilogue_tile(G, acc[t], on, oq, m0 + (wm * MTW + t) * 32, kh);
}

bool dwpw_supported(int k, int stride) { return (k == 3 || k == 5) && (stride == 1 || stride == 2); }

namespace {

struct DwPwLayout {
    int wm, mtw, ntw;
    int bm() const { return wm * mtw * 32; }
    int bn() const { return (4 / wm) * ntw * 32; }
};
// the instantiated layouts (BM x BN): 32x128 64x128 96x128 128x128 | 64x64 128x64 256x64 |
// 128x32 256x32
constexpr DwPwLayout kLayouts[] = {{1, 1, 1}, {1, 2, 1}, {1, 3, 1}, {1, 4, 1}, {2, 1, 1},
                                   {2, 2, 1}, {2, 4, 1}, {4, 1, 1}, {4, 2, 1}};

// The V4 depthwise form (see dwpw_kernel) applies when rows split into aligned quads and the
// layer uses the models' TF-style pads.
static bool v4_ok(const DwPwParams &p) {
    const int pl = p.stride == 1 ? p.k / 2 : p.k / 2 - 1;
    return form_on(FORM_V4) && p.OW % 4 == 0 && p.in.W % 4 == 0 && p.pad_l == pl && p.pad_t == pl &&
           p.g.ncols % 4 == 0 && p.g.P % 4 == 0;
}

// LDS bytes of the DMA form for this layer and tile (0 when it does not apply): the longest
// input run any BN-column tile needs, rounded to 16 B, and whole 1 KiB DMA wave-instructions.
template <int K, int S, int WM, int MTW, int DFKC>
static size_t dma_plan(const DwPwParams &p, int *runmax, int *bufsz) {
    constexpr int BN = (4 / WM) * 32, BM = WM * MTW * 32, KKP = (DFKC * K * K + 3) / 4 * 4;
    const int H = p.in.H, W = p.in.W, Pin = H * W, Pq = p.g.P, OW = p.OW;
    // (runs are rounded out to 16-B ends inside the channel plane: sC % 4 == 0 leaves room)
    if (!form_on(FORM_DMA) || p.in.sN != Pin || p.in.sC % 4 || p.g.K % 4 ||
        ((uintptr_t)p.in.p | (uintptr_t)p.g.wt | (uintptr_t)p.dw_w | (uintptr_t)p.dw_b) % 16)
        return 0;
    int rm = 0;
    for (int j0 = 0; j0 < p.g.ncols; j0 += BN) {  // tiles repeat with the image period
        const int jb = std::min(j0 + BN, p.g.ncols) - 1;
        const int na = j0 / Pq, qa = j0 - na * Pq, nb = jb / Pq, qb = jb - nb * Pq;
        const int ya = std::max(qa / OW * S - p.pad_t, 0), yb = std::min(qb / OW * S - p.pad_t + K - 1, H - 1);
        const int s0 = (na * Pin + ya * W) & ~3, e0 = (nb * Pin + (yb + 1) * W + 3) & ~3;
        rm = std::max(rm, e0 - s0);
        if (na >= 4 && (j0 % Pq) == 0) break;  // the pattern has repeated (whole images seen)
    }
    const int words = DFKC * rm + DFKC * BM + KKP + DFKC;
    *runmax = rm;
    *bufsz = (words + 255) / 256 * 256;
    if (p.pad_t * W + p.pad_l > 256) return 0;  // the guard in front of the buffers
    const size_t lds = sizeof(float) * (256 + 2 * (size_t)*bufsz + DFKC * BN);
    return lds <= 80 * 1024 ? lds : 0;
}

template <int K, int S, int WM, int MTW>
const char *dwpw_go(const DwPwParams &p, hipStream_t s) {
    constexpr int BN = (4 / WM) * 32, BM = WM * MTW * 32;
    const int nct = (p.g.ncols + BN - 1) / BN;
    const int mb = (p.g.Mpad + BM - 1) / BM;
    dim3 grid((nct + 7) / 8 * 8, mb);
    int runmax = 0, bufsz = 0;
    if (const size_t lds = dma_plan<K, S, WM, MTW, 16>(p, &runmax, &bufsz)) {
        hipLaunchKernelGGL((dwpw_dma_kernel<K, S, WM, MTW, 16>), grid, dim3(256), lds, s, p, nct, runmax, bufsz);
        return kernel_name("dwpw_dma_kernel<%d,%d,%d,%d,16>", K, S, WM, MTW);
    }
    const bool v4 = v4_ok(p);
    if (v4) hipLaunchKernelGGL((dwpw_kernel<K, S, WM, MTW, 1, true>), grid, dim3(256), 0, s, p, nct);
    else hipLaunchKernelGGL((dwpw_kernel<K, S, WM, MTW, 1, false>), grid, dim3(256), 0, s, p, nct);
    return kernel_name("dwpw_kernel<%d,%d,%d,%d,1,%s>", K, S, WM, MTW, v4 ? "true" : "false");
}

template <int K, int S>
const char *dwpw_layout(const DwPwParams &p, const DwPwLayout &l, hipStream_t s) {
    switch (l.wm * 10 + l.mtw) {
    case 11: return dwpw_go<K, S, 1, 1>(p, s);
    case 12: return dwpw_go<K, S, 1, 2>(p, s);
    case 13: return dwpw_go<K, S, 1, 3>(p, s);
    case 14: return dwpw_go<K, S, 1, 4>(p, s);
    case 21: return dwpw_go<K, S, 2, 1>(p, s);
    case 22: return dwpw_go<K, S, 2, 2>(p, s);
    case 24: return dwpw_go<K, S, 2, 4>(p, s);
    case 41: return dwpw_go<K, S, 4, 1>(p, s);
    default: return dwpw_go<K, S, 4, 2>(p, s);
    }
}

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
    const bool small = db && !(CO == 32 && fit8);
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

// Layout choice.  High-resolution planes with few channels take the VALU form; otherwise (MFMA
// form): no M split unless Mpad > 256, at most 1/3 padded rows; among those, the widest
// column tile that still gives >= 4 workgroups per CU (else the most workgroups).
const char *launch_dwpw(const DwPwParams &p, hipStream_t s) {
    if (valu_form(p)) {
        if (p.k == 3) return p.stride == 1 ? dwpw_valu_co<3, 1>(p, s) : dwpw_valu_co<3, 2>(p, s);
        return p.stride == 1 ? dwpw_valu_co<5, 1>(p, s) : dwpw_valu_co<5, 2>(p, s);
    }
    // workgroups one launch should reach (ZARU_HIP_MINWGS overrides it for layout sweeps)
    static const int64_t min_wgs = [] {
        const char *e = std::getenv("ZARU_HIP_MINWGS");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (int64_t)(v > 0 ? v : 1024);
    }();
    const DwPwLayout *best = nullptr;
    int64_t best_wgs = 0;
    for (const DwPwLayout &l : kLayouts) {
        const int mb = (p.g.Mpad + l.bm() - 1) / l.bm();
        if (mb > 1 && l.bm() < 256) continue;
        if ((int64_t)mb * l.bm() * 3 > (int64_t)p.g.Mpad * 4 && p.g.Mpad <= 256) continue;
        const int64_t wgs = (int64_t)((p.g.ncols + l.bn() - 1) / l.bn()) * mb;
        bool better;
        if (!best) better = true;
        else if ((wgs >= min_wgs) != (best_wgs >= min_wgs)) better = wgs >= min_wgs;
        else if (wgs >= min_wgs) better = l.bn() > best->bn() || (l.bn() == best->bn() && l.bm() < best->bm());
        else better = wgs > best_wgs || (wgs == best_wgs && l.bm() < best->bm());
        if (better) {
            best = &l;
            best_wgs = wgs;
        }
    }
    if (!best) {
        // no tile height wastes <= 1/3 of its rows without an M split (e.g. Mpad = 160, the
        // 144-channel blocks of BlazeFace full range): the unsplit tile with the fewest padded
        // rows, else the tallest split one
        int waste = 1 << 30;
        for (const DwPwLayout &l : kLayouts) {
            const int mb = (p.g.Mpad + l.bm() - 1) / l.bm();
            if (mb > 1 && l.bm() < 256) continue;
            const int w = mb * l.bm() - p.g.Mpad;
            if (w < waste) {
                waste = w;
                best = &l;
            }
        }
    }
    if (p.k == 3) return p.stride == 1 ? dwpw_layout<3, 1>(p, *best, s) : dwpw_layout<3, 2>(p, *best, s);
    return p.stride == 1 ? dwpw_layout<5, 1>(p, *best, s) : dwpw_layout<5, 2>(p, *best, s);
}

}  // namespace zr
