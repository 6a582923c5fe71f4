// dwpw_mfma.h -- the depthwise KxK -> 1x1 BlazeBlock (inverted-residual tail) as one launch
// for the low-resolution, many-channel layers: the depthwise output of a column tile lives only
// in LDS and feeds an f32 MFMA GEMM (v_mfma_f32_32x32x2_f32, exact f32) whose epilogue applies
// bias, activation, residual (+pad/+pool) and activation.
// Reference: the Conv nodes of the four ONNX graphs that ORT/tract execute at
// crates/zaru/src/nn/mod.rs:483-533 (the BlazeBlocks).
#pragma once
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "../runtime/zr_kernels.h"
#include "act.h"
#include "epilogue.h"
#include "group.h"
#include "lds_dma.h"

namespace zr {

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
    if (G.nact && j0 >= *G.nact * G.P) return;  // images past the device count
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


// LDS-DMA form of the MFMA dwpw for the low-resolution layers (24^2 ... 3^2 planes with 64-256
// channels), whose register-staged form waits on memory most of the time.  Per chunk of DFKC
// input channels one LDS buffer receives, by global_load_lds_dwordx4 (no VGPRs, no staging
// instructions beyond the address math), the contiguous CNHW run of input each channel needs for
// the tile's BN columns (images are contiguous inside a channel: the run from the first needed
// row of the first image to the last needed row of the last one) and the chunk's depthwise
// weights and biases.  Two buffers: the next chunk's copy is in flight while this chunk's
// depthwise (from LDS) and MFMAs run; the barrier that publishes the depthwise tile to the MFMAs
// is a bare s_barrier, so it does not drain that copy.
// WREG (MTW == 1): the 1x1 weights (the MFMA A operand) do not pass through LDS: each wave loads
// its own 32-row slice of the chunk's transposed weights into registers one chunk ahead
// (coalesced 128-B rows, L2 hits -- every workgroup reads the same few KiB).  Staged in LDS they
// are ~60 % of a chunk's copy; in registers they leave room for 32-channel chunks at the same
// occupancy.  With MTW = 2 the two register sets would cost a wave per SIMD, so
// those layouts stage the weights' chunk rows in the DMA buffer.
// (MTW == 1: 4 waves per SIMD fit in 128 registers without spills)
// RT > 0 (form "rt"): the depthwise runs as row tasks instead of one tap read per output and tap.
// A task is RT adjacent outputs of one output row of one channel; it reads each of its K input
// rows once as a window of (RT - 1) * S + K floats with 8-byte LDS reads (RT * K FMAs per row for
// ceil(window / 2) reads, where the per-output form issues K reads per row per output), keeps the
// channel's K^2 weights in registers for its NRT tasks, and masks the padding statically: a row
// outside the image reads a zeroed LDS block, the first / last segment of a row zeroes its PL / PR
// window floats.  The arithmetic is the per-output form's: bias + fmaf over the taps in (ky, kx)
// order, masked taps as fmaf(w, 0, a) -- so the bits are too (tests/test_gpu_forms.py, -rt).
// RD = 1 (form "pin", dwpw_dma_pin_kernel; a task step RT * S that is a multiple of 4, W % 4 == 0):
// the window rows are read as whole 16-byte vectors from 16-byte aligned starts (ds_read_b128).
// Left alone the compiler drops a window's unused first / last float and re-pairs the rest into
// ds_read2_b32 -- two 4-byte reads per lane, banks mod 32, so lanes whose windows are 16 B apart
// meet 4-way conflicts; an empty asm that takes each loaded vector whole keeps the full read, and
// b128's 16-lane groups cover a 256-byte bank row with 16-byte-apart lanes where b64's 32-lane
// groups wrap it twice (PMC: FaceMesh 24^2 4.33 -> 0.13 conflict cycles per LDS instruction).
// A 4-wide task also stores its outputs as one ds_write_b128.
template <int K, int S, int WM, int MTW, int DFKC, int RT, int RD = 0>
__device__ __forceinline__ void dwpw_dma_body(const DwPwParams &P, int nct, int runmax, int bufsz, int bx, int by, int gx) {
    constexpr int WN = 4 / WM, BN = WN * 32, BM = WM * MTW * 32, KK = K * K;
    constexpr int CPAR = 256 / BN, PER = DFKC / CPAR;
    constexpr int KKP = (DFKC * KK + 3) / 4 * 4;
    constexpr bool WREG = MTW == 1;
    // [guard: 256 words] [2 x bufsz] [sD: DFKC x BN]; masked taps of the first run may index up
    // to pad_t * W + pad_l words before it, into the guard rather than out of the allocation
    extern __shared__ __attribute__((aligned(16))) float lds_all[];
    float *smem = lds_all + 256;
    float *sD = smem + 2 * bufsz;
    const GemmParams &G = P.g;

    const int cpx = gx >> 3;  // the grid's x extent is a multiple of 8
    const int tile = (bx & 7) * cpx + (bx >> 3);
    if (tile >= nct) return;  // whole workgroup, before any barrier
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kh = lane >> 5, col = lane & 31;
    const int wm = wave % WM, wn = wave / WM;
    const int j0 = tile * BN, m0 = by * BM;
    if (G.nact && j0 >= *G.nact * G.P) return;  // images past the device count
    const int Cin = G.K, H = P.in.H, W = P.in.W, Pin = H * W, OW = P.OW, Pq = G.P;
    const int pt = P.pad_t, pl = P.pad_l;

    // the input run of this tile (floats from a channel's base; 16-byte aligned ends)
    const int ja = j0, jb = min(j0 + BN, G.ncols) - 1;
    const int na = ja / Pq, qa = ja - na * Pq, nb = jb / Pq, qb = jb - nb * Pq;
    const int ya = max(qa / OW * S - pt, 0), yb = min(qb / OW * S - pt + K - 1, H - 1);
    const int s0 = (na * Pin + ya * W) & ~3;
    const int e0 = (nb * Pin + (yb + 1) * W + 3) & ~3;
    const int run4 = (e0 - s0) >> 2;  // <= runmax / 4

    // slot regions of a buffer (16-byte slots): input runs | 1x1 weight rows (!WREG) |
    // depthwise weights | biases
    const int rq = runmax >> 2;
    const int r1 = DFKC * rq, r2 = r1 + (WREG ? 0 : DFKC * (BM / 4)), r3 = r2 + KKP / 4, r4 = r3 + DFKC / 4;
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
    // this lane's A fragments of a chunk: W^T[kc + 2s + kh][row t*32 + col of the wave's slice];
    // rows past Kpad / Mpad are the zero padding (clamped address + select, no branch)
    const int mw = m0 + wm * MTW * 32 + col;
    constexpr int WT = WREG ? MTW : 1, WS = WREG ? DFKC / 2 : 1;
    auto wload = [&](int kc, float (&w)[WT][WS]) {
        if constexpr (!WREG) return;
#pragma unroll
        for (int s = 0; s < DFKC / 2; ++s) {
            const int k = kc + 2 * s + kh;
#pragma unroll
            for (int t = 0; t < MTW; ++t) {
                const bool ok = k < G.Kpad && mw + t * 32 < G.Mpad;
                const float x = G.wt[ok ? (uint32_t)k * (uint32_t)G.Mpad + (uint32_t)(mw + t * 32) : 0u];
                w[t][s] = ok ? x : 0.f;
            }
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

    // row-task geometry (RT > 0): thread tid runs NRT tasks of one channel (SEGS % NRT == 0), SPT
    // threads per channel; its task r is segment r * SPT + tid % SPT, so the lanes of a wave read
    // adjacent windows (8-byte reads of adjacent lanes RT * S floats apart: at RT = 2, S = 1 no two
    // lanes of a half-wave share a bank).  Per task: the run index of its aligned window start in
    // row ky = 0, the rows inside the image, and whether it is the first / last segment of its row
    constexpr int RTE = RT > 0 ? RT : 1;
    static_assert(RD == 0 || (RTE * S) % 4 == 0, "pinned reads: 16-byte window steps");
    constexpr bool V16 = RD > 0;                                    // 16-byte window reads
    constexpr int VW = V16 ? 4 : 2;                                 // floats per window read
    constexpr int PLx = DwPad<K, S>::L, OFF = V16 ? (4 - PLx % 4) % 4 : PLx & 1;
    constexpr int WW = (RTE - 1) * S + K, PR = WW - RTE * S - PLx;  // window floats, right pad
    constexpr int NB64 = (OFF + WW + VW - 1) / VW;                  // reads per window row
    constexpr int SEGS = BN / RTE, TASKS = DFKC * SEGS, NRT = TASKS > 256 ? TASKS / 256 : 1;
    static_assert(RT == 0 || (RT % 2 == 0 && BN % RT == 0 && SEGS % NRT == 0 && (TASKS <= 256 || TASKS % 256 == 0)),
                  "row-task layout");
    constexpr int SPT = SEGS / NRT;
    const int rt_c = RT > 0 ? tid / SPT : 0, rt_g = tid % SPT;
    const bool rt_on = RT > 0 && tid * NRT < TASKS;
    int rt_base[NRT];
    uint32_t rt_vm[NRT];
    bool rt_first[NRT], rt_last[NRT], rt_ok[NRT];
    if constexpr (RT > 0) {
        if (tid < 16) reinterpret_cast<float4 *>(lds_all)[tid] = make_float4(0.f, 0.f, 0.f, 0.f);  // the zero rows
#pragma unroll
        for (int r = 0; r < NRT; ++r) {
            const int g = r * SPT + rt_g;
            const int j = j0 + g * RT;
            rt_ok[r] = rt_on && j < G.ncols;
            const int jj = rt_ok[r] ? j : 0;
            const int tn = jj / Pq, tq = jj - tn * Pq, toy = tq / OW, tox = tq - toy * OW;
            const int iy0 = toy * S - pt;
            rt_base[r] = tn * Pin + iy0 * W + tox * S - PLx - OFF - s0;
            uint32_t vm = 0;
#pragma unroll
            for (int ky = 0; ky < K; ++ky) vm |= (iy0 + ky >= 0 && iy0 + ky < H ? 1u : 0u) << ky;
            rt_vm[r] = vm;
            rt_first[r] = tox == 0;
            rt_last[r] = tox + RT == OW;
        }
    }

    f32x16 acc[MTW];
#pragma unroll
    for (int t = 0; t < MTW; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    float wa[WT][WS], wnx[WT][WS];
    stage(0, smem);
    wload(0, wa);
    for (int kc = 0, it = 0; kc < Cin; kc += DFKC, ++it) {
        const float *buf = smem + (it & 1) * bufsz;
        __syncthreads();  // vmcnt(0) + barrier: this chunk has landed; last chunk's readers are done
        if (kc + DFKC < Cin) {
            stage(kc + DFKC, smem + ((it + 1) & 1) * bufsz);
            wload(kc + DFKC, wnx);
        }
        const float *sIn = buf, *sW = buf + DFKC * runmax, *sDW = sW + (WREG ? 0 : DFKC * BM), *sDB = sDW + KKP;
        if constexpr (RT > 0) {
            if (rt_on) {
                const int c = rt_c;
                float wr[KK];
#pragma unroll
                for (int t = 0; t < KK; ++t) wr[t] = sDW[c * KK + t];
                const float bb = sDB[c];
                const bool live = kc + c < Cin;
                const float *chan = sIn + c * runmax;
#pragma unroll
                for (int r = 0; r < NRT; ++r) {
                    float a[RTE];
#pragma unroll
                    for (int o = 0; o < RTE; ++o) a[o] = bb;
#pragma unroll
                    for (int ky = 0; ky < K; ++ky) {
                        const float *row = ((rt_vm[r] >> ky) & 1u) ? chan + rt_base[r] + ky * W : lds_all;
                        float x[VW * NB64];
#pragma unroll
                        for (int e = 0; e < NB64; ++e) {
                            if constexpr (RD == 0) {
                                const float2 v = *reinterpret_cast<const float2 *>(row + 2 * e);
                                x[2 * e] = v.x;
                                x[2 * e + 1] = v.y;
                            } else {
                                typedef float fv __attribute__((ext_vector_type(VW)));
                                fv v = *reinterpret_cast<const fv *>(row + VW * e);
                                asm("" : "+v"(v));  // the whole vector: no narrowed / re-paired reads
#pragma unroll
                                for (int i = 0; i < VW; ++i) x[VW * e + i] = v[i];
                            }
                        }
#pragma unroll
                        for (int e = 0; e < PLx; ++e) x[OFF + e] = rt_first[r] ? 0.f : x[OFF + e];
#pragma unroll
                        for (int e = WW - PR; e < WW; ++e) x[OFF + e] = rt_last[r] ? 0.f : x[OFF + e];
#pragma unroll
                        for (int kx = 0; kx < K; ++kx)
#pragma unroll
                            for (int o = 0; o < RTE; ++o) a[o] = __builtin_fmaf(wr[ky * K + kx], x[OFF + o * S + kx], a[o]);
                    }
                    apply_act_n<RTE>(P.dw_act, a, [&](int) { return live ? kc + c : Cin - 1; });
                    float *dst = sD + c * BN + (r * SPT + rt_g) * RTE;
                    if constexpr (RD > 0 && RTE % 4 == 0) {
                        const bool w = live && rt_ok[r];
#pragma unroll
                        for (int o = 0; o < RTE; o += 4)
                            *reinterpret_cast<float4 *>(dst + o) =
                                make_float4(w ? a[o] : 0.f, w ? a[o + 1] : 0.f, w ? a[o + 2] : 0.f, w ? a[o + 3] : 0.f);
                    } else {
#pragma unroll
                        for (int o = 0; o < RTE; o += 2)
                            *reinterpret_cast<float2 *>(dst + o) =
                                make_float2(live && rt_ok[r] ? a[o] : 0.f, live && rt_ok[r] ? a[o + 1] : 0.f);
                    }
                }
            }
        } else {
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
        }
        // publish sD without draining the next chunk's DMA and weight loads (a __syncthreads
        // would wait vmcnt(0))
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int s = 0; s < DFKC / 2; ++s) {
            const float b = sD[(2 * s + kh) * BN + wn * 32 + col];
#pragma unroll
            for (int t = 0; t < MTW; ++t) {
                float a;
                if constexpr (WREG) a = wa[t][s];
                else a = sW[(2 * s + kh) * BM + (wm * MTW + t) * 32 + col];
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
            }
        }
        if constexpr (WREG) {
#pragma unroll
            for (int t = 0; t < WT; ++t)
#pragma unroll
                for (int s = 0; s < WS; ++s) wa[t][s] = wnx[t][s];
        }
    }

    const int j = j0 + wn * 32 + col;
    if (j >= G.ncols) return;
    const int on = j / Pq, oq = j - on * Pq;
#pragma unroll
    for (int t = 0; t < MTW; ++t) {
        // opaque row base / half: otherwise the compiler hoists every row's channel index and
        // bias / residual address out of the chunk loop and holds them across it
        int mb = m0 + (wm * MTW + t) * 32, h = kh;
        asm volatile("" : "+v"(mb), "+v"(h));
        epilogue_tile(G, acc[t], on, oq, mb, h);
    }
}

// 4 waves per SIMD (<= 128 VGPRs) where the layout fits them: MTW = 1, and MTW = 2 at 3x3
// (BlazeFace's 16^2 blocks 48.6 -> 46.0 us at 341 images; the palm's 5x5 MTW-2 layouts measured
// 1-5 % slower at 4 waves, with 2-53 spilled registers: profiles/r05_layers/)
template <int K, int WM, int MTW> constexpr int dma_waves(int rt) {
    return MTW == 1 || (MTW == 2 && K == 3) ? 4 : rt > 0 ? 2 : 1;
}
template <int K, int S, int WM, int MTW, int DFKC, int RT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(dma_waves<K, WM, MTW>(RT))))
void dwpw_dma_kernel(const DwPwParams P, int nct, int runmax, int bufsz) {
    dwpw_dma_body<K, S, WM, MTW, DFKC, RT>(P, nct, runmax, bufsz, blockIdx.x, blockIdx.y, gridDim.x);
}
// form "pin": the row-task reads at full width (RD = 1 above)
template <int K, int S, int WM, int MTW, int DFKC, int RT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(dma_waves<K, WM, MTW>(RT))))
void dwpw_dma_pin_kernel(const DwPwParams P, int nct, int runmax, int bufsz) {
    dwpw_dma_body<K, S, WM, MTW, DFKC, RT, 1>(P, nct, runmax, bufsz, blockIdx.x, blockIdx.y, gridDim.x);
}

// sibling layers in one launch (group.h): a0 = nct, a1 = runmax, a2 = bufsz of each part
template <int K, int S, int WM, int MTW, int DFKC, int RT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(dma_waves<K, WM, MTW>(RT))))
void dwpw_dma_group_kernel(const LaunchGroup<DwPwParams> G) {
    const GroupSlot t = group_slot(G);
    dwpw_dma_body<K, S, WM, MTW, DFKC, RT>(G.p[t.g], G.a0[t.g], G.a1[t.g], G.a2[t.g], t.bx, t.by, G.gx[t.g]);
}

struct DwPwLayout {
    int wm, mtw, ntw;
    int bm() const { return wm * mtw * 32; }
    int bn() const { return (4 / wm) * ntw * 32; }
};
// the instantiated layouts (BM x BN): 32x128 64x128 96x128 128x128 | 64x64 128x64 256x64 |
// 128x32 256x32
constexpr DwPwLayout kLayouts[] = {{1, 1, 1}, {1, 2, 1}, {1, 3, 1}, {1, 4, 1}, {2, 1, 1},
                                   {2, 2, 1}, {2, 4, 1}, {4, 1, 1}, {4, 2, 1}};

namespace {

// The V4 depthwise form (see dwpw_kernel) applies when rows split into aligned quads and the
// layer uses the models' TF-style pads.
static bool v4_ok(const DwPwParams &p) {
    const int pl = p.stride == 1 ? p.k / 2 : p.k / 2 - 1;
    return form_on(FORM_V4) && p.OW % 4 == 0 && p.in.W % 4 == 0 && p.pad_l == pl && p.pad_t == pl &&
           p.g.ncols % 4 == 0 && p.g.P % 4 == 0;
}

// LDS bytes of the DMA form for this layer and tile (0 when it does not apply): the longest
// input run any BN-column tile needs, rounded to 16 B, and whole 1 KiB DMA wave-instructions.
// LDS bytes for a channel stride of rm words (0: over the 80 KiB two workgroups per CU leave)
template <int K, int WM, int MTW, int DFKC>
static size_t dma_lds(int rm, int *bufsz) {
    constexpr int BN = (4 / WM) * 32, BM = WM * MTW * 32, KKP = (DFKC * K * K + 3) / 4 * 4;
    const int words = DFKC * rm + (MTW == 1 ? 0 : DFKC * BM) + KKP + DFKC;  // (WREG: no 1x1 weights)
    *bufsz = (words + 255) / 256 * 256;
    const size_t lds = sizeof(float) * (256 + 2 * (size_t)*bufsz + DFKC * BN);
    return lds <= 80 * 1024 ? lds : 0;
}

template <int K, int S, int WM, int MTW, int DFKC>
static size_t dma_plan(const DwPwParams &p, int *runmax, int *bufsz) {
    constexpr int BN = (4 / WM) * 32;
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
    *runmax = rm;
    if (p.pad_t * W + p.pad_l > 256) return 0;  // the guard in front of the buffers
    return dma_lds<K, WM, MTW, DFKC>(rm, bufsz);
}

// the widest channel chunk the DMA form may use (ZARU_HIP_DFKC: 16 / 32 / 64, for A/B runs)
static int dfkc_env() {
    static const int v = [] {
        const char *e = std::getenv("ZARU_HIP_DFKC");
        const long x = e ? std::strtol(e, nullptr, 10) : 0;
        return x >= 64 ? 64 : x >= 32 ? 32 : x > 0 ? 16 : 0;
    }();
    return v;
}

// Channel chunk of the 3x3 MTW = 1 layouts: 32 for launches of < 512 workgroups (FaceMesh's
// 6^2 / 3^2 blocks at 341 images: half the dependent DMA round trips of a workgroup that is
// alone on its CU, 18.9 -> 17.0 us at 3^2, profiles/r04_layers/), else 16 (at 12^2 and up the
// wider chunk's DMA costs more than the barriers it saves: r03).  ZARU_HIP_DFKC forces one.
static int dfkc_for(int wgs, int cin) {
    if (const int e = dfkc_env()) return e;
    return wgs < 512 && cin >= 64 ? 32 : 16;  // (32 channels in one chunk measured slower: 12.9 -> 15.2 us)
}

// Outputs per row task of the DMA form (0: the per-output depthwise).  R_hi = DFKC * BN / 256 keeps
// every thread busy with one task per NRT; R_hi / 2 when the output width does not split into R_hi
// segments.  Needs the models' TF-style padding with W = OW * S (so a row's first / last segment
// holds all of its padding) and an even R (8-byte aligned windows: even W and run starts).
// the widest row task an instance is built for: DFKC * BN / 256, capped where the window and the
// K^2 weights would cost occupancy next to the accumulators (5x5 at MTW = 1 and MTW >= 3: 2, else 8;
// the hand 28^2 5x5 block at 4-wide 16-byte-read tasks: 145 -> 200 us, profiles/r06_layers/
// hand_landmark_lite_341_k5rt4_vs_2.txt).
// MTW = 2: 4 (an 8-wide task's lanes read windows 32 B apart: 4-way bank conflicts on ds_read_b64;
// 4-wide, 16 B apart: 2-way.  The palm 48^2 5x5 blocks: 219 -> 210 us at 256 frames,
// profiles/r05_layers/; FaceMesh's 24^2 3x3 blocks: 48.1 / 47.8 -> 43.9 / 42.3 us at 256 images,
// profiles/r06_layers/face_landmark_256_rtcap4_vs_8.txt; 2-wide tasks there: per-output form, slower)
constexpr int rt_hi(int K, int MTW, int r) {
    return r < 2 ? 2 : (MTW == 1 && K == 5) || MTW >= 3 ? 2 : MTW == 2 && r > 4 ? 4 : r > 8 ? 8 : r;
}

// A/B knob (bitwise neutral, like the form switches): ZARU_HIP_RT_CAP = the widest row task
static int rt_cap() {
    static const int v = [] {
        const char *e = std::getenv("ZARU_HIP_RT_CAP");
        return e ? (int)std::strtol(e, nullptr, 10) : 0;
    }();
    return v;
}

template <int K, int S>
static int rt_for(const DwPwParams &p, int bn, int r_hi) {
    if (!form_on(FORM_RT) || p.pad_l != DwPad<K, S>::L || p.pad_t != DwPad<K, S>::L || p.in.W != p.OW * S) return 0;
    for (int r = r_hi; r >= 2 && r >= r_hi / 2; r /= 2)
        if ((rt_cap() < 2 || r <= rt_cap()) && p.OW % r == 0 && bn % r == 0) return r;
    return 0;
}

static bool dma_pad_on() {
    static const bool v = [] {
        const char *e = std::getenv("ZARU_HIP_DMA_PAD");
        return e && std::strtol(e, nullptr, 10) > 0;
    }();
    return v;
}

template <int K, int S, int WM, int MTW, int DFKC, int RT>
static const char *dma_go(const DwPwParams &p, dim3 grid, size_t lds, int nct, int runmax, int bufsz, hipStream_t s) {
    // form "pin" where the task step RT * S makes 16-byte window reads (ds_read_b128: FaceMesh 24^2
    // 44.7 -> 43.2 us, BlazePalm 48^2 205 -> 192 us, 48 -> 24 172 -> 150 us at 256 frames); the
    // 8-byte form measured slower than the compiler's own narrowed reads (FaceMesh 12^2 39.7 -> 41.1,
    // hand 28^2 5x5 146 -> 182 us), so 2-float steps keep dwpw_dma_kernel
    // (profiles/r06_layers/*_pin_vs_not.txt)
    if constexpr (RT > 0 && (RT * S) % 4 == 0)
        if (form_on(FORM_PIN) && p.in.W % 4 == 0) {
            // channel stride: a half-wave's b128 groups hold 8 lanes of each of 2 channels (16
            // tasks per channel) or 4 of each of 4 (8 tasks); with 16-byte-apart lanes they are
            // conflict-free when consecutive channels sit 0 resp. 32 words apart mod 64
            // (tools/lds_banks.py).  ZARU_HIP_DMA_PAD=1 pads the stride so: PMC conflicts 1.2-2.9
            // -> 0.2-0.5 per LDS instruction, but no launch faster and the face line 268 k vs 271 k,
            // BlazePalm +1.3 % (profiles/r06_layers/*_pinpad_vs_packed.txt) -- off by default
            constexpr int BN = (4 / WM) * 32, SEGS = BN / RT, TASKS = DFKC * SEGS;
            constexpr int SPT = SEGS / (TASKS > 256 ? TASKS / 256 : 1), RES = SPT == 16 ? 0 : SPT == 8 ? 32 : -1;
            if constexpr (RES >= 0)
                if (dma_pad_on()) {
                    int rm = runmax, bz = 0;
                    while (rm % 64 != RES) rm += 4;
                    if (const size_t l = dma_lds<K, WM, MTW, DFKC>(rm, &bz)) runmax = rm, bufsz = bz, lds = l;
                }
            hipLaunchKernelGGL((dwpw_dma_pin_kernel<K, S, WM, MTW, DFKC, RT>), grid, dim3(256), lds, s, p, nct, runmax, bufsz);
            return kernel_name("dwpw_dma_pin_kernel<%d,%d,%d,%d,%d,%d>", K, S, WM, MTW, DFKC, RT);
        }
    hipLaunchKernelGGL((dwpw_dma_kernel<K, S, WM, MTW, DFKC, RT>), grid, dim3(256), lds, s, p, nct, runmax, bufsz);
    return kernel_name("dwpw_dma_kernel<%d,%d,%d,%d,%d,%d>", K, S, WM, MTW, DFKC, RT);
}

template <int K, int S, int WM, int MTW, int DFKC>
static const char *dma_launch(const DwPwParams &p, dim3 grid, size_t lds, int nct, int runmax, int bufsz, hipStream_t s) {
    constexpr int BN = (4 / WM) * 32, RH = rt_hi(K, MTW, DFKC * BN / 256);
    const int rt = rt_for<K, S>(p, BN, RH);
    if (rt == RH) return dma_go<K, S, WM, MTW, DFKC, RH>(p, grid, lds, nct, runmax, bufsz, s);
    if constexpr (RH >= 4)
        if (rt == RH / 2) return dma_go<K, S, WM, MTW, DFKC, RH / 2>(p, grid, lds, nct, runmax, bufsz, s);
    return dma_go<K, S, WM, MTW, DFKC, 0>(p, grid, lds, nct, runmax, bufsz, s);
}

template <int K, int S, int WM, int MTW>
const char *dwpw_go(const DwPwParams &p, hipStream_t s) {
    constexpr int BN = (4 / WM) * 32, BM = WM * MTW * 32;
    const int nct = (p.g.ncols + BN - 1) / BN;
    const int mb = (p.g.Mpad + BM - 1) / BM;
    dim3 grid((nct + 7) / 8 * 8, mb);
    int runmax = 0, bufsz = 0;
    if constexpr (K == 3 && MTW == 1) {
        // wider channel chunks: fewer dependent DMA round trips per tile (the 6^2 / 3^2 launches
        // of a few dozen workgroups are nothing but those round trips)
        // (32-column stride-1 tiles: 32 channels make the row tasks 4 wide, so the window reads
        // go 16-byte (form pin): FaceMesh 12^2 39.3 / 38.1 -> 35.3 / 34.4 us, BlazeFace 8^2 16-18
        // -> 14-16 us at 256 images, profiles/r06_layers/*_dfkc32_vs_16.txt)
        const int dk = S == 1 && WM == 4 && !dfkc_env() && form_on(FORM_PIN) ? 32 : dfkc_for(nct * mb, p.g.K);
        if (dk >= 64)
            if (const size_t lds = dma_plan<K, S, WM, MTW, 64>(p, &runmax, &bufsz))
                return dma_launch<K, S, WM, MTW, 64>(p, grid, lds, nct, runmax, bufsz, s);
        if (dk >= 32)
            if (const size_t lds = dma_plan<K, S, WM, MTW, 32>(p, &runmax, &bufsz))
                return dma_launch<K, S, WM, MTW, 32>(p, grid, lds, nct, runmax, bufsz, s);
    }
    if (const size_t lds = dma_plan<K, S, WM, MTW, 16>(p, &runmax, &bufsz))
        return dma_launch<K, S, WM, MTW, 16>(p, grid, lds, nct, runmax, bufsz, s);
    if constexpr ((K == 5 && S == 2 && MTW >= 4) || (K == 3 && S == 2 && MTW == 2)) {
        // stride-2 5x5 tiles over large planes whose input runs do not fit two 16-channel
        // buffers: 8-channel chunks.  BlazePalm's 48^2 -> 24^2 block (128 rows): 163 vs 232 us
        // register-staged at 256 frames; its 96^2 -> 48^2 block (64 rows, MTW 2) measured slower
        // (272 vs 259 us), so it keeps the register-staged form (profiles/r05_layers/)
        // (3x3 stride 2, MTW 2 -- FaceMesh's 48^2 -> 24^2 block: only with form pin, whose
        // 4-wide tasks read 16-byte windows)
        if (K == 5 || form_on(FORM_PIN))
            if (const size_t lds = dma_plan<K, S, WM, MTW, 8>(p, &runmax, &bufsz))
                return dma_launch<K, S, WM, MTW, 8>(p, grid, lds, nct, runmax, bufsz, s);
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

}  // namespace

// the per-(K, S) launchers, each in a translation unit of its own (dwpw_mfma_k*.hip) so the
// instances compile in parallel
const char *dwpw_layout_k3s1(const DwPwParams &p, const DwPwLayout &l, hipStream_t s);
const char *dwpw_layout_k3s2(const DwPwParams &p, const DwPwLayout &l, hipStream_t s);
const char *dwpw_layout_k5s1(const DwPwParams &p, const DwPwLayout &l, hipStream_t s);
const char *dwpw_layout_k5s2(const DwPwParams &p, const DwPwLayout &l, hipStream_t s);

}  // namespace zr
