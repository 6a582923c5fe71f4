// dwpw_ws.hip -- the weight-stationary form of the fused depthwise KxK -> 1x1 block (BlazeBlock /
// BlazePalm block: DW -> PW + bias + act + residual (+pad / +pool) + act) for the low-resolution,
// many-channel layers (24^2 ... 3^2 planes, 32-128 channels): FaceMesh V1 from 24^2 down,
// BlazeFace's 16^2 / 8^2 blocks, the palm detector's small planes.
//
// Those layers are f32-MFMA bound (128 -> 128 channels at 12^2 is 34 flop per algorithmic byte,
// above the 157 TF / 8 TB/s ridge of 20) but few columns wide, so a per-tile kernel that stages
// the 1x1 weights through LDS for every 32-128 column tile spends most of its time waiting:
// two thirds of what its DMA moves are weights.  Here instead
//   * each workgroup is persistent: it loads its waves' slices of the transposed 1x1 weights
//     into VGPRs ONCE (the MFMA A operand, 32 rows x 2 k per register: MW x KS registers) and
//     then walks column tiles (contiguous ranges per XCD, so neighbouring tiles' halo rows are L2
//     hits on the XCD that fetched them);
//   * per tile and chunk of CH = 32 input channels, LDS-DMA (global_load_lds_dwordx4) brings the
//     contiguous CNHW input run the tile's columns need into one of two buffers -- the next
//     chunk's copy, or the next tile's first, is in flight while this one is computed;
//   * the depthwise runs from LDS into a BN-wide tile sD (rows padded so the B-operand reads of
//     both lane halves hit different banks), published by a bare s_barrier (no vmcnt drain of
//     the copy in flight), and every wave runs v_mfma_f32_32x32x2_f32 with A from its registers
//     and B from sD: 16 k-steps x MW MFMAs per barrier;
//   * epilogue_tile: bias, activation, residual (+pad / +pool), activation.
// Arithmetic and accumulation order are those of dwpw_dma_kernel / dwpw_kernel (depthwise taps
// in (ky, kx) order from the bias, then 2 k per MFMA in k order), so the form is bitwise neutral
// (tests/test_gpu_forms.py).
// Reference: the Conv nodes ORT/tract execute at crates/zaru/src/nn/mod.rs:483-533 (SURVEY
// Appendix A: BlazeBlocks of BlazeFace, FaceMesh V1, BlazePalm).
#include <algorithm>
#include <mutex>

#include "../runtime/zr_kernels.h"
#include "act.h"
#include "epilogue.h"

namespace zr {
namespace {

__device__ const float4 ws_zero4 = {0.f, 0.f, 0.f, 0.f};  // LDS-DMA source of the zero slots

// a / b for 0 <= a < 2^22 through the f32 reciprocal, corrected to the exact quotient
__device__ __forceinline__ int wdiv(int a, int b, float inv_b) {
    int q = (int)((float)a * inv_b);
    const int r = a - q * b;
    q += r >= b ? 1 : 0;
    q -= r < 0 ? 1 : 0;
    return q;
}

constexpr int WS_CH = 32;     // input channels per chunk (16 k-steps)

int device_cus() {
    static std::once_flag once;
    static int ncu = 256;
    std::call_once(once, [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            ncu = n;
    });
    return ncu;
}
constexpr int WS_GUARD = 256; // LDS floats in front of / behind the input buffers (masked taps)

// Geometry of one BN-column tile: its input run (floats from a channel plane's base, 16-byte
// aligned ends) and this thread's depthwise column.
struct WsTile {
    int j0, s0, run4;
    int n, q, tb;
    uint32_t mask;
};

template <int K, int S, int BN>
__device__ __forceinline__ WsTile ws_tile(const DwPwParams &P, int tile, int dj) {
    const GemmParams &G = P.g;
    const int H = P.in.H, W = P.in.W, Pin = H * W, OW = P.OW, Pq = G.P;
    WsTile t;
    t.j0 = tile * BN;
    const int ja = t.j0, jb = min(t.j0 + BN, G.ncols) - 1;
    const int na = ja / Pq, qa = ja - na * Pq, nb = jb / Pq, qb = jb - nb * Pq;
    const int ya = max(qa / OW * S - P.pad_t, 0), yb = min(qb / OW * S - P.pad_t + K - 1, H - 1);
    t.s0 = (na * Pin + ya * W) & ~3;
    const int e0 = (nb * Pin + (yb + 1) * W + 3) & ~3;
    t.run4 = (e0 - t.s0) >> 2;
    const int jd = min(t.j0 + dj, G.ncols - 1);
    t.n = jd / Pq;
    t.q = jd - t.n * Pq;
    const int oy = t.q / OW, ox = t.q - oy * OW;
    const int iy0 = oy * S - P.pad_t, ix0 = ox * S - P.pad_l;
    t.tb = t.n * Pin + iy0 * W + ix0 - t.s0;  // run index of tap (0, 0); < 0 only when masked
    t.mask = 0;
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
            const int iy = iy0 + ky, ix = ix0 + kx;
            t.mask |= (iy >= 0 && iy < H && ix >= 0 && ix < W ? 1u : 0u) << (ky * K + kx);
        }
    return t;
}

// WM waves along M, each holding MW 32-row tiles; WN = 4 / WM waves along N (BN = 32 WN columns).
// KS: k-steps the weight registers cover (Kpad / 2 rounded up to 16); ks (runtime) <= KS.
template <int K, int S, int WM, int MW, int KS>
__global__ __launch_bounds__(256) void dwpw_ws_kernel(const DwPwParams P, int ntiles, int runmax, int sdst) {
    constexpr int WN = 4 / WM, BN = WN * 32, KK = K * K;
    constexpr int CPAR = 256 / BN, PER = WS_CH / CPAR;
    constexpr int NCH = KS / 16;
    static_assert(KS % 16 == 0 && PER >= 1, "chunking");
    constexpr int KKP = (WS_CH * KK + 3) / 4 * 4;  // the chunk's depthwise weights, 16-B multiple
    extern __shared__ __attribute__((aligned(16))) float lds_ws[];
    // one buffer: the chunk's input runs (WS_CH x runmax), its depthwise weights and biases;
    // whole 256-float DMA rows
    const int bufsz = (WS_CH * runmax + KKP + WS_CH + 255) / 256 * 256;
    float *inb = lds_ws + WS_GUARD;                // 2 buffers, then the tail guard
    float *sD = inb + 2 * bufsz + WS_GUARD;        // the depthwise tile, WS_CH x sdst
    const GemmParams &G = P.g;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kh = lane >> 5, col = lane & 31;
    const int wm = wave % WM, wn = wave / WM;
    const int Cin = G.K;

    // this workgroup's tiles: XCD x = blockIdx % 8 owns the contiguous range [x*per, (x+1)*per)
    const int nwg = gridDim.x >> 3;  // workgroups per XCD (gridDim.x is a multiple of 8)
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int per = (ntiles + 7) >> 3;
    const int t_end = min((xcd + 1) * per, ntiles);
    int tile = xcd * per + slot;
    if (tile >= t_end) return;  // whole workgroup, before any barrier

    // the stationary A operand: rows (wm * MW + t) * 32 + col (< Mpad = BM), k = 2 s + kh; the
    // plan stores the transposed weights with zero rows up to a multiple of 32 (= 2 KS)
    float wa[MW][KS];
#pragma unroll
    for (int t = 0; t < MW; ++t) {
        const uint32_t m = (uint32_t)((wm * MW + t) * 32 + col);
#pragma unroll
        for (int s = 0; s < KS; ++s) wa[t][s] = G.wt[(uint32_t)(2 * s + kh) * (uint32_t)G.Mpad + m];
    }

    const int dj = tid % BN;
    int dc = tid / BN;
    if constexpr (BN >= 64) dc = __builtin_amdgcn_readfirstlane(dc);  // one channel per wave
    const int rq = runmax >> 2;
    const float inv_rq = 1.f / (float)rq;
    const int nwi = bufsz >> 8;  // 64-slot DMA wave-instructions per buffer
    const int r1 = WS_CH * rq, r2 = r1 + KKP / 4, r3 = r2 + WS_CH / 4;  // slot regions
    auto stage = [&](const WsTile &g, int c0, float *dst) {
        for (int wi = wave; wi < nwi; wi += 4) {
            const int sl = wi * 64 + lane;
            const float *src = (const float *)&ws_zero4;
            if (sl < r1) {
                const int c = wdiv(sl, rq, inv_rq), i = sl - c * rq;
                if (c0 + c < Cin && i < g.run4)
                    src = P.in.p + (size_t)(uint32_t)(c0 + c) * (uint32_t)P.in.sC + (uint32_t)(g.s0 + 4 * i);
            } else if (sl < r2) {  // depthwise weights [c][KK] of channels c0 ...
                const int i = sl - r1;
                if (c0 * KK + 4 * i < Cin * KK) src = P.dw_w + c0 * KK + 4 * i;
            } else if (sl < r3) {  // and their biases (Cin % 4 == 0: whole 16-B slots)
                const int i = sl - r2;
                if (c0 + 4 * i < Cin) src = P.dw_b + c0 + 4 * i;
            }
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(dst + wi * 256), 16, 0, 0);
        }
    };

    WsTile g = ws_tile<K, S, BN>(P, tile, dj);
    stage(g, 0, inb);
    int it = 0;
    while (true) {
        const int next = tile + nwg;
        const bool more = next < t_end;
        const WsTile gn = ws_tile<K, S, BN>(P, more ? next : tile, dj);
        f32x16 acc[MW];
#pragma unroll
        for (int t = 0; t < MW; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
#pragma unroll
        for (int c = 0; c < NCH; ++c, ++it) {
            const int c0 = c * WS_CH;
            if (c0 >= Cin) break;  // uniform: the weight registers past ks are zero anyway
            const float *buf = inb + (it & 1) * bufsz;
            const float *sDW = buf + WS_CH * runmax, *sDB = sDW + KKP;
            // vmcnt(0) + barrier: this chunk has landed, and every wave is past the previous
            // chunk's depthwise (its input buffer may be refilled) and MFMAs (sD may be rewritten)
            __syncthreads();
            const bool last = c + 1 == NCH || c0 + WS_CH >= Cin;
            if (!last) stage(g, c0 + WS_CH, inb + ((it + 1) & 1) * bufsz);
            else if (more) stage(gn, 0, inb + ((it + 1) & 1) * bufsz);
            // depthwise outputs of this thread's column, DG channels at a time (bounded live set)
            // (a rolled loop: unrolled, the scheduler hoists every group's tap reads and constant
            // loads and the live set exhausts the VGPRs / SGPRs)
            constexpr int DG = PER < 4 ? PER : 4;
#pragma unroll 1
            for (int i0 = 0; i0 < PER; i0 += DG) {
                float dv[DG];
#pragma unroll
                for (int u = 0; u < DG; ++u) {
                    const int cl = dc + CPAR * (i0 + u);
                    const float *t0 = buf + cl * runmax + g.tb;
                    const float *w = sDW + cl * KK;
                    float a = sDB[cl];
#pragma unroll
                    for (int ky = 0; ky < K; ++ky)
#pragma unroll
                        for (int kx = 0; kx < K; ++kx) {
                            const int t = ky * K + kx;
                            const float x = t0[ky * P.in.W + kx];
                            a = __builtin_fmaf(w[t], ((g.mask >> t) & 1u) ? x : 0.f, a);
                        }
                    dv[u] = a;
                }
                apply_act_n<DG>(P.dw_act, dv, [&](int u) { return min(c0 + dc + CPAR * (i0 + u), Cin - 1); });
#pragma unroll
                for (int u = 0; u < DG; ++u) {
                    const int cl = dc + CPAR * (i0 + u);
                    sD[cl * sdst + dj] = c0 + cl < Cin ? dv[u] : 0.f;
                }
            }
            // publish sD without draining the DMA in flight (a __syncthreads would wait vmcnt(0))
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            // all 16 k-steps of the chunk: past Kpad the weights and sD rows are zero, which adds
            // exact zeros (a branch per step would cost more than the MFMA it skips)
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const float b = sD[(2 * s + kh) * sdst + wn * 32 + col];
#pragma unroll
                for (int t = 0; t < MW; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[t][c * 16 + s], b, acc[t], 0, 0, 0);
            }
        }
        const int j = g.j0 + wn * 32 + col;
        if (j < G.ncols) {
            // 4 rows at a time: the weights stay live, so the epilogue's hoisted bias / residual /
            // slope loads must not all be in flight at once
            const int on = j / G.P, oq = j - on * G.P;
            const uint32_t ob = (uint32_t)on * (uint32_t)G.o_sN + (uint32_t)oq * (uint32_t)G.o_sP;
            // the row offsets (m * o_sC, m * r_sC, bias / slope addresses) are loop-invariant:
            // hoisted out of the tile loop they would hold ~64 VGPRs for the kernel's lifetime
            int khl = kh;
            asm volatile("" : "+v"(khl));
#pragma unroll
            for (int t = 0; t < MW; ++t)
#pragma unroll
                for (int r0 = 0; r0 < 16; r0 += 4) {
                    float v[4];
                    epilogue_part<4>(G, acc[t], on, oq, (wm * MW + t) * 32, khl, r0, v);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int m = (wm * MW + t) * 32 + mfma32_row(r0 + r, khl);
                        if (m < G.M) G.out[ob + (uint32_t)m * (uint32_t)G.o_sC] = v[r];
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
        }
        if (!more) break;
        tile = next;
        g = gn;
    }
}

// LDS plan: the longest input run any BN-column tile needs (floats, 16-byte multiple), buffers
// rounded to whole 1 KiB DMA wave-instructions.  0 when the layer does not qualify.
template <int K, int S, int BN>
size_t ws_plan(const DwPwParams &p, int *runmax, int *sdst) {
    const int H = p.in.H, W = p.in.W, Pin = H * W, Pq = p.g.P, OW = p.OW;
    const int nimg = p.g.ncols / Pq;
    if (p.in.sN != Pin || p.in.sC % 4 || ((int64_t)nimg * Pin) % 4 || p.g.K % 4 || p.dw_act.kind == ACT_SIGMOID ||
        ((uintptr_t)p.in.p | (uintptr_t)p.g.wt | (uintptr_t)p.dw_w | (uintptr_t)p.dw_b) % 16)
        return 0;
    // masked taps (padding rows above the first / below the last image of a run) stay in the guards
    if (p.pad_t * W + p.pad_l > WS_GUARD || (K - 1) * W + K > WS_GUARD) return 0;
    int rm = 0;
    for (int j0 = 0; j0 < p.g.ncols; j0 += BN) {  // tiles repeat with the image period
        const int jb = std::min(j0 + BN, p.g.ncols) - 1;
        const int na = j0 / Pq, qa = j0 - na * Pq, nb = jb / Pq, qb = jb - nb * Pq;
        const int ya = std::max(qa / OW * S - p.pad_t, 0), yb = std::min(qb / OW * S - p.pad_t + K - 1, H - 1);
        const int s0 = (na * Pin + ya * W) & ~3, e0 = (nb * Pin + (yb + 1) * W + 3) & ~3;
        rm = std::max(rm, e0 - s0);
        if (na >= 4 && (j0 % Pq) == 0) break;  // the pattern has repeated (whole images seen)
    }
    // WS_CH * runmax must be whole 256-float DMA rows: runmax a multiple of 8
    rm = (rm + 7) / 8 * 8;
    *runmax = rm;
    *sdst = BN % 64 == 0 ? BN + 32 : BN;  // the two lane halves' B rows on different banks
    const int bufsz = (WS_CH * rm + (WS_CH * K * K + 3) / 4 * 4 + WS_CH + 255) / 256 * 256;
    const size_t floats = 2 * WS_GUARD + 2 * (size_t)bufsz + (size_t)WS_CH * *sdst;
    const size_t lds = sizeof(float) * floats;
    return lds <= 144 * 1024 ? lds : 0;
}

template <int K, int S, int WM, int MW, int KS>
const char *ws_go(const DwPwParams &p, hipStream_t s) {
    constexpr int BN = (4 / WM) * 32;
    int runmax = 0, sdst = 0;
    const size_t lds = ws_plan<K, S, BN>(p, &runmax, &sdst);
    if (!lds) return nullptr;
    const int ntiles = (p.g.ncols + BN - 1) / BN;
    // persistent grid: as many workgroups as fit on the chip at once (this instance's registers,
    // the layer's LDS), never more than the tiles, a multiple of 8 (one tile range per XCD)
    static std::once_flag once;
    static int per_cu = 1;
    std::call_once(once, [] {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dwpw_ws_kernel<K, S, WM, MW, KS>, 256, 0) == hipSuccess &&
            n > 0)
            per_cu = n;
    });
    const int fit = std::max(1, (int)((160 * 1024) / lds));
    const int wgs_cu = std::max(1, std::min(per_cu, fit));
    int grid = std::min(ntiles, device_cus() * wgs_cu);
    grid = (grid + 7) / 8 * 8;
    hipLaunchKernelGGL((dwpw_ws_kernel<K, S, WM, MW, KS>), dim3(grid), dim3(256), lds, s, p, ntiles, runmax, sdst);
    return kernel_name("dwpw_ws_kernel<%d,%d,%d,%d,%d>", K, S, WM, MW, KS);
}

template <int K, int S, int WM, int MW>
const char *ws_ks(const DwPwParams &p, hipStream_t s) {
    const int ks = p.g.Kpad / 2;
#ifdef ZR_WS_PROBE  // resource-usage probe builds: one instance per layout
    return ks <= 64 ? ws_go<K, S, WM, MW, 64>(p, s) : nullptr;
#else
    if (ks <= 16) return ws_go<K, S, WM, MW, 16>(p, s);
    if (ks <= 32) return ws_go<K, S, WM, MW, 32>(p, s);
    if (ks <= 48) return ws_go<K, S, WM, MW, 48>(p, s);
    return ws_go<K, S, WM, MW, 64>(p, s);
#endif
}

template <int K, int S>
const char *ws_layout(const DwPwParams &p, hipStream_t s) {
    switch ((p.g.Mpad + 31) / 32) {
    case 1: return ws_ks<K, S, 1, 1>(p, s);  // BN 128
    case 2: return ws_ks<K, S, 2, 1>(p, s);  // BN 64
    case 3: return ws_ks<K, S, 1, 3>(p, s);  // BN 128, every wave all 96 rows
    default: return ws_ks<K, S, 4, 1>(p, s); // BN 32
    }
}

}  // namespace

// The weight-stationary form applies to depthwise 3x3 / 5x5 -> 1x1 blocks with Mpad <= 128 and
// Kpad <= 128 over CNHW inputs (launch_dwpw calls this first; nullptr = not applicable).
const char *launch_dwpw_ws(const DwPwParams &p, hipStream_t s) {
    // (Mpad is a multiple of 32, so every layout's BM equals it and no weight row is out of range)
    if (!form_on(FORM_WS) || p.g.Mpad > 128 || p.g.Kpad > 128 || p.g.Mpad % 32 || p.g.KK != 1) return nullptr;
#ifdef ZR_WS_PROBE
    return p.k == 3 && p.stride == 1 ? ws_layout<3, 1>(p, s) : nullptr;
#endif
    if (p.k == 3) return p.stride == 1 ? ws_layout<3, 1>(p, s) : ws_layout<3, 2>(p, s);
    if (p.k == 5) return p.stride == 1 ? ws_layout<5, 1>(p, s) : ws_layout<5, 2>(p, s);
    return nullptr;
}

}  // namespace zr
