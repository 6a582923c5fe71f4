// dwpw_ws.hip -- the depthwise KxK -> 1x1 BlazeBlock for the low-resolution,
// many-channel layers as a warp-specialized persistent kernel.  Reference: the Conv nodes of the
// four ONNX graphs ORT / tract execute at crates/zaru/src/nn/mod.rs:483-533.
//
// What bounds these layers (profiles/r03_layers/): per output column the 1x1 costs Cin * Cout MFMA
// MACs and the depthwise Cin * K^2 VALU FMAs -- the two are within 3x of each other -- and the
// per-tile forms (dwpw_dma_kernel) run them back to back in every wave, read every depthwise tap
// from LDS with its own ds_read_b32 (25 LDS dwords per output at 5x5: the LDS array, not the
// MFMA, set their pace) and wait one HBM round trip per 16-channel chunk.  Here:
//   * one 512-thread workgroup per CU walks a run of BN-column tiles (contiguous per XCD);
//   * waves 4..7 are producers: they stream each chunk's CNHW input runs (+ the chunk's depthwise
//     weights, bias and PReLU slopes) into a D-stage LDS ring by LDS-DMA, D - 1 chunks ahead
//     across tile boundaries, and compute the depthwise of chunk g + 1 into one of two tiles
//     while ...
//   * waves 0..3 are consumers: they run chunk g's v_mfma_f32_32x32x2_f32 from the other tile,
//     with their 1x1 weight fragments in registers (loaded a chunk ahead), and the epilogue.
//     Every SIMD holds one wave of each role, so the matrix pipe and the VALU work side by side;
//   * a producer task is one whole output row (R = the output width <= 16) of one channel: each
//     input row is read once, with wide LDS reads, for R outputs (K + (R-1)S dwords for R*K
//     FMAs, not K*K per output), the task's K*K weights are held in registers, and the padding
//     columns are static (fmaf with a 0 operand, the other forms' arithmetic for masked taps).
// One s_barrier per chunk hands the tiles over.  The arithmetic is the other forms' to the bit:
// the depthwise is bias + fmaf over the taps in (ky, kx) order with masked taps fmaf'd as 0, the
// 1x1 the same MFMA chain over k, the epilogue epilogue_tile (tests/test_gpu_forms.py).
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "../runtime/zr_kernels.h"
#include "act.h"
#include "epilogue.h"
#include "lds_dma.h"

namespace zr {

namespace {

constexpr int WS_FC = 16;  // input channels per chunk

// Host-computed layout of one launch.
struct WsPlan {
    int nct;     // column tiles of BN columns
    int tpx;     // tiles per XCD range
    int nch;     // chunks per tile (ceil(Cin / WS_FC))
    int rq;      // 16-B slots per channel input run in a stage (the longest tile run / 4)
    int stg;     // floats per stage (whole 1 KiB DMA wave-instructions)
    int D;       // ring depth
    int o_ring;  // LDS offset of the ring (floats)
    int o_d;     // LDS offset of the two depthwise tiles
};

// the workgroup barrier that hands the tiles over: this wave's LDS stores are complete, but no
// wait on vector memory (the ring's DMA stays in flight; producers count it themselves)
__device__ __forceinline__ void ws_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// epilogue_tile, with its row / address math kept in the epilogue branch: without the opaque
// mbase / kh the compiler hoists every row's channel index and bias / residual / slope address
// out of the chunk loop and holds them across it (spilling at MTW = 2)
__device__ __forceinline__ void ws_epilogue(const GemmParams &G, const f32x16 &acc, int n, int q, int mbase, int kh) {
    asm volatile("" : "+v"(mbase), "+v"(kh));
    epilogue_tile(G, acc, n, q, mbase, kh);
}

template <int K, int S, int R, int WM, int MTW, int NTW>
__global__ __launch_bounds__(512) void dwpw_ws_kernel(const DwPwParams P, const WsPlan L) {
    constexpr int FC = WS_FC, KK = K * K, WN = 4 / WM;
    constexpr int BN = WN * NTW * 32;
    constexpr int PL = DwPad<K, S>::L;             // the models' padding (host-checked)
    constexpr int IW = S * R;                      // input row width (host-checked)
    constexpr int RPT = BN / R;                    // output rows per tile
    constexpr int NRND = (FC * RPT + 255) / 256;   // tasks per producer lane per chunk
    constexpr int KKP = (FC * KK + 3) / 4 * 4;     // depthwise weight floats in a stage
    static_assert(BN % R == 0, "a tile holds whole output rows");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const GemmParams &G = P.g;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kh = lane >> 5, col = lane & 31;

    // this workgroup's tiles: XCD x owns [x * tpx, (x + 1) * tpx), its workgroups take them round robin
    const int G8 = gridDim.x >> 3, xcd = blockIdx.x & 7, wslot = blockIdx.x >> 3;
    const int t_beg = xcd * L.tpx + wslot, t_end = min((xcd + 1) * L.tpx, L.nct);
    const int ntl = t_beg < t_end ? (t_end - t_beg + G8 - 1) / G8 : 0;
    if (ntl == 0) return;  // whole workgroup, before any barrier
    const int nst = ntl * L.nch;
    const int Cin = G.K, H = P.in.H, Pin = H * IW, Pq = G.P;
    const int rs4 = 4 * L.rq;
    float *const ring = lds + L.o_ring, *const sD = lds + L.o_d;
    // slot regions of a stage (16-B slots): input runs | depthwise weights | bias | PReLU slopes
    const int r1 = FC * L.rq, r2 = r1 + KKP / 4, r3 = r2 + FC / 4, r4 = r3 + FC / 4;
    const float inv_rq = 1.f / (float)L.rq;

    // the input run of tile t: first float (16-B aligned, from a channel's base) and length / 4
    auto run_of = [&](int t, int &s0, int &run4) {
        const int ja = t * BN, jb = min(ja + BN, G.ncols) - 1;
        const int na = ja / Pq, qa = ja - na * Pq, nb = jb / Pq, qb = jb - nb * Pq;
        const int ya = max(qa / R * S - PL, 0), yb = min(qb / R * S - PL + K - 1, H - 1);
        s0 = (na * Pin + ya * IW) & ~3;
        run4 = (((nb * Pin + (yb + 1) * IW + 3) & ~3) - s0) >> 2;
    };

    if (wave >= 4) {
        // ================================================================ producers
        const int pw = wave - 4, ptid = tid - 256;
        const int nwi = L.stg >> 8;                              // DMA wave-instructions per stage
        const int cnt_w = pw < nwi ? (nwi - pw + 3) / 4 : 0;     // of them issued by this wave
        const bool prelu = P.dw_act.kind == ACT_PRELU;
        int i_k = 0, i_chunk = 0, i_s0 = 0, i_run4 = 0, issued = 0;
        run_of(t_beg, i_s0, i_run4);
        auto issue = [&]() {  // stage `issued` (tile i_k, chunk i_chunk) into ring slot issued % D
            const int kc = i_chunk * FC;
            float *dst = ring + (issued % L.D) * L.stg;
            for (int wi = pw; wi < nwi; wi += 4) {
                const int sl = wi * 64 + lane;
                const float *src = (const float *)&zr_zero4;
                if (sl < r1) {
                    const int c = qdiv(sl, L.rq, inv_rq), i = sl - c * L.rq;
                    if (kc + c < Cin && i < i_run4)
                        src = P.in.p + (size_t)(uint32_t)(kc + c) * (uint32_t)P.in.sC + (uint32_t)(i_s0 + 4 * i);
                } else if (sl < r2) {
                    const int i = sl - r1;
                    if (kc * KK + 4 * i < Cin * KK) src = P.dw_w + kc * KK + 4 * i;
                } else if (sl < r3) {
                    const int i = sl - r2;
                    if (kc + 4 * i < Cin) src = P.dw_b + kc + 4 * i;
                } else if (sl < r4) {
                    const int i = sl - r3;
                    if (prelu && kc + 4 * i < Cin) src = P.dw_act.slope + kc + 4 * i;
                }
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                                 (__attribute__((address_space(3))) void *)(dst + wi * 256), 16, 0, 0);
            }
            ++issued;
            if (++i_chunk == L.nch) {
                i_chunk = 0;
                if (++i_k < ntl) run_of(t_beg + i_k * G8, i_s0, i_run4);
            }
        };
        // the depthwise side: stage d_g (tile d_k, chunk d_chunk).  Task i of a chunk is output
        // row rr = i % RPT of the tile in channel c = i / RPT; per tile each round keeps its row's
        // run offset (-1: no task) and valid-row mask
        int d_g = -1, d_k = -1, d_chunk = L.nch - 1;
        int g_tb[NRND];
        uint32_t g_m[NRND];
        auto d_advance = [&]() {
            ++d_g;
            if (++d_chunk < L.nch) return;
            d_chunk = 0;
            const int t = t_beg + (++d_k) * G8;
            int s0, run4;
            run_of(t, s0, run4);
            const int j0 = t * BN, rows = (min(j0 + BN, G.ncols) - j0) / R;
#pragma unroll
            for (int r = 0; r < NRND; ++r) {
                const int i = ptid + 256 * r, rr = i % RPT;
                g_tb[r] = INT_MIN;  // no task
                g_m[r] = 0;
                if (i < FC * RPT && rr < rows) {
                    const int j = j0 + rr * R;
                    const int n = j / Pq, oy = (j - n * Pq) / R, iy0 = oy * S - PL;
                    uint32_t m = 0;
#pragma unroll
                    for (int ky = 0; ky < K; ++ky) m |= (iy0 + ky >= 0 && iy0 + ky < H ? 1u : 0u) << ky;
                    g_tb[r] = n * Pin + iy0 * IW - s0;
                    g_m[r] = m;
                }
            }
        };
        auto d_compute = [&]() {  // the depthwise of stage d_g into tile d_g & 1
            const float *stage = ring + (d_g % L.D) * L.stg;
            const float *sW = stage + 4 * r1, *sB = stage + 4 * r2, *sS = stage + 4 * r3;
            float *dst = sD + (d_g & 1) * FC * BN;
            const int kc = d_chunk * FC;
#pragma unroll
            for (int r = 0; r < NRND; ++r) {
                if (g_tb[r] == INT_MIN) continue;  // no task this round
                const int i = ptid + 256 * r, c = i / RPT, rr = i - c * RPT;
                const float *base = stage + c * rs4 + g_tb[r];
                const uint32_t m = g_m[r];
                float w[KK];
#pragma unroll
                for (int t = 0; t < KK; ++t) w[t] = sW[c * KK + t];
                float acc[R];
                const float b = sB[c];
#pragma unroll
                for (int o = 0; o < R; ++o) acc[o] = b;
#pragma unroll
                for (int ky = 0; ky < K; ++ky) {
                    // the input row (clamped to a valid row of the run when outside the image)
                    const bool rv = (m >> ky) & 1u;
                    const float *row = base + (rv ? ky * IW : PL * IW);
                    float x[IW];
                    if constexpr (IW % 4 == 0) {
#pragma unroll
                        for (int e = 0; e < IW; e += 4) {
                            const float4 v = *reinterpret_cast<const float4 *>(row + e);
                            x[e] = v.x, x[e + 1] = v.y, x[e + 2] = v.z, x[e + 3] = v.w;
                        }
                    } else if constexpr (IW % 2 == 0) {
#pragma unroll
                        for (int e = 0; e < IW; e += 2) {
                            const float2 v = *reinterpret_cast<const float2 *>(row + e);
                            x[e] = v.x, x[e + 1] = v.y;
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < IW; ++e) x[e] = row[e];
                    }
#pragma unroll
                    for (int e = 0; e < IW; ++e) x[e] = rv ? x[e] : 0.f;
#pragma unroll
                    for (int kx = 0; kx < K; ++kx)
#pragma unroll
                        for (int o = 0; o < R; ++o) {
                            const int xi = o * S + kx - PL;  // static: padding columns read 0
                            acc[o] = __builtin_fmaf(w[ky * K + kx], xi >= 0 && xi < IW ? x[xi < 0 ? 0 : xi >= IW ? IW - 1 : xi] : 0.f, acc[o]);
                        }
                }
                switch (P.dw_act.kind) {  // apply_act_n's arithmetic, the slope from the stage
                case ACT_RELU:
#pragma unroll
                    for (int o = 0; o < R; ++o) acc[o] = fmaxf(acc[o], 0.f);
                    break;
                case ACT_CLIP:
#pragma unroll
                    for (int o = 0; o < R; ++o) acc[o] = fminf(fmaxf(acc[o], P.dw_act.lo), P.dw_act.hi);
                    break;
                case ACT_PRELU: {
                    const float sl = sS[c];
#pragma unroll
                    for (int o = 0; o < R; ++o) acc[o] = acc[o] < 0.f ? acc[o] * sl : acc[o];
                    break;
                }
                case ACT_SIGMOID:
#pragma unroll
                    for (int o = 0; o < R; ++o) acc[o] = 1.f / (1.f + expf(-acc[o]));
                    break;
                default: break;
                }
                const bool live = kc + c < Cin;
                float *out = dst + c * BN + rr * R;
#pragma unroll
                for (int o = 0; o < R; ++o) out[o] = live ? acc[o] : 0.f;
            }
        };
        // prologue: the first D stages in flight; stage 0 landed (this wave's part) ...
        while (issued < L.D && issued < nst) issue();
        wait_vmcnt_dyn((issued - 1) * cnt_w);
        ws_barrier();  // ... for every wave
        d_advance();
        d_compute();
        if (nst > 1) wait_vmcnt_dyn((issued - 2) * cnt_w);
        ws_barrier();
        for (int g = 0; g < nst; ++g) {
            if (issued < nst) issue();  // into the slot stage g occupied (its depthwise is done)
            if (g + 1 < nst) {
                d_advance();
                d_compute();
            }
            if (g + 2 < nst) wait_vmcnt_dyn(max(0, issued - (g + 3)) * cnt_w);
            ws_barrier();
        }
    } else {
        // ================================================================ consumers
        const int wm = wave % WM, wn = wave / WM;
        const int mw = wm * MTW * 32 + col;
        f32x16 acc[MTW][NTW];
#pragma unroll
        for (int t = 0; t < MTW; ++t)
#pragma unroll
            for (int u = 0; u < NTW; ++u)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[t][u][e] = 0.f;
        // this lane's A fragments of a chunk: W^T[kc + 2s + kh][mw + 32t] (rows past Kpad / Mpad
        // zero); loaded raw a chunk ahead and selected when they become current, so no load is
        // waited for before the chunk's MFMAs
        float wa[MTW][FC / 2], wb[MTW][FC / 2];
        auto wok = [&](int chunk, int s, int t) { return chunk * FC + 2 * s + kh < G.Kpad && mw + t * 32 < G.Mpad; };
        auto wload = [&](int chunk, float (&w)[MTW][FC / 2]) {
#pragma unroll
            for (int s = 0; s < FC / 2; ++s)
#pragma unroll
                for (int t = 0; t < MTW; ++t) {
                    const int k = chunk * FC + 2 * s + kh;
                    w[t][s] = G.wt[wok(chunk, s, t) ? (uint32_t)k * (uint32_t)G.Mpad + (uint32_t)(mw + t * 32) : 0u];
                }
        };
        auto wsel = [&](int chunk, float (&w)[MTW][FC / 2]) {
#pragma unroll
            for (int s = 0; s < FC / 2; ++s)
#pragma unroll
                for (int t = 0; t < MTW; ++t) w[t][s] = wok(chunk, s, t) ? w[t][s] : 0.f;
        };
        wload(0, wa);
        wsel(0, wa);
        ws_barrier();
        ws_barrier();
        int c_k = 0, c_chunk = 0;
        for (int g = 0; g < nst; ++g) {
            const int nx = c_chunk + 1 == L.nch ? 0 : c_chunk + 1;
            if (g + 1 < nst) wload(nx, wb);
            const float *bD = sD + (g & 1) * FC * BN + wn * NTW * 32 + col;
#pragma unroll
            for (int s = 0; s < FC / 2; ++s) {
                float bv[NTW];
#pragma unroll
                for (int u = 0; u < NTW; ++u) bv[u] = bD[(2 * s + kh) * BN + u * 32];
#pragma unroll
                for (int t = 0; t < MTW; ++t)
#pragma unroll
                    for (int u = 0; u < NTW; ++u)
                        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[t][s], bv[u], acc[t][u], 0, 0, 0);
            }
            if (c_chunk + 1 == L.nch) {  // the tile's last chunk: epilogue
                const int j0 = (t_beg + c_k * G8) * BN;
#pragma unroll
                for (int u = 0; u < NTW; ++u) {
                    const int j = j0 + (wn * NTW + u) * 32 + col;
                    if (j < G.ncols) {
                        const int n = j / Pq, q = j - n * Pq;
#pragma unroll
                        for (int t = 0; t < MTW; ++t) ws_epilogue(G, acc[t][u], n, q, (wm * MTW + t) * 32, kh);
                    }
                }
#pragma unroll
                for (int t = 0; t < MTW; ++t)
#pragma unroll
                    for (int u = 0; u < NTW; ++u)
#pragma unroll
                        for (int e = 0; e < 16; ++e) acc[t][u][e] = 0.f;
                ++c_k;
            }
            c_chunk = nx;
            if (g + 1 < nst) {
                wsel(nx, wb);
#pragma unroll
                for (int t = 0; t < MTW; ++t)
#pragma unroll
                    for (int s = 0; s < FC / 2; ++s) wa[t][s] = wb[t][s];
            }
            ws_barrier();
        }
    }
}

template <int K, int S, int R, int WM, int MTW, int NTW>
const char *ws_go(const DwPwParams &p, hipStream_t s, bool launch) {
    constexpr int FC = WS_FC, BN = (4 / WM) * NTW * 32, KKP = (FC * K * K + 3) / 4 * 4;
    constexpr int PL = DwPad<K, S>::L;
    const GemmParams &g = p.g;
    const int H = p.in.H, W = p.in.W, Pin = H * W, Pq = g.P;
    if (p.OW != R || W != S * R || p.pad_t != PL || p.pad_l != PL || g.Mpad > WM * MTW * 32) return nullptr;
    WsPlan L{};
    L.nct = (g.ncols + BN - 1) / BN;
    L.nch = (g.K + FC - 1) / FC;
    int rm = 0;
    for (int j0 = 0; j0 < g.ncols; j0 += BN) {  // tiles repeat with the image period
        const int jb = std::min(j0 + BN, g.ncols) - 1;
        const int na = j0 / Pq, qa = j0 - na * Pq, nb = jb / Pq, qb = jb - nb * Pq;
        const int ya = std::max(qa / R * S - PL, 0), yb = std::min(qb / R * S - PL + K - 1, H - 1);
        const int s0 = (na * Pin + ya * W) & ~3, e0 = (nb * Pin + (yb + 1) * W + 3) & ~3;
        rm = std::max(rm, e0 - s0);
        if (na >= 4 && (j0 % Pq) == 0) break;  // the pattern has repeated (whole images seen)
    }
    static const int ncu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    // a persistent workgroup per CU pays off only with about a tile per CU or more (at 341 hand
    // ROIs the 7^2 layers have 75 tiles: 2.2x slower than the per-tile form)
    if (L.nct * 5 < ncu * 4) return nullptr;
    L.rq = rm / 4;
    const int slots = FC * L.rq + KKP / 4 + 2 * (FC / 4);
    L.stg = (slots + 63) / 64 * 256;
    // LDS: ring | two depthwise tiles (every row a task reads, clamped ones included, lies in its run)
    const int budget = 160 * 1024 / 4;
    L.D = std::min(4, (budget - 2 * FC * BN) / L.stg);
    if (L.D < 2) return nullptr;
    L.o_ring = 0;
    L.o_d = L.D * L.stg;
    const size_t lds = sizeof(float) * (size_t)(L.o_d + 2 * FC * BN);
    const int G = (std::min(L.nct, ncu) + 7) / 8 * 8;
    L.tpx = (L.nct + 7) / 8;
    if (!launch) return "dwpw_ws_kernel";
    static const bool attr = hipFuncSetAttribute((const void *)dwpw_ws_kernel<K, S, R, WM, MTW, NTW>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL((dwpw_ws_kernel<K, S, R, WM, MTW, NTW>), dim3(G), dim3(512), lds, s, p, L);
    return kernel_name("dwpw_ws_kernel<%d,%d,%d,%d,%d,%d>", K, S, R, WM, MTW, NTW);
}

bool ws_enabled() { return form_on(FORM_WS); }  // ZARU_HIP_FORMS=-ws: the per-tile forms instead

// The instances (K, S, R = output width, Mpad class): the hand landmark network's 14^2 / 7^2
// blocks at 1024 ROIs, where a launch has >= ~1 tile per CU and the per-tile forms are paced by
// their depthwise LDS reads (profiles/r04_layers/).  The lower-resolution face / palm layers keep
// the per-tile forms: a persistent kernel of BN-column tiles leaves most CUs idle there.
// Mpad <= 64 -> 2 x 2 waves, <= 128 -> 4 x 1; N tiles per wave so a tile holds whole rows.
#define ZR_WS64(K, S, R, NT) if (mp <= 64) return ws_go<K, S, R, 2, 1, NT>(p, s, launch);
#define ZR_WS128(K, S, R, NT) if (mp <= 128) return ws_go<K, S, R, 4, 1, NT>(p, s, launch);

const char *ws_dispatch(const DwPwParams &p, hipStream_t s, bool launch) {
    const int mp = p.g.Mpad, ow = p.OW;

    if (p.k == 3 && p.stride == 1 && ow == 14) { ZR_WS64(3, 1, 14, 7) }
    if (p.k == 5 && p.stride == 1 && ow == 14) { ZR_WS64(5, 1, 14, 7) }
    if (p.k == 5 && p.stride == 1 && ow == 7) { ZR_WS128(5, 1, 7, 7) }
    if (p.k == 5 && p.stride == 2 && ow == 7) { ZR_WS128(5, 2, 7, 7) }
    return nullptr;
}
#undef ZR_WS64
#undef ZR_WS128

}  // namespace

// nullptr when the layer does not fit the form: an input that is not a plain CNHW tensor with
// 16-B aligned channel planes, or a (kernel, stride, width, Mpad) without an instance above, or
// too few tiles.  launch = false: only whether it would run.
const char *launch_dwpw_ws(const DwPwParams &p, hipStream_t s, bool launch) {
    if (!ws_enabled() || p.g.K % 4 || p.in.sN != (int64_t)p.in.H * p.in.W || p.in.sC % 4 ||
        ((uintptr_t)p.in.p | (uintptr_t)p.g.wt | (uintptr_t)p.dw_w | (uintptr_t)p.dw_b) % 16 ||
        (p.dw_act.kind == ACT_PRELU && (uintptr_t)p.dw_act.slope % 16))
        return nullptr;
    return ws_dispatch(p, s, launch);
}

}  // namespace zr
