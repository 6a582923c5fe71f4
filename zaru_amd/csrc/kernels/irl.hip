// irl.hip -- the MobileNetV2 inverted residual of the hand landmark network's low-resolution
// blocks (14^2 planes with 288 / 384 expanded channels, 7^2 with 672) in one launch.  Reference:
// the Conv / Clip / Add nodes of hand_landmark_lite.onnx that ORT / tract execute at
// crates/zaru/src/nn/mod.rs:483-533 (hand/landmark.rs:251-322).
//
// Unfused, each of these blocks is an expand GEMM that writes 4-6x the block's channels to HBM
// and a depthwise -> 1x1 launch that reads them back over 18-42 serial 16-channel chunks, with a
// DMA round trip per chunk (profiles/r05_layers/: 170-190 us per block at 341 ROIs).  Here one
// 512-thread workgroup owns one image's whole plane (196 or 49 positions) and walks the expanded
// channels in chunks of 16 as a three-stage pipeline, one barrier per step:
//   * waves 0-3 (one per SIMD) run the matrix work of step t: the expand of chunk t on f32 MFMA
//     (v_mfma_f32_16x16x4f32; A = the chunk's 16 rows of the expand weights, loaded a step ahead;
//     B = the block input, in registers for the whole launch) + bias, activation, into a
//     zero-bordered padded plane in LDS (the border is the depthwise's zero padding, written
//     once), then the projection of chunk t - 2 (v_mfma_f32_32x32x2f32 into registers; a wave
//     owns one 32-row slice and every (4 / slices)-th 32-column tile);
//   * waves 4-7 run the depthwise of chunk t - 1 beside them, as row tasks (RW adjacent outputs of
//     one row of one channel: each of the K input rows read once, 8-byte LDS reads where rows are
//     aligned; K^2 weights and the bias from LDS) into a [16][columns] tile, and stage chunk t's
//     depthwise weights;
//   * planes, tiles and weights are double-buffered by step parity; the barrier waits for LDS
//     traffic only, so the next step's weight loads stay in flight.
// Epilogue: epilogue_tile (bias, activation, residual, activation), as the unfused launches.
//
// Arithmetic and order are the unfused launches': the expand is an f32 MFMA chain over k in order
// (16x16x4 and 32x32x2 both sum an output's products in k order like an fmaf chain --
// tools/debug/mfma_order.hip, profiles/r04_mfma_order_probe.json) then + bias and the activation
// (gemm_tiled_kernel's epilogue); the depthwise is bias + fmaf over the taps in (ky, kx) order
// with the padding read as +0 (the masked taps' fmaf(w, 0, a)); the projection the same MFMA
// chain over the expanded channels.  So fusing changes no output bit (tests/test_gpu_forms.py,
// -irl).
#include "../runtime/zr_kernels.h"
#include "act.h"
#include "epilogue.h"

namespace zr {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int IRL_CEC = 16;  // expanded channels per chunk

// ZR_IRL_TRACE (tools/debug/irl_trace.sh builds a separate library with it; never the product):
// lane 0 of every wave of the first IRL_TRACE_WG workgroups stores the shader clock (s_memtime)
// at the start of each step and where its work ends before the step's barrier, into a device
// buffer of IRL_TRACE_LAUNCHES launches x IRL_TRACE_WG workgroups x 8 waves x 256 slots (slot 4 t +
// 2: step t starts, + 3: the M waves' expand / the D waves' staging is issued, + 4: its work ends;
// 0 / 1: the prologue, 254 / 255: the epilogue).
#ifdef ZR_IRL_TRACE
constexpr int IRL_TRACE_WG = 16, IRL_TRACE_LAUNCHES = 32;
__device__ unsigned long long zr_irl_trace_buf[IRL_TRACE_LAUNCHES * IRL_TRACE_WG * 8 * 256];
// (the clocks go to LDS during the steps -- a global store there would sit in the wave's vmcnt
// and delay the next wait for its weight loads -- and to the buffer after the epilogue)
#define IRL_TS(slot) \
    if (lane == 0) sT[wave][slot] = __builtin_amdgcn_s_memtime();
#define IRL_TRACE_ARG , int tslot
#else
#define IRL_TS(slot)
#define IRL_TRACE_ARG
#endif

// a workgroup barrier that waits for this wave's LDS traffic, not its vector-memory loads
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS layout of an instance (LV > 0): the padded planes' row pitch, their stride and the depthwise
// tile's channel stride, chosen with tools/lds_banks_irl.py's bank model (MI355X_MICROARCH.md §LDS)
// over the expand's stores, the row tasks' window reads and their tile stores.  The plain layout
// (row pitch = the padded width rounded to even, packed planes, NI * NCP tile rows) puts a
// half-wave's 14 row tasks of one channel on 2-4 bank groups (pitch 16: lanes 64 B apart) and the
// 4 channels of an expand store 4 * PP apart on the same banks.
struct IrlLds {
    int pw, pp, dc;  // row pitch (>= padded width, even), plane pad, tile channel pad (floats)
};
// LV 2: for 16-byte window reads (ds_read_b128 from 16-byte aligned rows: pitch and strides % 4
// == 0).  PMC at 341 ROIs: 1.85-2.93 -> 0.26-0.34 conflict cycles per LDS instruction, and every
// launch within +-2 us (the step is not bound by LDS banks: profiles/r06_layers/
// hand_landmark_lite_341_irllds_vs_plain.txt); the stride-2 14^2 block at two images per
// workgroup spills at this layout (108 -> 140 us) and keeps the plain one.
constexpr IrlLds irl_lds(int K, int HW, int S, int NI, int LV) {
    if (LV >= 2) {
        if (K == 3 && HW == 14 && S == 1) return {20, 24, 4};
        if (K == 5 && HW == 14 && S == 1) return {20, 48, 4};
        if (K == 5 && HW == 14 && S == 2) return {20, 16, 8};
        if (K == 5 && HW == 7 && S == 1) return {12, 16, NI == 1 ? 8 : 4};
    }
    return {0, 0, 0};
}

// HW: input plane side; S: the depthwise stride (TF-style 'same' padding: the output plane is
// HW / S); CX: block-input channels (the expand's K); MP: 32-row slices of the projection (Mpad / 32);
// NI: images per workgroup (2 at 7^2: each M wave then runs two independent MFMA chains, and a
// few hundred ROIs fill the CUs in one round instead of one and a third); LV: the LDS layout
// (irl_lds; 2: the window rows read as whole 16-byte vectors)
template <int K, int HW, int S, int CX, int MP, int NI, int LV>
__global__ __launch_bounds__(512) void irl_kernel(const GemmParams E, const DwPwParams D IRL_TRACE_ARG) {
    constexpr int HO = HW / S, P = HW * HW, PO = HO * HO, PL = S == 1 ? K / 2 : K / 2 - 1;
    constexpr IrlLds LY = irl_lds(K, HW, S, NI, LV);
    constexpr int PH = (HO - 1) * S + K, PW0 = (PH + 1) & ~1;
    constexpr int PW = LY.pw > PW0 ? LY.pw : PW0, PP = PH * PW + LY.pp;  // padded plane (even rows)
    constexpr int NE = (P + 15) / 16, NET = NI * NE, NEW = (NET + 3) / 4;   // expand column tiles (per M wave)
    constexpr int NCT = (PO + 31) / 32, NCP = NCT * 32, NCTT = NI * NCT;    // projection column tiles (per image)
    constexpr int DCS = NI * NCP + LY.dc;                                   // tile channel stride
    constexpr int CPW = 4 / MP, TPW = (NCTT + CPW - 1) / CPW;          // tile stride, tiles per M wave
    constexpr int KS = CX / 4, KK = K * K, NSW = IRL_CEC * KK + IRL_CEC;
    // depthwise task: RW outputs of a row (a half row when whole rows leave half the D threads idle)
    constexpr int RW = IRL_CEC * HO * 2 <= 256 && HO % 2 == 0 ? HO / 2 : HO, RPR = HO / RW;
    constexpr int WWIN = LV >= 2 ? ((RW - 1) * S + K + 3) & ~3  // window floats per input row (% 4)
                                 : ((RW - 1) * S + K + 1) & ~1;  // (even)
    constexpr bool W64 = RW == HO || S == 2;           // 8-byte aligned window starts: 8-byte reads
    constexpr int NTASK = IRL_CEC * HO * RPR;          // depthwise tasks per image
    static_assert(4 % MP == 0 && CX % 4 == 0 && NI * NTASK <= 256 && NE >= 4 && HW % S == 0, "irl layout");
    static_assert(LV < 2 || (RPR == 1 && PW % 4 == 0 && PP % 4 == 0 && W64), "irl: 16-byte aligned window rows");
    // image j of the workgroup: planes sE[.][j][c], tile columns sD[.][c][j * NCP + q]
    __shared__ __attribute__((aligned(16))) float sE[2][NI * IRL_CEC * PP];  // expanded planes (zero border)
    __shared__ __attribute__((aligned(16))) float sD[2][IRL_CEC * DCS];  // depthwise tiles
    __shared__ float sW[2][NSW];  // a chunk's depthwise weights, then its biases
    // the M waves' operands of step t in sM[t & 1]: chunk t's expand weights [CX][16] and biases,
    // then chunk t - 2's projection weights [16][MP * 32]
    constexpr int MWA = 0, MB = CX * IRL_CEC, MW2 = MB + IRL_CEC, NSM = MW2 + IRL_CEC * MP * 32;
    __shared__ __attribute__((aligned(16))) float sM[2][NSM];
#ifdef ZR_IRL_TRACE
    __shared__ unsigned long long sT[8][256];
#endif

    const GemmParams &G = D.g;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n0 = blockIdx.x * NI;  // images n0 .. n0 + NI - 1 below nlim
    const int nimg = D.g.ncols / PO, nlim = G.nact && *G.nact < nimg ? *G.nact : nimg;
    if (n0 >= nlim) return;  // (whole workgroup, before any barrier)
    const int nch = E.M / IRL_CEC;
    const bool mrole = wave < 4;         // waves 0-3: MFMA (expand, projection); 4-7: depthwise

    for (int i = tid; i < 2 * NI * IRL_CEC * PP; i += 512) (&sE[0][0])[i] = 0.f;  // the borders stay 0

    // ---- M waves: expand operands (lane (col, kq): x[4 s + kq][t * 16 + col] of tiles
    // t = wave + 4 i as B -- tile t is tile t % NE of image t / NE; W1[c0 + col][4 s + kq] as A)
    // and projection accumulators (32-row slice m0, column tiles ct0, ct0 + CPW, ...)
    const int col = lane & 15, kq = lane >> 4;
    const int mw = wave & 3;
    const int m0 = (mw % MP) * 32, ct0 = mw / MP;
    const int pcol = lane & 31, kh = lane >> 5;
    float xr[NEW][KS];
    f32x16 acc[TPW];
    if (mrole) {
#pragma unroll
        for (int i = 0; i < NEW; ++i) {
            const int t = mw + 4 * i, j = t / NE, p = (t - j * NE) * 16 + col;
            const int ni = t < NET && n0 + j < nlim ? n0 + j : n0;
            const float *xb = E.x + (size_t)(uint32_t)ni * (uint32_t)E.x_sN;
            const uint32_t pc = t < NET && p < P ? (uint32_t)p : 0u;
#pragma unroll
            for (int s = 0; s < KS; ++s) xr[i][s] = xb[(uint32_t)(4 * s + kq) * (uint32_t)E.x_sC + pc];
        }
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    }
    const Bounds eb = bounds(E.pre), db = bounds(D.dw_act);  // (E.post: none, host-checked)

    // ---- D waves: channel dc of a chunk, outputs dx0 .. dx0 + RW - 1 of row dy
    const int dt = tid - 256;
    const bool dw_on = !mrole && dt < NI * NTASK;
    const int dj = dw_on ? dt / NTASK : 0, dtj = dt - dj * NTASK;  // image dj of the workgroup
    const int dc = dw_on ? dtj / (HO * RPR) : 0, dr = dtj - dc * HO * RPR, dy = dr / RPR, dx0 = (dr - dy * RPR) * RW;
    // The D waves stage every weight through LDS, loaded a step ahead into registers and stored
    // in the step before their use; the M waves then issue no memory loads in the step loop
    // (the compiler's vmcnt waits for operand registers loaded one or two steps earlier counted
    // the newest loads too, so each step paid a whole memory latency).
    // M operands of step ce: 16-byte pieces (expand rows of 16, biases, projection rows),
    // chunk indices clamped past the ends.
    constexpr int NF = NSM / 4, NFR = (NF + 255) / 256;
    float mr[4 * NFR];  // (scalars: a float4 array of this shape was kept in scratch)
    auto load_m = [&](int ce) {
        const int c0 = (ce < nch ? ce : nch - 1) * IRL_CEC;
        const int c2 = (ce < 2 ? 0 : ce - 2 < nch ? ce - 2 : nch - 1) * IRL_CEC;
#pragma unroll
        for (int j = 0; j < NFR; ++j) {
            // (branch-free, from a clamped piece: a private array behind branches goes to scratch)
            const int f = dt + 256 * j < NF ? dt + 256 * j : NF - 1, e = 4 * f;
            const int k = e / IRL_CEC, r = (e - MW2) / (MP * 32);
            const uint32_t oa = (uint32_t)k * (uint32_t)E.Mpad + (uint32_t)(c0 + e - k * IRL_CEC);
            const uint32_t ob = (uint32_t)(c0 + e - MB);
            const uint32_t o2 = (uint32_t)(c2 + r) * (uint32_t)G.Mpad + (uint32_t)(e - MW2 - r * MP * 32);
            const float *src = e < MB ? E.wt + oa : e < MW2 ? E.bias + ob : G.wt + o2;
            const float4 v = *reinterpret_cast<const float4 *>(src);
            mr[4 * j] = v.x;
            mr[4 * j + 1] = v.y;
            mr[4 * j + 2] = v.z;
            mr[4 * j + 3] = v.w;
        }
    };
    auto store_m = [&](int ce) {
#pragma unroll
        for (int j = 0; j < NFR; ++j)
            if (dt + 256 * j < NF) reinterpret_cast<float4 *>(sM[ce & 1])[dt + 256 * j] = make_float4(mr[4 * j], mr[4 * j + 1], mr[4 * j + 2], mr[4 * j + 3]);
    };
    // chunk c's depthwise weights and biases (NSW <= 512: two words per D thread)
    constexpr int NSR = (NSW + 255) / 256;
    float swr[NSR];
    auto load_w = [&](int c) {
        c = c < nch ? c : nch - 1;
#pragma unroll
        for (int j = 0; j < NSR; ++j) {
            const int i = dt + 256 * j;
            swr[j] = i < IRL_CEC * KK ? D.dw_w[c * IRL_CEC * KK + i] : i < NSW ? D.dw_b[c * IRL_CEC + i - IRL_CEC * KK] : 0.f;
        }
    };

    // Step t: the M waves expand chunk t into sE[t & 1] and project chunk t - 2 from sD[t & 1];
    // the D waves run chunk t - 1's depthwise (sE[(t - 1) & 1] -> sD[(t - 1) & 1]) and stage chunk
    // t's depthwise weights.  One barrier per step hands the buffers over.
    auto step = [&](int t) {
        IRL_TS(4 * t + 2);
        const float *sm = sM[t & 1];
        if (mrole) {
            if (t < nch) {
                // expand; each tile's MFMA chain is issued before the previous tile's epilogue
                float *pe = sE[t & 1];
                float wa[KS], bias[4];
#pragma unroll
                for (int s = 0; s < KS; ++s) wa[s] = sm[MWA + (4 * s + kq) * IRL_CEC + col];
#pragma unroll
                for (int r = 0; r < 4; ++r) bias[r] = sm[MB + 4 * kq + r];
                auto chain = [&](int i) {
                    f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int s = 0; s < KS; ++s) d = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[s], xr[i][s], d, 0, 0, 0);
                    return d;
                };
                auto epi = [&](int i, const f32x4 &d) {  // gemm_tiled_kernel's epilogue (RES = false)
                    const int t = mw + 4 * i, j = t / NE, p = (t - j * NE) * 16 + col;
                    if (p < P) {
                        const int y = p / HW, x = p - y * HW;
                        float *e = pe + (j * IRL_CEC + 4 * kq) * PP + (y + PL) * PW + x + PL;
#pragma unroll
                        for (int r = 0; r < 4; ++r) e[r * PP] = clamp(eb, d[r] + bias[r]);
                    }
                };
                f32x4 dcur = chain(0);
#pragma unroll
                for (int i = 0; i < NEW; ++i) {
                    f32x4 dn = dcur;
                    if (i + 1 < NEW && mw + 4 * (i + 1) < NET) dn = chain(i + 1);
                    if (mw + 4 * i < NET) epi(i, dcur);  // (wave-uniform)
                    dcur = dn;
                }
            }
            IRL_TS(4 * t + 3);
            if (t >= 2) {
                // projection: acc += W2[m0 .. m0 + 31][chunk t - 2] x its depthwise tile
                const float *pd = sD[t & 1];
#pragma unroll
                for (int s = 0; s < IRL_CEC / 2; ++s) {
                    const float w2 = sm[MW2 + (2 * s + kh) * (MP * 32) + m0 + pcol];
                    const float *b = pd + (2 * s + kh) * DCS + pcol;
#pragma unroll
                    for (int i = 0; i < TPW; ++i) {
                        const int ct = ct0 + CPW * i;
                        if (ct < NCTT) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(w2, b[ct * 32], acc[i], 0, 0, 0);
                    }
                }
            }
        } else {
            // the stores of last step's loads first: a store after this step's loads would wait
            // for them too
            if (t < nch) {
#pragma unroll
                for (int j = 0; j < NSR; ++j)
                    if (dt + 256 * j < NSW) sW[t & 1][dt + 256 * j] = swr[j];
            }
            store_m(t + 1);  // (read in step t + 1; step t reads the other buffer)
            IRL_TS(4 * t + 5);
            if (t < nch) load_w(t + 1);
            load_m(t + 2);
            IRL_TS(4 * t + 3);
            if (t >= 1 && t <= nch && dw_on) {
                // depthwise of chunk t - 1: RW outputs of one row of one channel, each input row once
                const float *w = sW[(t - 1) & 1] + dc * KK;
                const float *pe = sE[(t - 1) & 1] + (dj * IRL_CEC + dc) * PP + dx0 * S;
                float a[RW];
                const float bb = sW[(t - 1) & 1][IRL_CEC * KK + dc];
#pragma unroll
                for (int o = 0; o < RW; ++o) a[o] = bb;
                if constexpr (LV >= 3) {
                    // the window rows double-buffered: row ky + 1's reads are issued before row
                    // ky's FMAs, and each vector is taken whole just before its use (the one
                    // depthwise wave per SIMD otherwise waits out an LDS latency per row)
                    constexpr int NR = WWIN / 4;
                    f32x4 rb[2][NR];
#pragma unroll
                    for (int e = 0; e < NR; ++e) rb[0][e] = reinterpret_cast<const f32x4 *>(pe + dy * S * PW)[e];
#pragma unroll
                    for (int ky = 0; ky < K; ++ky) {
                        // this row's weights first: LDS returns in order, so waiting for them
                        // does not wait for the next row's reads issued after them
                        float wr[K];
#pragma unroll
                        for (int kx = 0; kx < K; ++kx) wr[kx] = w[ky * K + kx];
                        if (ky + 1 < K) {
#pragma unroll
                            for (int e = 0; e < NR; ++e)
                                rb[(ky + 1) & 1][e] = reinterpret_cast<const f32x4 *>(pe + (dy * S + ky + 1) * PW)[e];
                        }
                        __builtin_amdgcn_sched_barrier(0);  // (keep the reads ahead of the FMAs)
                        float xw[WWIN];
#pragma unroll
                        for (int e = 0; e < NR; ++e) {
                            f32x4 v = rb[ky & 1][e];
                            asm("" : "+v"(v));
#pragma unroll
                            for (int i = 0; i < 4; ++i) xw[4 * e + i] = v[i];
                        }
#pragma unroll
                        for (int kx = 0; kx < K; ++kx) {
#pragma unroll
                            for (int o = 0; o < RW; ++o) a[o] = __builtin_fmaf(wr[kx], xw[o * S + kx], a[o]);
                        }
                    }
                } else {
#pragma unroll
                    for (int ky = 0; ky < K; ++ky) {
                        const float *row = pe + (dy * S + ky) * PW;
                        float xw[WWIN];
                        if constexpr (W64) {
                            if constexpr (LV >= 2) {
#pragma unroll
                                for (int e = 0; e < WWIN / 4; ++e) {
                                    f32x4 v = reinterpret_cast<const f32x4 *>(row)[e];
                                    asm("" : "+v"(v));  // (whole: no narrowed / re-paired reads)
#pragma unroll
                                    for (int i = 0; i < 4; ++i) xw[4 * e + i] = v[i];
                                }
                            } else {
#pragma unroll
                                for (int e = 0; e < WWIN / 2; ++e) {
                                    const float2 v = reinterpret_cast<const float2 *>(row)[e];
                                    xw[2 * e] = v.x;
                                    xw[2 * e + 1] = v.y;
                                }
                            }
                        } else {
#pragma unroll
                            for (int e = 0; e < (RW - 1) * S + K; ++e) xw[e] = row[e];
                        }
#pragma unroll
                        for (int kx = 0; kx < K; ++kx) {
                            const float wt = w[ky * K + kx];
#pragma unroll
                            for (int o = 0; o < RW; ++o) a[o] = __builtin_fmaf(wt, xw[o * S + kx], a[o]);
                        }
                    }
                }
                float *dst = sD[(t - 1) & 1] + dc * DCS + dj * NCP + dy * HO + dx0;
#pragma unroll
                for (int o = 0; o < RW; ++o) dst[o] = clamp(db, a[o]);
            }
        }
        IRL_TS(4 * t + 4);
        lds_barrier();
    };

    IRL_TS(0);
    if (!mrole) {
        load_w(0);
        load_m(0);
        store_m(0);
        load_m(1);
    }
    IRL_TS(1);
    lds_barrier();  // the zeroed planes, step 0's M operands
    for (int t = 0; t < nch + 2; t += 2) {  // (nch even, host-checked: buffer t & 1 is static)
        step(t);
        step(t + 1);
    }

    IRL_TS(254);
    if (mrole) {
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int ct = ct0 + CPW * i, j = ct / NCT;
            const int q = (ct - j * NCT) * 32 + pcol;
            if (ct < NCTT && q < PO && n0 + j < nlim) {
                // opaque row base / half: otherwise the compiler hoists every row's channel index
                // and bias / residual address out of the step loop and holds them across it
                int mb = m0, h = kh;
                asm volatile("" : "+v"(mb), "+v"(h));
                epilogue_tile(G, acc[i], n0 + j, q, mb, h);
            }
        }
    }
    IRL_TS(255);
#ifdef ZR_IRL_TRACE
    if (blockIdx.x < IRL_TRACE_WG)
        for (int i = lane; i < 256; i += 64)
            zr_irl_trace_buf[(((tslot % IRL_TRACE_LAUNCHES) * IRL_TRACE_WG + blockIdx.x) * 8 + wave) * 256 + i] = sT[wave][i];
#endif
}

#ifdef ZR_IRL_TRACE
int irl_trace_launches = 0;  // (trace builds: the buffer's launch slot of the next irl launch)
#endif

// ZARU_HIP_IRL_LDS (A/B knob, bitwise neutral): 0 the plain layout everywhere, 2 the padded one,
// 3 (default) padded + double-buffered window rows
int irl_lds_env() {
    static const int v = [] {
        const char *e = std::getenv("ZARU_HIP_IRL_LDS");
        return e ? (int)std::strtol(e, nullptr, 10) : 3;
    }();
    return v;
}

template <int K, int HW, int S, int CX, int MP, int NI = 1>
const char *irl_go(const GemmParams &e, const DwPwParams &d, hipStream_t s) {
    const int N = d.g.ncols / ((HW / S) * (HW / S));
    constexpr bool padded = !(S == 2 && NI == 2);
#ifdef ZR_IRL_TRACE
#define IRL_TRACE_PASS , irl_trace_launches++
#else
#define IRL_TRACE_PASS
#endif
    const int lv = irl_lds_env();
    if (padded && lv >= 3)
        hipLaunchKernelGGL((irl_kernel<K, HW, S, CX, MP, NI, padded ? 3 : 0>), dim3((N + NI - 1) / NI), dim3(512), 0, s, e, d IRL_TRACE_PASS);
    else if (padded && lv == 2)
        hipLaunchKernelGGL((irl_kernel<K, HW, S, CX, MP, NI, padded ? 2 : 0>), dim3((N + NI - 1) / NI), dim3(512), 0, s, e, d IRL_TRACE_PASS);
    else hipLaunchKernelGGL((irl_kernel<K, HW, S, CX, MP, NI, 0>), dim3((N + NI - 1) / NI), dim3(512), 0, s, e, d IRL_TRACE_PASS);
    return NI == 1 ? kernel_name("irl_kernel<%d,%d,%d,%d,%d>", K, HW, S, CX, MP)
                   : kernel_name("irl_kernel<%d,%d,%d,%d,%d,%d>", K, HW, S, CX, MP, NI);
}

// CUs of the current device
int cu_count() {
    static const int ncu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    return ncu;
}

}  // namespace

#ifdef ZR_IRL_TRACE
// the trace buffer, for tools/debug/irl_trace.py (trace builds only)
extern "C" int zr_debug_irl_trace(unsigned long long *dst, size_t n, int clear) {
    const size_t cap = sizeof(zr_irl_trace_buf) / sizeof(zr_irl_trace_buf[0]);
    if (n > cap) n = cap;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(dst, HIP_SYMBOL(zr_irl_trace_buf), n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    if (clear) {
        static unsigned long long zero[IRL_TRACE_LAUNCHES * IRL_TRACE_WG * 8 * 256];
        if (hipMemcpyToSymbol(HIP_SYMBOL(zr_irl_trace_buf), zero, sizeof(zero), 0, hipMemcpyHostToDevice) != hipSuccess) return -1;
    }
    return (int)n;
}
#endif

// The fused form applies to an expand (1x1, no residual, CNHW input) whose output only the next
// depthwise -> 1x1 step reads (plan.cpp mark_inverted_residuals), with the models' TF-style
// 'same' padding over a 14^2 or 7^2 plane (stride 1, or stride 2 from 14^2 to 7^2), with
// expanded channels in whole chunks of 16, Relu / Clip activations on the expand and depthwise,
// and the hand network's (K, plane, stride, input channels, output rows) combinations.
const char *launch_irl(const GemmParams &e, const DwPwParams &d, hipStream_t s) {
    const int S = d.stride, pl = S == 1 ? d.k / 2 : d.k / 2 - 1;
    if (!form_on(FORM_IRL) || e.KK != 1 || e.res_mode != 0 || e.x_sN != e.P || e.M != d.g.K || e.M % IRL_CEC != 0 ||
        e.out != d.in.p || e.nact != d.g.nact || (S != 1 && S != 2) || d.in.H != d.in.W || d.in.W % S != 0 ||
        d.OW * S != d.in.W || d.g.P != d.OW * d.OW || e.P != d.in.H * d.in.W || d.in.sN != (int64_t)e.P ||
        d.g.o_sP != 1 || d.g.ncols % d.g.P != 0 || e.ncols != d.in.H * d.in.W * (d.g.ncols / d.g.P) ||
        d.pad_t != pl || d.pad_l != pl || d.g.res_mode == 2 || (d.g.res_mode == 1 && S != 1) ||
        e.M % (2 * IRL_CEC) != 0 || e.post.kind != ACT_NONE || !bounds_act(e.pre) || !bounds_act(d.dw_act))
        return nullptr;
    const int hw = d.in.W, cx = e.K, mp = d.g.Mpad / 32;
    // (the weights are staged in 16-byte pieces)
    if (d.g.Mpad % 32 != 0 || e.Mpad % 4 != 0 || ((uintptr_t)e.wt | (uintptr_t)e.bias | (uintptr_t)d.g.wt) % 16 != 0)
        return nullptr;
    if (S == 1 && d.k == 3 && hw == 14 && cx == 48 && mp == 2) return irl_go<3, 14, 1, 48, 2>(e, d, s);
    if (S == 1 && d.k == 5 && hw == 14 && cx == 48 && mp == 2) return irl_go<5, 14, 1, 48, 2>(e, d, s);
    if (S == 1 && d.k == 5 && hw == 14 && cx == 64 && mp == 2) return irl_go<5, 14, 1, 64, 2>(e, d, s);
    if (S == 1 && d.k == 5 && hw == 7 && cx == 112 && mp == 4) {
        // two images per workgroup once the images outnumber the CUs (below that, halving the
        // workgroups leaves CUs idle)
        if (form_on(FORM_IRL2) && d.g.ncols / d.g.P > cu_count()) return irl_go<5, 7, 1, 112, 4, 2>(e, d, s);
        return irl_go<5, 7, 1, 112, 4>(e, d, s);
    }
    if (S == 2 && d.k == 5 && hw == 14 && cx == 64 && mp == 4) {
        if (form_on(FORM_IRL2) && d.g.ncols / d.g.P > cu_count()) return irl_go<5, 14, 2, 64, 4, 2>(e, d, s);
        return irl_go<5, 14, 2, 64, 4>(e, d, s);
    }
    return nullptr;
}

}  // namespace zr
