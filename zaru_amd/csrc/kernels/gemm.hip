// gemm.hip -- 1x1 convolution / Gemm / full-plane convolution as an f32 MFMA GEMM with the
// whole BlazeBlock tail fused into the epilogue (bias, activation, channel-padded and
// optionally 2x2-max-pooled residual, second activation) and the graph-output layout
// (Transpose/Reshape/Concat) folded into the store addressing.
//
// out[m][j] = post( pre( sum_k W[m][k] * X[k][j] + b[m] ) + R[m][j] ),  j = n*P + q.
//
// Tiling (gfx950, wave64): v_mfma_f32_32x32x2_f32 (exact f32, 64 FLOP/clk/SIMD, the same
// rate as the f32 VALU).  A workgroup is 4 waves; each wave owns 32 columns and MT 32-row
// tiles (MT*16 accumulator VGPRs).  Weights are staged through LDS in K-chunks of 32 rows
// ([k][m] layout: a half-wave reads 32 consecutive floats, conflict-free); the activation
// operand is read straight from HBM into the B fragment (lane l: X[k0 + l/32][j0 + l%32],
// two fully coalesced 128-B rows per wave instruction), 16 loads per lane in flight.
// Reference: the 1x1 Conv / Gemm nodes of the four ONNX graphs executed by ORT/tract at
// crates/zaru/src/nn/mod.rs:483-533.
#include "../runtime/zr_kernels.h"
#include <algorithm>
#include <cstdlib>
#include "act.h"
#include "epilogue.h"
#include "group.h"

namespace zr {

constexpr int KC = 32;  // K rows per LDS stage

// (the kernel bodies take their block coordinates as arguments: a grouped launch, group.h,
// runs them for several parts of one grid)
template <int MT, bool FULLPLANE>
__device__ __forceinline__ void gemm_body(const GemmParams &P, int bx, int by) {
    __shared__ float sW[KC][MT * 32];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kh = lane >> 5, col = lane & 31;
    const int m0 = by * (MT * 32);
    if (P.nact && bx * 128 >= *P.nact * P.P) return;  // (whole workgroup) images past the device count
    const int j = (bx * 4 + wave) * 32 + col;
    const bool valid = j < P.ncols;
    const int jj = valid ? j : 0;
    const int n = jj / P.P, q = jj - n * P.P;
    const float *xc;
    // im2col walk of this lane's k = kh, kh + 2, ... as (ci, ky, kx): no per-element division
    int ci = 0, ky = 0, kx = kh;
    if constexpr (FULLPLANE) {
        const int oy = q / P.out_W, ox = q - oy * P.out_W;
        xc = P.x + (int64_t)n * P.x_sN + (int64_t)oy * P.ph * P.x_W + ox * P.pk;
        ky = kh / P.pk;
        kx = kh - ky * P.pk;
    } else {
        xc = P.x + (int64_t)n * P.x_sN + q;
    }

    f32x16 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    for (int kc = 0; kc < P.Kpad; kc += KC) {
        __syncthreads();
        for (int i = threadIdx.x; i < KC * MT * 32; i += 256) {
            const int r = i / (MT * 32), c = i - r * (MT * 32);
            const int kk = kc + r, mm = m0 + c;
            sW[r][c] = (kk < P.Kpad && mm < P.Mpad) ? P.wt[(int64_t)kk * P.Mpad + mm] : 0.f;
        }
        // activation fragments for this chunk: load from a clamped (always valid) row and
        // zero the padded rows with a select, so no load sits behind a branch.
        float b[KC / 2];
#pragma unroll
        for (int s = 0; s < KC / 2; ++s) {
            const int k = kc + 2 * s + kh;
            const int kcl = k < P.K ? k : P.K - 1;
            float v;
            if constexpr (FULLPLANE) {
                v = xc[k < P.K ? (int64_t)ci * P.x_sC + ky * P.x_W + kx : 0];
                kx += 2;  // pk >= 2: at most one wrap of kx, then of ky (which wraps at ph)
                const bool wx = kx >= P.pk;
                kx -= wx ? P.pk : 0;
                ky += wx ? 1 : 0;
                const bool wy = ky >= P.ph;
                ky -= wy ? P.ph : 0;
                ci += wy ? 1 : 0;
            } else {
                v = xc[(int64_t)kcl * P.x_sC];
            }
            b[s] = k < P.K ? v : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < KC / 2; ++s)
#pragma unroll
            for (int t = 0; t < MT; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(sW[2 * s + kh][t * 32 + col], b[s],
                                                              acc[t], 0, 0, 0);
    }

    if (!valid) return;
#pragma unroll
    for (int t = 0; t < MT; ++t) epilogue_tile(P, acc[t], n, q, m0 + t * 32, kh);
}

template <int MT, bool FULLPLANE>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmParams P) {
    gemm_body<MT, FULLPLANE>(P, blockIdx.x, blockIdx.y);
}

template <int MT, bool FULLPLANE>
__global__ __launch_bounds__(256) void gemm_group_kernel(const LaunchGroup<GemmParams> G) {
    const GroupSlot t = group_slot(G);
    gemm_body<MT, FULLPLANE>(G.p[t.g], t.bx, t.by);
}

// Small-K form of gemm_kernel<1, false> (K <= NCH * 32, M <= 32: the FaceMesh tail's 128 -> 32
// 1x1 convs over batch x 3x3 columns that the LDS-tiled form cannot take, ncols % 4 != 0).  Every
// operand of the whole K extent is loaded up front in straight-line code (the weights straight
// from global memory: 16 KB, L2-resident), so the launch costs one load latency instead of one
// per chunk (gemm_kernel stages each chunk through LDS behind two barriers).  The MFMA sequence
// is gemm_kernel's, operand for operand, so the bits are too.
template <int NCH>
__device__ __forceinline__ void gemm_smallk_body(const GemmParams &P, int bx) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kh = lane >> 5, col = lane & 31;
    const int j = (bx * 4 + wave) * 32 + col;
    const bool valid = j < P.ncols;
    const int jj = valid ? j : 0;
    const int n = jj / P.P, q = jj - n * P.P;
    const float *xc = P.x + (int64_t)n * P.x_sN + q;
    float a[NCH * KC / 2], b[NCH * KC / 2];
#pragma unroll
    for (int s = 0; s < NCH * KC / 2; ++s) {
        const int k = 2 * s + kh;
        a[s] = k < P.Kpad && col < P.Mpad ? P.wt[(int64_t)(k < P.Kpad ? k : 0) * P.Mpad + col] : 0.f;
        const float v = xc[(int64_t)(k < P.K ? k : P.K - 1) * P.x_sC];
        b[s] = k < P.K ? v : 0.f;
    }
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int s = 0; s < NCH * KC / 2; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
    if (!valid) return;
    epilogue_tile(P, acc, n, q, 0, kh);
}

template <int NCH>
__global__ __launch_bounds__(256) void gemm_smallk_kernel(const GemmParams P) {
    gemm_smallk_body<NCH>(P, blockIdx.x);
}

template <int NCH>
__global__ __launch_bounds__(256) void gemm_smallk_group_kernel(const LaunchGroup<GemmParams> G) {
    const GroupSlot t = group_slot(G);
    gemm_smallk_body<NCH>(G.p[t.g], t.bx);
}

// ---------------------------------------------------------------- LDS-tiled variant
// For the common case of a CNHW activation (X is then a plain row-major [K][ncols] matrix with
// leading dimension x_sC) with ncols % 4 == 0: both operands are staged through LDS with
// 16-byte loads (one wave instruction moves a whole 1 KiB row segment), double-buffered with
// the next K-chunk's loads in flight during the current chunk's MFMAs.  Each wave owns NT
// 32-column tiles x MT 32-row tiles, so every A fragment feeds NT MFMAs and every B fragment MT.
// Block -> tile mapping is XCD-aware (see gemm_tiled_body).
constexpr int TKC = 16;  // K rows per stage

// vec: the output tile leaves through LDS as 16-byte row segments (a wave's 32x32 tile in 4
// dwordx4 store instructions instead of 16 dword ones) -- the host sets it when a 4-column group
// never straddles an image and every row segment is 16-B aligned (o_sP == 1, P % 4 == 0, ...).
// (<1,1>: the skinny store-bound expand convs -- 4 waves per SIMD fit without spills and hide
// more of the store latency than 3)
template <int MT, int NT, bool RES>
__device__ __forceinline__ void gemm_tiled_body(const GemmParams &P, int mblocks, int nct, int vec, int bx, int gx) {
    constexpr int BN = 4 * NT * 32, MR = MT * 32;
    constexpr int XV = TKC * BN / 4 / 256;  // float4 of X staged per thread per chunk
    constexpr int WV = (TKC * MR / 4 + 255) / 256;
    __shared__ __attribute__((aligned(16))) float sX[2][TKC][BN];
    __shared__ __attribute__((aligned(16))) float sW[2][TKC][MR];

    // XCD-contiguous: launch slot bx runs on XCD bx % 8 (round-robin dispatch), and each XCD
    // takes one contiguous eighth of the (column tile, M block) pairs, M blocks innermost -- the
    // M blocks of a column tile share its X tile in that XCD's L2, and the XCD's output rows
    // leave as long runs of adjacent segments.
    const int idx = (bx & 7) * (gx >> 3) + (bx >> 3);
    const int ct = idx / mblocks, mb = idx - ct * mblocks;
    if (ct >= nct) return;  // whole workgroup, before any barrier
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kh = lane >> 5, col = lane & 31;
    const int j0 = ct * BN, m0 = mb * MR;
    if (P.nact && j0 >= *P.nact * P.P) return;  // images past the device count
    const int nchunks = (P.K + TKC - 1) / TKC;

    float4 rx[XV], rw[WV];
    auto load = [&](int kc) {
#pragma unroll
        for (int u = 0; u < XV; ++u) {
            const int i = tid + 256 * u, row = i / (BN / 4), c4 = i - row * (BN / 4);
            const int k = kc + row, j = j0 + 4 * c4;
            rx[u] = (k < P.K && j < P.ncols)
                        ? *reinterpret_cast<const float4 *>(P.x + (int64_t)k * P.x_sC + j)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < WV; ++u) {
            const int i = tid + 256 * u, row = i / (MR / 4), c4 = i - row * (MR / 4);
            const int k = kc + row;
            rw[u] = (i < TKC * MR / 4 && k < P.K && m0 + 4 * c4 < P.Mpad)
                        ? *reinterpret_cast<const float4 *>(P.wt + (int64_t)k * P.Mpad + m0 + 4 * c4)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int u = 0; u < XV; ++u) {
            const int i = tid + 256 * u, row = i / (BN / 4), c4 = i - row * (BN / 4);
            *reinterpret_cast<float4 *>(&sX[buf][row][4 * c4]) = rx[u];
        }
#pragma unroll
        for (int u = 0; u < WV; ++u) {
            const int i = tid + 256 * u, row = i / (MR / 4), c4 = i - row * (MR / 4);
            if (i < TKC * MR / 4) *reinterpret_cast<float4 *>(&sW[buf][row][4 * c4]) = rw[u];
        }
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int u = 0; u < NT; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;

    load(0);
    store(0);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        const int buf = c & 1;
        if (c + 1 < nchunks) load((c + 1) * TKC);
#pragma unroll
        for (int s = 0; s < TKC / 2; ++s) {
            float a[MT], b[NT];
#pragma unroll
            for (int t = 0; t < MT; ++t) a[t] = sW[buf][2 * s + kh][t * 32 + col];
#pragma unroll
            for (int u = 0; u < NT; ++u) b[u] = sX[buf][2 * s + kh][(wave * NT + u) * 32 + col];
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int u = 0; u < NT; ++u)
                    acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[u], acc[t][u], 0, 0, 0);
        }
        if (c + 1 < nchunks) store(buf ^ 1);
        __syncthreads();
    }

    if (vec) {
        // the loop's last barrier released sX: each wave takes 32x32 floats of it (BN >= 128)
        float *sT = &sX[0][0][0] + wave * 1024;
#pragma unroll
        for (int u = 0; u < NT; ++u) {
            const int jt = j0 + (wave * NT + u) * 32;
            const int j = min(jt + col, P.ncols - 1);
            const int n = j / P.P, q = j - n * P.P;
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                float v[16];
                epilogue_values<RES>(P, acc[t][u], n, q, m0 + t * 32, kh, v);
#pragma unroll
                for (int r = 0; r < 16; ++r) sT[mfma32_row(r, kh) * 32 + col] = v[r];
                __builtin_amdgcn_wave_barrier();  // LDS ops of a wave complete in order
                const int c4 = lane & 7, jj = jt + 4 * c4;
                const int nn = jj / P.P, qq = jj - nn * P.P;
#pragma unroll
                for (int it = 0; it < 4; ++it) {
                    const int rr = it * 8 + (lane >> 3), m = m0 + t * 32 + rr;
                    const float4 x = *reinterpret_cast<const float4 *>(sT + rr * 32 + 4 * c4);
                    if (jj < P.ncols && m < P.M)
                        *reinterpret_cast<float4 *>(P.out + (uint32_t)nn * (uint32_t)P.o_sN + (uint32_t)qq +
                                                    (uint32_t)m * (uint32_t)P.o_sC) = x;
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        return;
    }
#pragma unroll
    for (int u = 0; u < NT; ++u) {
        const int j = j0 + (wave * NT + u) * 32 + col;
        if (j >= P.ncols) continue;
        const int n = j / P.P, q = j - n * P.P;
#pragma unroll
        for (int t = 0; t < MT; ++t) epilogue_tile<RES>(P, acc[t][u], n, q, m0 + t * 32, kh);
    }
}

template <int MT, int NT, bool RES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MT * NT == 1 ? 4 : 1)))
void gemm_tiled_kernel(const GemmParams P, int mblocks, int nct, int vec) {
    gemm_tiled_body<MT, NT, RES>(P, mblocks, nct, vec, blockIdx.x, gridDim.x);
}

template <int MT, int NT, bool RES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MT * NT == 1 ? 4 : 1)))
void gemm_tiled_group_kernel(const LaunchGroup<GemmParams> G) {
    const GroupSlot t = group_slot(G);
    gemm_tiled_body<MT, NT, RES>(G.p[t.g], G.a0[t.g], G.a1[t.g], G.a2[t.g], t.bx, G.gx[t.g]);
}

// ---------------------------------------------------------------- image-row variant
// Full-plane convolutions on a 1-position output (the landmark heads: 3x3 conv over a 3x3
// plane, M = 1404 / 1, K = Cin * 9) with the images as the GEMM's rows: C^T[n][m] =
// X^T[n][k] . W^T[k][m].  The column-per-image form reads X with a stride of one image per lane
// and stores each output row with a stride of M per lane; here a lane's B fragment
// W^T[k][m0 + lane % 16] and its stores out[n][m0 + lane % 16] are coalesced rows, and the A
// fragment X^T[n0 + lane % 16][k] stays L1/L2-resident.  16x16 tiles of v_mfma_f32_16x16x4_f32:
// each wave's chain is K / 4 MFMAs of 8 passes (the 32x32x2 form: K / 2 of 16 passes, 4x the
// chain latency for these 1-output-position launches), and a launch has 4x the waves.  The
// 16x16x4 MFMA sums each output's products in k order exactly as the 32x32x2 one and an fmaf
// chain do (tools/debug/mfma_order.hip, profiles/r04_mfma_order_probe.json), so the bits are
// the other forms' (tests/test_gpu_forms.py switches this one off).
// NCH > 0: the K loop fully unrolled for exactly NCH 32-deep chunks (the FaceMesh heads: K = 288,
// 9 chunks): straight-line code keeps the next chunk's loads in flight (a runtime loop's back
// edge makes the compiler's wait counting drain them).
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int RC = 32;  // K per chunk (8 MFMA steps of 4)

template <bool FULLPLANE, int NCH>
__device__ __forceinline__ void gemm_rows_body(const GemmParams &P, int mtiles, int bx, int by) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int mt = by * 4 + wave;
    if (mt >= mtiles) return;  // no barriers in this kernel
    const int m0 = mt * 16, n0 = bx * 16;
    const int nimg = P.ncols;  // P == 1: one column per image
    const int na = min(n0 + r, nimg - 1);
    const float *xa = P.x + (int64_t)na * P.x_sN;
    const float *wb = P.wt + m0 + r;  // [Kpad][Mpad]

    float a[2][RC / 4], b[2][RC / 4];
    // k = ci * KK + kk of this lane's next A element, advanced by 4 per step (no division)
    int ci = 0, kk = kq;
    if constexpr (FULLPLANE) {
        while (kk >= P.KK) {
            kk -= P.KK;
            ++ci;
        }
    }
    auto load = [&](int kc, int buf) {
#pragma unroll
        for (int t = 0; t < RC / 4; ++t) {
            const int k = kc + 4 * t + kq;
            float v;
            if constexpr (FULLPLANE) {
                const bool in = k < P.K;
                v = xa[in ? (uint32_t)ci * (uint32_t)P.x_sC + (uint32_t)kk * (uint32_t)P.x_sK : 0u];
                kk += 4;
                while (kk >= P.KK) {
                    kk -= P.KK;
                    ++ci;
                }
            } else {
                v = xa[(int64_t)(k < P.K ? k : P.K - 1) * P.x_sC];
            }
            a[buf][t] = k < P.K ? v : 0.f;
            b[buf][t] = wb[(int64_t)(k < P.Kpad ? k : 0) * P.Mpad];
            if (k >= P.Kpad) b[buf][t] = 0.f;
        }
    };
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    load(0, 0);
    if constexpr (NCH > 0) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (c + 1 < NCH) load((c + 1) * RC, (c + 1) & 1);
#pragma unroll
            for (int t = 0; t < RC / 4; ++t)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c & 1][t], b[c & 1][t], acc, 0, 0, 0);
        }
    } else for (int kc = 0; kc < P.Kpad; kc += 2 * RC) {
        if (kc + RC < P.Kpad) load(kc + RC, 1);
#pragma unroll
        for (int t = 0; t < RC / 4; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0][t], b[0][t], acc, 0, 0, 0);
        if (kc + RC >= P.Kpad) break;
        if (kc + 2 * RC < P.Kpad) load(kc + 2 * RC, 0);
#pragma unroll
        for (int t = 0; t < RC / 4; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1][t], b[1][t], acc, 0, 0, 0);
    }

    // acc[i] = C^T[n0 + 4 * kq + i][m0 + r]
    const int m = m0 + r;
    if (m >= P.M) return;
    const float bias = P.bias[m];
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = acc[i] + bias;
    auto chan = [&](int) { return m; };
    apply_act_n<4>(P.pre, v, chan);
    apply_act_n<4>(P.post, v, chan);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int n = n0 + 4 * kq + i;
        if (n < nimg) P.out[(uint32_t)n * (uint32_t)P.o_sN + (uint32_t)m * (uint32_t)P.o_sC] = v[i];
    }
}

template <bool FULLPLANE, int NCH>
__global__ __launch_bounds__(256) void gemm_rows_kernel(const GemmParams P, int mtiles) {
    gemm_rows_body<FULLPLANE, NCH>(P, mtiles, blockIdx.x, blockIdx.y);
}

template <bool FULLPLANE, int NCH>
__global__ __launch_bounds__(256) void gemm_rows_group_kernel(const LaunchGroup<GemmParams> G) {
    const GroupSlot t = group_slot(G);
    gemm_rows_body<FULLPLANE, NCH>(G.p[t.g], G.a0[t.g], t.bx, t.by);
}

// ---------------------------------------------------------------- launch choice
// The form, template variant, grid and scalar arguments launch_gemm picks for a GEMM; grouped
// launches use it to check that sibling steps would run the same kernel instance.
enum GemmForm { GF_GENERIC, GF_TILED, GF_ROWS, GF_SMALLK };
struct GemmChoice {
    GemmForm form;
    int v0 = 0, v1 = 0, v2 = 0;  // generic: MT, FULLPLANE; tiled: MT, NT, RES; rows: NCH; smallk: NCH
    int gx = 1, gy = 1;
    int a0 = 0, a1 = 0, a2 = 0;  // tiled: mblocks, nct, vec; rows: mtiles
    bool same_instance(const GemmChoice &o) const { return form == o.form && v0 == o.v0 && v1 == o.v1 && v2 == o.v2; }
};

static GemmChoice choose_gemm(const GemmParams &p) {
    GemmChoice c{};
    const int mtiles = p.Mpad / 32;
    // LDS-tiled path: X must be a row-major [K][ncols] matrix with 16-B aligned rows.  A row whose
    // length is not a multiple of 4 (N x 7^2 or N x 3^2 columns for odd N) is read in whole float4s
    // up to round_up(ncols, 4): the arena pads every channel plane to whole groups of 4 images
    // (Binding::Ns), so the slack is inside the row; its columns are computed and never stored.
    // (K <= 128 single-tile 1x1s over such rows keep the small-K form: the FaceMesh 3^2 tail.)
    const int nch_k = (p.Kpad + KC - 1) / KC;
    const bool tail_ok = (p.ncols % 4) == 0 ||
                         (p.x_sC >= (int64_t)(p.ncols + 3) / 4 * 4 && !(mtiles == 1 && nch_k <= 4 && form_on(FORM_ROWS)));
    const bool rowmajor = p.KK == 1 && p.x_sN == p.P && (p.x_sC % 4) == 0 && tail_ok &&
                          ((uintptr_t)p.x % 16) == 0 && (p.Mpad % 4) == 0 && ((uintptr_t)p.wt % 16) == 0;
    if (rowmajor) {
        // K <= 64 (the expand convs): one or two K-chunks, so operand reuse buys nothing and
        // the launch is bound by its output stores -- small tiles, high occupancy
        const bool skinny = p.K <= 64;
        int mt = std::min(skinny ? 1 : 4, mtiles);
        const int nt = !skinny && p.ncols >= 256 * 256 ? 2 : 1;  // wide tiles once there are >= 256 of them
        const int bn = 4 * nt * 32;
        // keep >= ~2 workgroups per CU: trade M-tile reuse for parallelism on small problems
        while (mt > 1 && (int64_t)((p.ncols + bn - 1) / bn) * ((mtiles + mt - 1) / mt) < 512) --mt;
        mt = std::max(mt, 1);
        const int nct = (p.ncols + bn - 1) / bn;
        const int mblocks = (p.Mpad + mt * 32 - 1) / (mt * 32);
        // 16-B output segments: whole 4-column groups inside one image, aligned rows
        const int vec = form_on(FORM_VSTORE) && p.o_sP == 1 && p.P % 4 == 0 && p.o_sN % 4 == 0 &&
                        p.o_sC % 4 == 0 && ((uintptr_t)p.out % 16) == 0;
        c.form = GF_TILED;
        c.v0 = mt, c.v1 = nt, c.v2 = p.res_mode != 0;
        c.gx = (nct * mblocks + 7) / 8 * 8;
        c.a0 = mblocks, c.a1 = nct, c.a2 = vec;
        return c;
    }
    if (p.P == 1 && p.res_mode == 0 && p.KK > 1 && form_on(FORM_ROWS)) {  // a head over whole planes (KK >= 2)
        c.form = GF_ROWS;
        c.v0 = (p.Kpad + RC - 1) / RC == 9 ? 9 : 0;
        const int mt16 = (p.Mpad + 15) / 16;  // 16-row tiles
        c.gx = (p.ncols + 15) / 16, c.gy = (mt16 + 3) / 4;
        c.a0 = mt16;
        return c;
    }
    const int bx = (p.ncols + 127) / 128;
    const int nch = (p.Kpad + KC - 1) / KC;
    if (p.KK == 1 && mtiles == 1 && nch <= 4 && form_on(FORM_ROWS)) {
        c.form = GF_SMALLK;
        c.v0 = std::max(nch, 1);
        c.gx = bx;
        return c;
    }
    // Largest M tile (operand reuse) that still leaves >= 2 workgroups per CU of parallelism.
    int mt = 4;
    while (mt > 1 && (int64_t)bx * ((mtiles + mt - 1) / mt) < 512) --mt;
    if (mt > mtiles) mt = mtiles;
    mt = std::max(mt, 1);
    c.form = GF_GENERIC;
    c.v0 = mt, c.v1 = p.KK > 1;
    c.gx = bx, c.gy = (mtiles + mt - 1) / mt;
    return c;
}

// names as rocprofv3 prints the instance (bench.py joins the two by symbol)
template <int MT, int NT, bool RES>
static const char *launch_tiled(const GemmParams &p, const GemmChoice &c, hipStream_t s) {
    hipLaunchKernelGGL((gemm_tiled_kernel<MT, NT, RES>), dim3(c.gx), dim3(256), 0, s, p, c.a0, c.a1, c.a2);
    return kernel_name("gemm_tiled_kernel<%d,%d,%s>", MT, NT, RES ? "true" : "false");
}

template <int NT, bool RES>
static const char *launch_tiled_mt(const GemmParams &p, const GemmChoice &c, hipStream_t s) {
    switch (c.v0) {
    case 4: return launch_tiled<4, NT, RES>(p, c, s);
    case 3: return launch_tiled<3, NT, RES>(p, c, s);
    case 2: return launch_tiled<2, NT, RES>(p, c, s);
    default: return launch_tiled<1, NT, RES>(p, c, s);
    }
}

template <int MT>
static const char *launch_mt(const GemmParams &p, const GemmChoice &c, hipStream_t s) {
    const dim3 grid(c.gx, c.gy);
    if (c.v1) hipLaunchKernelGGL((gemm_kernel<MT, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((gemm_kernel<MT, false>), grid, dim3(256), 0, s, p);
    return kernel_name("gemm_kernel<%d,%s>", MT, c.v1 ? "true" : "false");
}

const char *launch_gemm(const GemmParams &p, hipStream_t s) {
    const GemmChoice c = choose_gemm(p);
    switch (c.form) {
    case GF_TILED:
        if (c.v1 == 2) return c.v2 ? launch_tiled_mt<2, true>(p, c, s) : launch_tiled_mt<2, false>(p, c, s);
        return c.v2 ? launch_tiled_mt<1, true>(p, c, s) : launch_tiled_mt<1, false>(p, c, s);
    case GF_ROWS:
        if (c.v0 == 9) {
            hipLaunchKernelGGL((gemm_rows_kernel<true, 9>), dim3(c.gx, c.gy), dim3(256), 0, s, p, c.a0);
            return "gemm_rows_kernel<true, 9>";
        }
        hipLaunchKernelGGL((gemm_rows_kernel<true, 0>), dim3(c.gx, c.gy), dim3(256), 0, s, p, c.a0);
        return "gemm_rows_kernel<true, 0>";
    case GF_SMALLK:
        switch (c.v0) {
        case 1: hipLaunchKernelGGL((gemm_smallk_kernel<1>), dim3(c.gx), dim3(256), 0, s, p); return "gemm_smallk_kernel<1>";
        case 2: hipLaunchKernelGGL((gemm_smallk_kernel<2>), dim3(c.gx), dim3(256), 0, s, p); return "gemm_smallk_kernel<2>";
        case 3: hipLaunchKernelGGL((gemm_smallk_kernel<3>), dim3(c.gx), dim3(256), 0, s, p); return "gemm_smallk_kernel<3>";
        default: hipLaunchKernelGGL((gemm_smallk_kernel<4>), dim3(c.gx), dim3(256), 0, s, p); return "gemm_smallk_kernel<4>";
        }
    default:
        switch (c.v0) {
        case 4: return launch_mt<4>(p, c, s);
        case 3: return launch_mt<3>(p, c, s);
        case 2: return launch_mt<2>(p, c, s);
        default: return launch_mt<1>(p, c, s);
        }
    }
}

// Sibling GEMMs in one launch when every part would run the same kernel instance and that
// instance has a grouped form (the ones the plans' sibling steps use: the hand heads' generic /
// tiled 1-tile GEMMs, the FaceMesh heads' row form and small-K 1x1s); nullptr otherwise.
const char *launch_gemm_group(const GemmParams *p, int n, hipStream_t s) {
    if (n < 2 || n > ZR_GROUP_MAX) return nullptr;
    GemmChoice c[ZR_GROUP_MAX];
    for (int i = 0; i < n; ++i) {
        c[i] = choose_gemm(p[i]);
        if (!c[i].same_instance(c[0])) return nullptr;
    }
    const GemmChoice &c0 = c[0];
    const bool ok = (c0.form == GF_GENERIC && c0.v0 == 1) || (c0.form == GF_TILED && c0.v0 == 1 && c0.v1 == 1 && !c0.v2) ||
                    c0.form == GF_ROWS || c0.form == GF_SMALLK;
    if (!ok) return nullptr;
    LaunchGroup<GemmParams> G{};
    G.n = n;
    int total = 0;
    for (int i = 0; i < n; ++i) {
        G.p[i] = p[i];
        G.a0[i] = c[i].a0, G.a1[i] = c[i].a1, G.a2[i] = c[i].a2;
        G.gx[i] = c[i].gx;
        G.start[i] = total;
        total += c[i].gx * c[i].gy;
    }
    for (int i = n; i <= ZR_GROUP_MAX; ++i) G.start[i] = total;
    const dim3 grid(total), block(256);
    switch (c0.form) {
    case GF_TILED:
        hipLaunchKernelGGL((gemm_tiled_group_kernel<1, 1, false>), grid, block, 0, s, G);
        return "gemm_tiled_group_kernel<1,1,false>";
    case GF_ROWS:
        if (c0.v0 == 9) {
            hipLaunchKernelGGL((gemm_rows_group_kernel<true, 9>), grid, block, 0, s, G);
            return "gemm_rows_group_kernel<true, 9>";
        }
        hipLaunchKernelGGL((gemm_rows_group_kernel<true, 0>), grid, block, 0, s, G);
        return "gemm_rows_group_kernel<true, 0>";
    case GF_SMALLK:
        switch (c0.v0) {
        case 1: hipLaunchKernelGGL((gemm_smallk_group_kernel<1>), grid, block, 0, s, G); return "gemm_smallk_group_kernel<1>";
        case 2: hipLaunchKernelGGL((gemm_smallk_group_kernel<2>), grid, block, 0, s, G); return "gemm_smallk_group_kernel<2>";
        case 3: hipLaunchKernelGGL((gemm_smallk_group_kernel<3>), grid, block, 0, s, G); return "gemm_smallk_group_kernel<3>";
        default: hipLaunchKernelGGL((gemm_smallk_group_kernel<4>), grid, block, 0, s, G); return "gemm_smallk_group_kernel<4>";
        }
    default:
        if (c0.v1) {
            hipLaunchKernelGGL((gemm_group_kernel<1, true>), grid, block, 0, s, G);
            return "gemm_group_kernel<1,true>";
        }
        hipLaunchKernelGGL((gemm_group_kernel<1, false>), grid, block, 0, s, G);
        return "gemm_group_kernel<1,false>";
    }
}

}  // namespace zr
