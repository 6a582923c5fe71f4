// spatial.hip -- depthwise convolution (K3) and dense direct convolution (K2 stems) for gfx950.
//
// Both stage an input tile (with the ONNX zero padding materialised) in LDS with coalesced
// row loads, then every thread produces its outputs from LDS.  The channel's KxK taps are
// wave-uniform, so they come from scalar loads.  Reference: the depthwise (group=C) and
// group=1 KxK Conv nodes of the four graphs, executed by ORT/tract
// at crates/zaru/src/nn/mod.rs:483-533.
#include "../runtime/zr_kernels.h"
#include "act.h"

namespace zr {

// ------------------------------------------------------------------ depthwise
// grid.x = planes (c*N + n), grid.y = row tiles.  Tile = TH output rows x all columns.
template <int K, int S>
__global__ __launch_bounds__(256) void dw_kernel(const DwParams P, int TH) {
    extern __shared__ __attribute__((aligned(16))) float tile[];
    const int plane = blockIdx.x;
    const int c = plane / P.N, n = plane - c * P.N;
    const int oy0 = blockIdx.y * TH;
    const int th = min(TH, P.OH - oy0);
    const int W = P.in.W, H = P.in.H;
    const int rin = (th - 1) * S + K;
    const int win = (P.OW - 1) * S + K;
    const int iy0 = oy0 * S - P.pad_t, ix0 = -P.pad_l;
    const float *src = P.in.p + (int64_t)n * P.in.sN + (int64_t)c * P.in.sC;

    for (int i = threadIdx.x; i < rin * win; i += blockDim.x) {
        const int r = i / win, cc = i - r * win;
        const int iy = iy0 + r, ix = ix0 + cc;
        tile[i] = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? src[(int64_t)iy * W + ix] : 0.f;
    }
    float w[K * K];
#pragma unroll
    for (int t = 0; t < K * K; ++t) w[t] = P.w[c * K * K + t];
    const float b = P.bias[c];
    __syncthreads();

    float *dst = P.out + (int64_t)n * P.o_sN + (int64_t)c * P.o_sC + (int64_t)oy0 * P.OW;
    for (int i = threadIdx.x; i < th * P.OW; i += blockDim.x) {
        const int oy = i / P.OW, ox = i - oy * P.OW;
        const float *t0 = tile + oy * S * win + ox * S;
        float acc = b;
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
            for (int kx = 0; kx < K; ++kx) acc += w[ky * K + kx] * t0[ky * win + kx];
        dst[i] = apply_act(P.act, acc, c);
    }
}

template <int K, int S>
static const char *dw_launch(const DwParams &p, hipStream_t s) {
    const int planes = p.in.C * p.N;
    // ~1024 outputs per 256-thread workgroup; tiny planes use a single wave
    int th = p.OH;
    if ((int64_t)p.OH * p.OW > 1024) th = max(1, 1024 / p.OW);
    const int outs = th * p.OW;
    const int threads = outs >= 256 ? 256 : (outs > 128 ? 256 : (outs > 64 ? 128 : 64));
    const int win = (p.OW - 1) * S + K, rin = (th - 1) * S + K;
    const size_t lds = sizeof(float) * (size_t)win * rin;
    dim3 grid(planes, (p.OH + th - 1) / th);
    hipLaunchKernelGGL((dw_kernel<K, S>), grid, dim3(threads), lds, s, p, th);
    return K == 3 ? (S == 1 ? "dw_kernel<3,1>" : "dw_kernel<3,2>") : (S == 1 ? "dw_kernel<5,1>" : "dw_kernel<5,2>");
}

const char *launch_dw(const DwParams &p, hipStream_t s) {
    if (p.k == 3 && p.stride == 1) return dw_launch<3, 1>(p, s);
    if (p.k == 3 && p.stride == 2) return dw_launch<3, 2>(p, s);
    if (p.k == 5 && p.stride == 1) return dw_launch<5, 1>(p, s);
    return dw_launch<5, 2>(p, s);
}

// ------------------------------------------------------------------ dense direct conv
// grid.x = spatial tiles (TH x TW outputs), grid.y = image, grid.z = groups of 8 output
// channels.  Input patch for a chunk of CC input channels lives in LDS; each thread owns
// one output position and 8 accumulators.
constexpr int DTH = 8, DTW = 32, DCO = 8;

__global__ __launch_bounds__(256) void direct_kernel(const DirectParams P, int CC) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tiles_x = (P.OW + DTW - 1) / DTW;
    const int ty0 = (blockIdx.x / tiles_x) * DTH, tx0 = (blockIdx.x % tiles_x) * DTW;
    const int n = blockIdx.y, co0 = blockIdx.z * DCO;
    const int Cin = P.in.C, H = P.in.H, W = P.in.W;
    const int rin = (DTH - 1) * P.stride + P.kh, win = (DTW - 1) * P.stride + P.kw;
    const int kk = P.kh * P.kw;
    float *patch = smem;                      // [CC][rin][win]
    float *ws = smem + CC * rin * win;        // [DCO][CC][kh*kw]
    const int oy = ty0 + threadIdx.x / DTW, ox = tx0 + threadIdx.x % DTW;
    const int iy0 = ty0 * P.stride - P.pad_t, ix0 = tx0 * P.stride - P.pad_l;

    float acc[DCO];
#pragma unroll
    for (int o = 0; o < DCO; ++o) acc[o] = 0.f;

    for (int cb = 0; cb < Cin; cb += CC) {
        const int cc = min(CC, Cin - cb);
        __syncthreads();
        for (int i = threadIdx.x; i < cc * rin * win; i += 256) {
            const int ci = i / (rin * win), rem = i - ci * rin * win;
            const int r = rem / win, x = rem - r * win;
            const int iy = iy0 + r, ix = ix0 + x;
            patch[i] = (iy >= 0 && iy < H && ix >= 0 && ix < W)
                           ? P.in.p[(int64_t)n * P.in.sN + (int64_t)(cb + ci) * P.in.sC +
                                    (int64_t)iy * W + ix]
                           : 0.f;
        }
        for (int i = threadIdx.x; i < DCO * cc * kk; i += 256) {
            const int o = i / (cc * kk), rem = i - o * cc * kk;
            const int ci = rem / kk, t = rem - ci * kk;
            const int co = co0 + o;
            ws[i] = co < P.Cout ? P.w[((int64_t)co * Cin + cb + ci) * kk + t] : 0.f;
        }
        __syncthreads();
        const int ly = (threadIdx.x / DTW) * P.stride, lx = (threadIdx.x % DTW) * P.stride;
        for (int ci = 0; ci < cc; ++ci)
            for (int ky = 0; ky < P.kh; ++ky)
                for (int kx = 0; kx < P.kw; ++kx) {
                    const float v = patch[(ci * rin + ly + ky) * win + lx + kx];
                    const int t = (ci * P.kh + ky) * P.kw + kx;
#pragma unroll
                    for (int o = 0; o < DCO; ++o) acc[o] += ws[o * cc * kk + t] * v;
                }
    }
    if (oy >= P.OH || ox >= P.OW) return;
    float *dst = P.out + (int64_t)n * P.o_sN + (int64_t)oy * P.OW + ox;
#pragma unroll
    for (int o = 0; o < DCO; ++o) {
        const int co = co0 + o;
        if (co < P.Cout) dst[(int64_t)co * P.o_sC] = apply_act(P.act, acc[o] + P.bias[co], co);
    }
}

const char *launch_direct(const DirectParams &p, hipStream_t s) {
    const int rin = (DTH - 1) * p.stride + p.kh, win = (DTW - 1) * p.stride + p.kw;
    const int kk = p.kh * p.kw;
    int cc = p.in.C;
    while (cc > 1 && sizeof(float) * ((size_t)cc * rin * win + (size_t)DCO * cc * kk) > 48 * 1024)
        cc = (cc + 1) / 2;
    const size_t lds = sizeof(float) * ((size_t)cc * rin * win + (size_t)DCO * cc * kk);
    const int tiles = ((p.OH + DTH - 1) / DTH) * ((p.OW + DTW - 1) / DTW);
    dim3 grid(tiles, p.N, (p.Cout + DCO - 1) / DCO);
    hipLaunchKernelGGL(direct_kernel, grid, dim3(256), lds, s, p, cc);
    return "direct_kernel";
}

}  // namespace zr
