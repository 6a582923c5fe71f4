// misc.hip -- the graph's remaining memory-bound operators (only launched when they cannot be
// folded into a GEMM epilogue): standalone activation / Add / MaxPool 2x2 / channel Pad,
// bilinear Resize (half_pixel, palm FPN), GlobalAveragePool (hand head), plus the detector
// candidate compaction that keeps the bit-exact decode on the host cheap.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <set>
#include <string>
#include "../runtime/zr_kernels.h"
#include "act.h"

namespace zr {

const char *kernel_name(const char *fmt, ...) {
    char buf[128];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    static std::mutex mu;
    static std::set<std::string> names;
    std::lock_guard<std::mutex> g(mu);
    return names.insert(buf).first->c_str();
}

bool form_on(Form f) {
    static const unsigned mask = [] {
        static const char *const names[FORM_COUNT] = {"dma", "v4", "valu", "valu_db", "rows", "vres", "vstore", "ws", "groups", "dwgap", "rt", "ir", "irl", "irl2", "bneck", "pin"};
        unsigned m = (1u << FORM_COUNT) - 1;
        const char *e = std::getenv("ZARU_HIP_FORMS");
        for (std::string s = e ? e : ""; !s.empty();) {
            const size_t comma = s.find(',');
            const std::string tok = s.substr(0, comma);
            s = comma == std::string::npos ? "" : s.substr(comma + 1);
            if (tok.size() < 2 || (tok[0] != '+' && tok[0] != '-')) continue;
            for (int i = 0; i < FORM_COUNT; i++)
                if (tok.compare(1, std::string::npos, names[i]) == 0)
                    m = tok[0] == '+' ? m | (1u << i) : m & ~(1u << i);
        }
        return m;
    }();
    return (mask >> f) & 1u;
}

__device__ __forceinline__ const float *plane_ptr(const Plane &p, int n, int c) {
    return p.p + (int64_t)n * p.sN + (int64_t)c * p.sC;
}

// ------------------------------------------------------------------ elementwise
// grid.x over planes (c*N + n), grid.y over positions of one plane
__global__ __launch_bounds__(256) void elt_kernel(const EltParams P) {
    const int plane = blockIdx.x;
    const int c = plane / P.N, n = plane - c * P.N;
    const int HW = P.H * P.W;
    float *dst = P.out + (int64_t)n * P.o_sN + (int64_t)c * P.o_sC;
    for (int q = blockIdx.y * blockDim.x + threadIdx.x; q < HW; q += gridDim.y * blockDim.x) {
        float v;
        if (P.op == 0) {
            v = plane_ptr(P.a, n, c)[q];
        } else if (P.op == 1) {
            v = plane_ptr(P.a, n, c)[q] + plane_ptr(P.b, n, c)[q];
        } else if (P.op == 2) {
            const int y = q / P.W, x = q - y * P.W;
            const float *s = plane_ptr(P.a, n, c) + (int64_t)(2 * y) * P.a.W + 2 * x;
            v = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[P.a.W], s[P.a.W + 1]));
        } else {
            v = c < P.a.C ? plane_ptr(P.a, n, c)[q] : 0.f;
        }
        dst[q] = apply_act(P.act, v, c);
    }
}

const char *launch_elt(const EltParams &p, hipStream_t s) {
    const int HW = p.H * p.W;
    dim3 grid(p.C * p.N, std::min((HW + 255) / 256, 64));
    hipLaunchKernelGGL(elt_kernel, grid, dim3(256), 0, s, p);
    return "elt_kernel";
}

// ------------------------------------------------------------------ resize (bilinear)
// ONNX Resize mode=linear, coordinate_transformation_mode=half_pixel: source coordinate
// (o + 0.5) * in/out - 0.5, neighbours clamped to the edge.
__global__ __launch_bounds__(256) void resize_kernel(const ResizeParams P) {
    const int plane = blockIdx.x;
    const int c = plane / P.N, n = plane - c * P.N;
    if (P.nact && n >= *P.nact) return;
    const float *src = plane_ptr(P.in, n, c);
    float *dst = P.out + (int64_t)n * P.o_sN + (int64_t)c * P.o_sC;
    const int H = P.in.H, W = P.in.W;
    for (int q = blockIdx.y * blockDim.x + threadIdx.x; q < P.OH * P.OW;
         q += gridDim.y * blockDim.x) {
        const int oy = q / P.OW, ox = q - oy * P.OW;
        const float fy = (oy + 0.5f) * P.scale_y - 0.5f, fx = (ox + 0.5f) * P.scale_x - 0.5f;
        const float y0f = floorf(fy), x0f = floorf(fx);
        const float ry = fy - y0f, rx = fx - x0f;
        int y0 = (int)y0f, x0 = (int)x0f;
        const int y1 = min(max(y0 + 1, 0), H - 1), x1 = min(max(x0 + 1, 0), W - 1);
        y0 = min(max(y0, 0), H - 1);
        x0 = min(max(x0, 0), W - 1);
        const float top = (1.f - rx) * src[y0 * W + x0] + rx * src[y0 * W + x1];
        const float bot = (1.f - rx) * src[y1 * W + x0] + rx * src[y1 * W + x1];
        dst[q] = (1.f - ry) * top + ry * bot;
    }
}

const char *launch_resize(const ResizeParams &p, hipStream_t s) {
    const int n = p.OH * p.OW;
    dim3 grid(p.in.C * p.N, std::min((n + 255) / 256, 64));
    hipLaunchKernelGGL(resize_kernel, grid, dim3(256), 0, s, p);
    return "resize_kernel";
}

// ------------------------------------------------------------------ global average pool
// one wave per (c, n) plane, 4 planes per workgroup, wave64 shuffle reduction
__global__ __launch_bounds__(256) void gap_kernel(const GapParams P, int planes) {
    const int plane = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (plane >= planes) return;
    const int c = plane / P.N, n = plane - c * P.N;
    const float *src = plane_ptr(P.in, n, c);
    const int HW = P.in.H * P.in.W;
    float s = 0.f;
    for (int q = lane; q < HW; q += 64) s += src[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) P.out[(int64_t)n * P.o_sN + (int64_t)c * P.o_sC] = s / (float)HW;
}

const char *launch_gap(const GapParams &p, hipStream_t s) {
    const int planes = p.in.C * p.N;
    hipLaunchKernelGGL(gap_kernel, dim3((planes + 3) / 4), dim3(256), 0, s, p, planes);
    return "gap_kernel";
}

// ------------------------------------------------------------------ depthwise -> global pool
// A depthwise KxK conv + activation whose only consumer is a global average pool (the hand
// landmark network's last block: 672 x 7^2 -> 672), in one launch: the depthwise plane never
// reaches HBM.  A workgroup stages DG_NB contiguous planes of one channel (coalesced, CNHW) in
// LDS; each wave reduces whole planes: lane q computes the depthwise outputs q, q + 64, ... with
// dw_kernel's arithmetic (bias, then + w * x per tap in (ky, kx) order, zero taps outside the
// plane) and accumulates them as gap_kernel does (s = 0 + v + ...), then gap_kernel's butterfly
// and division.  Bitwise equal to dw_kernel -> gap_kernel.
constexpr int DG_NB = 64;  // planes (images) per workgroup: one load latency for 64 planes

template <int K>
__global__ __launch_bounds__(256) void dwgap_kernel(const DwParams P, int S, int vec) {
    extern __shared__ __attribute__((aligned(16))) float pl[];  // DG_NB planes of H * W
    const int c = blockIdx.y, n0 = blockIdx.x * DG_NB;
    const int nb = min(DG_NB, P.N - n0);
    const int H = P.in.H, W = P.in.W, HW = H * W, OHW = P.OH * P.OW;
    const float *src = P.in.p + (int64_t)c * P.in.sC + (int64_t)n0 * P.in.sN;
    if (vec) {  // the planes are contiguous (sN = H * W) and the run starts 16-B aligned
        const int n4 = (nb * HW) >> 2;
        for (int i = threadIdx.x; i < n4; i += 256)
            reinterpret_cast<float4 *>(pl)[i] = reinterpret_cast<const float4 *>(src)[i];
        for (int i = 4 * n4 + threadIdx.x; i < nb * HW; i += 256) pl[i] = src[i];
    } else {
        for (int i = threadIdx.x; i < nb * HW; i += 256) {
            const int n = i / HW, q = i - n * HW;
            pl[i] = src[(int64_t)n * P.in.sN + q];
        }
    }
    float w[K * K];
#pragma unroll
    for (int t = 0; t < K * K; ++t) w[t] = P.w[c * K * K + t];
    const float b = P.bias[c];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int n = wave; n < nb; n += 4) {
        const float *x = pl + n * HW;
        float s = 0.f;
        for (int q = lane; q < OHW; q += 64) {
            const int oy = q / P.OW, ox = q - oy * P.OW;
            const int iy0 = oy * S - P.pad_t, ix0 = ox * S - P.pad_l;
            float acc = b;
#pragma unroll
            for (int ky = 0; ky < K; ++ky)
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const int iy = iy0 + ky, ix = ix0 + kx;
                    const bool in = iy >= 0 && iy < H && ix >= 0 && ix < W;
                    const float v = x[in ? iy * W + ix : 0];
                    acc += w[ky * K + kx] * (in ? v : 0.f);
                }
            s += apply_act(P.act, acc, c);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if (lane == 0) P.out[(int64_t)(n0 + n) * P.o_sN + (int64_t)c * P.o_sC] = s / (float)OHW;
    }
}

// One plane per lane for small planes (the hand tail: 3x3 on 7^2): the plane sits in registers,
// the KxK taps are static indices, and gap_kernel's butterfly (a tree of exact, commutative
// adds: lane 0 ends with ((s_0 + s_32) + (s_16 + s_48)) + ...) is replayed in-lane over the 64
// values it would have seen (s_q = 0 + v_q, zero past the plane).  No shuffles, no divergence:
// ~1000 VALU instructions per 64 planes instead of ~60 per plane.
template <int K, int H, int W, int S, int OH, int OW, int PT, int PL>
__global__ __launch_bounds__(256) void dwgap_lane_kernel(const DwParams P, int vec) {
    constexpr int HW = H * W, OHW = OH * OW;
    static_assert(OHW <= 64, "gap_kernel's single-pass butterfly");
    extern __shared__ __attribute__((aligned(16))) float pl[];  // 256 planes of H * W
    const int c = blockIdx.y, n0 = blockIdx.x * 256;
    const int nb = min(256, P.N - n0);
    const float *src = P.in.p + (int64_t)c * P.in.sC + (int64_t)n0 * P.in.sN;
    if (vec) {
        const int n4 = (nb * HW) >> 2;
        for (int i = threadIdx.x; i < n4; i += 256)
            reinterpret_cast<float4 *>(pl)[i] = reinterpret_cast<const float4 *>(src)[i];
        for (int i = 4 * n4 + threadIdx.x; i < nb * HW; i += 256) pl[i] = src[i];
    } else {
        for (int i = threadIdx.x; i < nb * HW; i += 256) {
            const int n = i / HW, q = i - n * HW;
            pl[i] = src[(int64_t)n * P.in.sN + q];
        }
    }
    __syncthreads();
    if ((int)threadIdx.x >= nb) return;
    float x[HW], w[K * K];
#pragma unroll
    for (int i = 0; i < HW; ++i) x[i] = pl[threadIdx.x * HW + i];
#pragma unroll
    for (int t = 0; t < K * K; ++t) w[t] = P.w[c * K * K + t];
    const float b = P.bias[c];
    float a[32];
#pragma unroll
    for (int q = 0; q < 64; ++q) {
        if (q >= OHW) break;
        const int oy = q / OW, ox = q % OW;
        float acc = b;
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const int iy = oy * S - PT + ky, ix = ox * S - PL + kx;
                const bool in = iy >= 0 && iy < H && ix >= 0 && ix < W;
                acc += w[ky * K + kx] * (in ? x[in ? iy * W + ix : 0] : 0.f);
            }
        const float sq = 0.f + apply_act(P.act, acc, c);
        if (q < 32) a[q] = sq;
        else a[q - 32] = a[q - 32] + sq;
    }
#pragma unroll
    for (int q = OHW; q < 32; ++q) a[q] = 0.f;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1)
#pragma unroll
        for (int j = 0; j < o; ++j) a[j] = a[j] + a[j + o];
    P.out[(int64_t)(n0 + threadIdx.x) * P.o_sN + (int64_t)c * P.o_sC] = a[0] / (float)OHW;
}

const char *launch_dwgap(const DwParams &p, hipStream_t s) {
    {
        const int hw = p.in.H * p.in.W;
        const int vec = p.in.sN == hw && p.in.sC % 4 == 0 && (256 * hw) % 4 == 0 && (uintptr_t)p.in.p % 16 == 0;
        if (p.k == 3 && p.stride == 1 && p.in.H == 7 && p.in.W == 7 && p.OH == 7 && p.OW == 7 && p.pad_t == 1 && p.pad_l == 1) {
            static const bool attr = hipFuncSetAttribute((const void *)dwgap_lane_kernel<3, 7, 7, 1, 7, 7, 1, 1>,
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024) == hipSuccess;
            (void)attr;
            const dim3 grid((p.N + 255) / 256, p.in.C);
            hipLaunchKernelGGL((dwgap_lane_kernel<3, 7, 7, 1, 7, 7, 1, 1>), grid, dim3(256), sizeof(float) * 256 * hw, s, p, vec);
            return "dwgap_lane_kernel<3,7,7,1,7,7,1,1>";
        }
    }
    const dim3 grid((p.N + DG_NB - 1) / DG_NB, p.in.C);
    const size_t lds = sizeof(float) * DG_NB * p.in.H * p.in.W;
    const int hw = p.in.H * p.in.W;
    const int vec = p.in.sN == hw && p.in.sC % 4 == 0 && (DG_NB * hw) % 4 == 0 && (uintptr_t)p.in.p % 16 == 0;
    if (p.k == 3) {
        hipLaunchKernelGGL((dwgap_kernel<3>), grid, dim3(256), lds, s, p, p.stride, vec);
        return "dwgap_kernel<3>";
    }
    hipLaunchKernelGGL((dwgap_kernel<5>), grid, dim3(256), lds, s, p, p.stride, vec);
    return "dwgap_kernel<5>";
}

// ------------------------------------------------------------------ detection candidates
// One workgroup per image.  Order of the compacted records is arbitrary (atomic slot);
// the host restores anchor order before the exact decode (face/detection.rs:109-121).
__global__ __launch_bounds__(256) void cand_kernel(const CandParams P) {
    const int n = blockIdx.x;
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const float *lg = P.logits + (int64_t)n * P.A;
    const float *bx = P.boxes + (int64_t)n * P.A * P.D;
    float *rec = P.rec + (int64_t)n * P.cap * (2 + P.D);
    for (int a = threadIdx.x; a < P.A; a += blockDim.x) {
        const float l = lg[a];
        if (l >= P.logit_min) {
            const int slot = atomicAdd(&cnt, 1);
            if (slot < P.cap) {
                float *r = rec + (int64_t)slot * (2 + P.D);
                r[0] = __int_as_float(a);
                r[1] = l;
                for (int d = 0; d < P.D; ++d) r[2 + d] = bx[(int64_t)a * P.D + d];
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) P.count[n] = cnt;
}

const char *launch_candidates(const CandParams &p, hipStream_t s) {
    hipLaunchKernelGGL(cand_kernel, dim3(p.N), dim3(256), 0, s, p);
    return "cand_kernel";
}

}  // namespace zr
