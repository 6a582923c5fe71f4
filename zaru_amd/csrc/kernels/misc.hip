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
        static const char *const names[FORM_COUNT] = {"dma", "v4", "valu", "valu_db", "rows", "vres", "vstore", "ws"};
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
