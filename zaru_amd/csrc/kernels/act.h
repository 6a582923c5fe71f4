// act.h -- activation epilogues of the ONNX graphs (Relu, Clip(0,6), PRelu, Sigmoid).
#pragma once
#include "../runtime/zr_kernels.h"

namespace zr {

// Read-only parameters (weights, biases, slopes) through the constant address space: such loads
// are invariant for the kernel, so uniform ones become scalar (s_load) loads even in kernels
// that write LDS by DMA, and no vector-memory wait (which would also drain the DMA) guards them.
__device__ __forceinline__ float ldc(const float *p, int i) {
    return ((const __attribute__((address_space(4))) float *)p)[i];
}

__device__ __forceinline__ float apply_act(const Act &a, float v, int c) {
    switch (a.kind) {
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_CLIP: return fminf(fmaxf(v, a.lo), a.hi);
    case ACT_PRELU: return v < 0.f ? v * ldc(a.slope, c) : v;
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
    }
}

// The same over N values, element r on channel ch(r).  The kind is uniform, so the switch
// sits outside the loop and every branch is straight-line code the scheduler can interleave
// (a switch per element would fence every load behind it).
template <int N, typename ChanFn>
__device__ __forceinline__ void apply_act_n(const Act &a, float *v, ChanFn ch) {
    switch (a.kind) {
    case ACT_RELU:
#pragma unroll
        for (int r = 0; r < N; ++r) v[r] = fmaxf(v[r], 0.f);
        break;
    case ACT_CLIP:
#pragma unroll
        for (int r = 0; r < N; ++r) v[r] = fminf(fmaxf(v[r], a.lo), a.hi);
        break;
    case ACT_PRELU: {
        float s[N];
#pragma unroll
        for (int r = 0; r < N; ++r) s[r] = ldc(a.slope, ch(r));
#pragma unroll
        for (int r = 0; r < N; ++r) v[r] = v[r] < 0.f ? v[r] * s[r] : v[r];
        break;
    }
    case ACT_SIGMOID:
#pragma unroll
        for (int r = 0; r < N; ++r) v[r] = 1.f / (1.f + expf(-v[r]));
        break;
    default: break;
    }
}

// The activations the fused inverted-residual forms take (ir.hip / irl.hip, host-checked): Relu /
// Clip / none, the same bounds on every channel, applied as min(max(v, lo), hi).  Bit for bit apply_act's result: Relu is max(v, 0)
// (min with +inf keeps it), Clip is the same min(max()), and max(v, -inf) / min(v, +inf) leave a
// finite v as it is.
struct Bounds {
    float lo, hi;
};
__device__ __forceinline__ Bounds bounds(const Act &a) {
    const float inf = __builtin_inff();
    return {a.kind == ACT_RELU ? 0.f : a.kind == ACT_CLIP ? a.lo : -inf, a.kind == ACT_CLIP ? a.hi : inf};
}
__device__ __forceinline__ float clamp(const Bounds &b, float v) { return fminf(fmaxf(v, b.lo), b.hi); }
inline bool bounds_act(const Act &a) { return a.kind == ACT_NONE || a.kind == ACT_RELU || a.kind == ACT_CLIP; }

}  // namespace zr
