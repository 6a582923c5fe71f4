// act.h -- activation epilogues of the ONNX graphs (Relu, Clip(0,6), PRelu, Sigmoid).
#pragma once
#include "../runtime/zr_kernels.h"

namespace zr {

__device__ __forceinline__ float apply_act(const Act &a, float v, int c) {
    switch (a.kind) {
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_CLIP: return fminf(fmaxf(v, a.lo), a.hi);
    case ACT_PRELU: return v < 0.f ? v * a.slope[c] : v;
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
    }
}

}  // namespace zr
