// lds_dma.h -- helpers shared by the LDS-DMA staged kernels (fused.hip, dwpw_mfma.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace zr {

// the models' TF-style left/top depthwise padding for a KxK stride-S conv
template <int K, int S> struct DwPad { static constexpr int L = S == 1 ? K / 2 : K / 2 - 1; };

// a / b for 0 <= a < 2^22 through the f32 reciprocal, corrected to the exact quotient
__device__ __forceinline__ int qdiv(int a, int b, float inv_b) {
    int q = (int)((float)a * inv_b);
    const int r = a - q * b;
    q += r >= b ? 1 : 0;
    q -= r < 0 ? 1 : 0;
    return q;
}

static __device__ const float4 zr_zero4 = {0.f, 0.f, 0.f, 0.f};  // LDS-DMA source of the zero slots

}  // namespace zr
