// lds_dma.h -- helpers shared by the LDS-DMA staged kernels (fused.hip, dwpw_mfma.hip, dwpw_ws.hip).
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

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate is a compile-time field): wait
// until at most n of this wave's vector-memory instructions (LDS-DMA included) are outstanding
__device__ __forceinline__ void wait_vmcnt_dyn(int n) {
    switch (__builtin_amdgcn_readfirstlane(n < 0 ? 0 : n)) {
#define ZR_VMW(i) case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
        ZR_VMW(0) ZR_VMW(1) ZR_VMW(2) ZR_VMW(3) ZR_VMW(4) ZR_VMW(5) ZR_VMW(6) ZR_VMW(7)
        ZR_VMW(8) ZR_VMW(9) ZR_VMW(10) ZR_VMW(11) ZR_VMW(12) ZR_VMW(13) ZR_VMW(14) ZR_VMW(15)
        ZR_VMW(16) ZR_VMW(17) ZR_VMW(18) ZR_VMW(19) ZR_VMW(20) ZR_VMW(21) ZR_VMW(22) ZR_VMW(23)
        ZR_VMW(24) ZR_VMW(25) ZR_VMW(26) ZR_VMW(27) ZR_VMW(28) ZR_VMW(29) ZR_VMW(30) ZR_VMW(31)
        ZR_VMW(32) ZR_VMW(33) ZR_VMW(34) ZR_VMW(35) ZR_VMW(36) ZR_VMW(37) ZR_VMW(38) ZR_VMW(39)
        ZR_VMW(40) ZR_VMW(41) ZR_VMW(42) ZR_VMW(43) ZR_VMW(44) ZR_VMW(45) ZR_VMW(46) ZR_VMW(47)
        ZR_VMW(48) ZR_VMW(49) ZR_VMW(50) ZR_VMW(51) ZR_VMW(52) ZR_VMW(53) ZR_VMW(54) ZR_VMW(55)
        ZR_VMW(56) ZR_VMW(57) ZR_VMW(58) ZR_VMW(59) ZR_VMW(60) ZR_VMW(61) ZR_VMW(62)
#undef ZR_VMW
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
    }
}

static __device__ const float4 zr_zero4 = {0.f, 0.f, 0.f, 0.f};  // LDS-DMA source of the zero slots

}  // namespace zr
