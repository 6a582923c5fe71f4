// preproc.hip -- K1: batched view sampling + ColorMapper, bit-exact with the reference.
//
// For every output element (view v, y, x) this reproduces, in IEEE f32 with no
// contraction (file compiled with -ffp-contract=off, plus the pragma below):
//   Cnn::new sample()           crates/zaru/src/nn/mod.rs:54-58   u = x/w, sx = round(u*viewW)
//   ViewData::image_coord()     crates/zaru/src/image/mod.rs:224-240
//   RotatedRect::transform_out  crates/zaru-image/src/rect.rs:417-423
//   Mat2 * Vec2 left fold       crates/zaru-linalg/src/matrix/ops.rs:68-77
//   ColorMapper::map            crates/zaru/src/nn/mod.rs:156-167
// cos/sin of the view angle come from the host's glibc (the reference evaluates them with
// the same libm per sample), so the only device math is +,-,*,/ and round - all exact.
// The tensor is written straight into the network's input layout (CNHW for the HIP
// runtime), so no separate relayout pass exists.
#include "../runtime/zr_kernels.h"

namespace zr {

__device__ __forceinline__ uint32_t sat_u32(float f) {  // Rust `f as u32`
    if (!(f > 0.f)) return 0u;
    if (f >= 4294967296.f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

__global__ __launch_bounds__(256) void preproc_kernel(const PreprocParams P) {
#pragma clang fp contract(off)
    const int v = blockIdx.y;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P.OW * P.OH) return;
    const int y = q / P.OW, x = q - y * P.OW;
    const ViewDesc d = P.views[v];
    const FrameDesc f = P.frames[d.frame];

    const float u = (float)x / (float)P.OW;
    const float w = (float)y / (float)P.OH;
    const uint32_t sx = sat_u32(roundf(u * d.view_w));
    const uint32_t sy = sat_u32(roundf(w * d.view_h));

    const float px = (float)sx + 0.5f, py = (float)sy + 0.5f;
    const float vx = px - d.half_w, vy = py - d.half_h;
    const float ns = -d.sin_r;
    const float rx = (0.f + d.cos_r * vx) + ns * vy;
    const float ry = (0.f + d.sin_r * vx) + d.cos_r * vy;
    const float ox = (rx + d.half_w) + d.tl_x;
    const float oy = (ry + d.half_h) + d.tl_y;
    const float fx = roundf(ox - 0.5f), fy = roundf(oy - 0.5f);

    uint32_t rgba = 0;  // Color::NONE
    if (!(fx < 0.f || fy < 0.f || ceilf(fx) >= 4294967296.f || ceilf(fy) >= 4294967296.f)) {
        const uint32_t ix = (uint32_t)roundf(fx), iy = (uint32_t)roundf(fy);
        if (ix < f.w && iy < f.h)
            rgba = *(const uint32_t *)(f.rgba + (uint64_t)iy * f.stride + (uint64_t)ix * 4);
    }
    float *o = P.out + (int64_t)v * P.o_sN + q;
    o[0] = (float)(rgba & 0xFF) * P.adjust + P.lo;
    o[P.o_sC] = (float)((rgba >> 8) & 0xFF) * P.adjust + P.lo;
    o[2 * P.o_sC] = (float)((rgba >> 16) & 0xFF) * P.adjust + P.lo;
}

const char *launch_preproc(const PreprocParams &p, hipStream_t s) {
    if (p.nviews == 0) return "preproc_kernel";
    dim3 grid((p.OW * p.OH + 255) / 256, p.nviews);
    hipLaunchKernelGGL(preproc_kernel, grid, dim3(256), 0, s, p);
    return "preproc_kernel";
}

}  // namespace zr
