// sample.h -- the reference's per-pixel view lookup (K1), shared by the standalone
// preprocessing kernel and the stem kernel that samples frames directly, so both produce the
// same bits.  For network-input pixel (x, y) of an ow x oh tensor this reproduces, in IEEE f32
// with no contraction (files compiled with -ffp-contract=off, plus the pragma below):
//   Cnn::new sample()           crates/zaru/src/nn/mod.rs:54-58   u = x/w, sx = round(u*viewW)
//   ViewData::image_coord()     crates/zaru/src/image/mod.rs:224-240
//   RotatedRect::transform_out  crates/zaru-image/src/rect.rs:417-423
//   Mat2 * Vec2 left fold       crates/zaru-linalg/src/matrix/ops.rs:68-77
// cos/sin of the view angle come from the host's glibc (the reference evaluates them with the
// same libm per sample), so the only device math is +,-,*,/ and round - all exact.
#pragma once
#include "../runtime/zr_kernels.h"

namespace zr {

__device__ __forceinline__ uint32_t sat_u32(float f) {  // Rust `f as u32`
    if (!(f > 0.f)) return 0u;
    if (f >= 4294967296.f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

// Byte offset into the frame of the pixel that network-input pixel (x, y) samples, or -1
// where the reference returns Color::NONE (outside the image).
__device__ __forceinline__ int64_t sample_offset(const ViewDesc &d, const FrameDesc &f, int x, int y,
                                                 int ow, int oh) {
#pragma clang fp contract(off)
    const float u = (float)x / (float)ow;
    const float w = (float)y / (float)oh;
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

    if (fx < 0.f || fy < 0.f || ceilf(fx) >= 4294967296.f || ceilf(fy) >= 4294967296.f) return -1;
    const uint32_t ix = (uint32_t)roundf(fx), iy = (uint32_t)roundf(fy);
    if (ix >= f.w || iy >= f.h) return -1;
    return (int64_t)((uint64_t)iy * f.stride + (uint64_t)ix * 4);
}

// The frame a view samples.  Device-built view tables (zr_cnn_estimate_device_views_async) are
// not range-checked on the host: an index past the frame table samples a 0x0 frame (every
// pixel Color::NONE) through frame 0's valid pointer instead of reading past the table.
__device__ __forceinline__ FrameDesc frame_of(const PreprocParams &P, const ViewDesc &d) {
    const bool ok = d.frame < (uint32_t)P.nframes;
    FrameDesc f = P.frames[ok ? d.frame : 0];
    if (!ok) f.w = f.h = 0;
    return f;
}

// Load of a sampled pixel without a branch around the load (Color::NONE = 0 for -1).
__device__ __forceinline__ uint32_t load_pixel(const FrameDesc &f, int64_t off) {
    const uint32_t v = *(const uint32_t *)(f.rgba + (off >= 0 ? off : 0));
    return off >= 0 ? v : 0u;
}

// RGBA8 of the frame pixel that network-input pixel (x, y) samples; Color::NONE (0) outside.
__device__ __forceinline__ uint32_t sample_view(const ViewDesc &d, const FrameDesc &f, int x, int y,
                                                int ow, int oh) {
    return load_pixel(f, sample_offset(d, f, x, y, ow, oh));
}

// ColorMapper::map (crates/zaru/src/nn/mod.rs:156-167): c * ((hi - lo) / 255) + lo
__device__ __forceinline__ float color_map(uint32_t rgba, int ch, float adjust, float lo) {
#pragma clang fp contract(off)
    return (float)((rgba >> (8 * ch)) & 0xFF) * adjust + lo;
}

}  // namespace zr
