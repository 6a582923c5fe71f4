// geom_dev.h -- the reference's f32 geometry on the device, operation for operation as
// host/geometry.cpp restates it (crates/zaru-image/src/rect.rs, zaru-linalg), with glibc's
// own sinf / cosf / atan2f / expf (glibc_math.h).  Every kernel that includes this is compiled
// with -ffp-contract=off, so each a * b + c rounds twice, as Rust does.  Shared by track.hip
// (LandmarkTracker::track_impl) and detpost.hip (Detector::detect_impl post-processing).
#pragma once
#include "glibc_math.h"

namespace zr {
namespace geo {

struct V2 {
    float x, y;
};
struct RRect {  // Rect as (centre, size) (rect.rs:15-18) + rotation
    float cx, cy, w, h, rad;
};

__device__ __forceinline__ V2 rot_ccw(V2 v, float r) {  // matrix.rs:571-579, ops.rs:68-77
    const float c = glibc::cosf(r), s = glibc::sinf(r), ns = -s;
    return {(0.f + c * v.x) + ns * v.y, (0.f + s * v.x) + c * v.y};
}

__device__ __forceinline__ float signed_angle_to(V2 a, V2 b) {  // vector.rs:568-573
    const float perp = a.x * b.y - a.y * b.x;
    const float dot = (0.f + a.x * b.x) + a.y * b.y;
    return -glibc::atan2f(perp, dot);
}

__device__ __forceinline__ float sigmoid(float v) { return 1.f / (1.f + glibc::expf(-v)); }  // num.rs:6-8

__device__ __forceinline__ RRect from_top_left(float x, float y, float w, float h, float rad) {
    return {x + w * 0.5f, y + h * 0.5f, w, h, rad};
}

__device__ __forceinline__ V2 top_left(const RRect &r) { return {r.cx - r.w * 0.5f, r.cy - r.h * 0.5f}; }

__device__ __forceinline__ RRect grow_to_fit_aspect(RRect r, int aw, int ah) {  // rect.rs:104-117
    const float a = (float)aw / (float)ah;
    const float tw = r.h * a;
    if (tw >= r.w) {
        r.w += tw - r.w;
    } else {
        const float th = r.w / a;
        r.h += th - r.h;
    }
    return r;
}

__device__ __forceinline__ RRect grow_rel(RRect r, float a) {  // rect.rs:84-93
    const float l = r.w * a, t = r.h * a;
    r.w = r.w + l + l;
    r.h = r.h + t + t;
    return r;
}

__device__ __forceinline__ V2 transform_out(const RRect &r, V2 p) {  // rect.rs:417-423
    const V2 half = {r.w * 0.5f, r.h * 0.5f};
    const V2 q = rot_ccw({p.x - half.x, p.y - half.y}, r.rad);
    const V2 tl = top_left(r);
    return {q.x + half.x + tl.x, q.y + half.y + tl.y};
}

// ViewData::view (image/mod.rs:201-210): child in the parent's local coordinates
__device__ __forceinline__ RRect view_of(const RRect &parent, const RRect &child) {
    const float rad = parent.rad + child.rad;
    const V2 c = transform_out(parent, {child.cx, child.cy});
    return from_top_left(c.x - child.w * 0.5f, c.y - child.h * 0.5f, child.w, child.h, rad);
}

// Rect::iou (rect.rs:193-214): intersection of the (top left, top left + size) boxes as a span,
// its area over area(a) + area(b) - intersection
__device__ __forceinline__ float iou(float acx, float acy, float aw, float ah, float bcx, float bcy, float bw,
                                     float bh) {
    const float ax = acx - aw * 0.5f, ay = acy - ah * 0.5f, bx = bcx - bw * 0.5f, by = bcy - bh * 0.5f;
    const float mnx = fmaxf(ax, bx), mny = fmaxf(ay, by);
    const float mxx = fminf(ax + aw, bx + bw), mxy = fminf(ay + ah, by + bh);
    float inter = 0.f;
    if (!(mnx > mxx || mny > mxy)) {
        // Rect::bounding of {mn, mx} -> span -> from_top_left: size (mx - mn)
        const float x0 = fminf(mnx, mxx), y0 = fminf(mny, mxy), x1 = fmaxf(mnx, mxx), y1 = fmaxf(mny, mxy);
        inter = (x1 - x0) * (y1 - y0);
    }
    return inter / (aw * ah + bw * bh - inter);
}

}  // namespace geo
}  // namespace zr
