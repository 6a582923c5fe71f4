// geometry.cpp -- see geometry.h.  Every function cites the Rust it reproduces.
#include "geometry.h"

#include <algorithm>

namespace zh {

// Mat2::rotation_counterclockwise (zaru-linalg/src/matrix.rs:571-579), columns
// [cos, sin], [-sin, cos]; Mat * Vec folds each row from 0 (matrix/ops.rs:68-77).
Vec2 rotate_counterclockwise(Vec2 v, float radians) {
    const float c = std::cos(radians), s = std::sin(radians), neg_s = -s;
    return {(0.f + c * v.x) + neg_s * v.y, (0.f + s * v.x) + c * v.y};
}

// rotation_clockwise(r) = rotation_counterclockwise(-r) (matrix.rs:563-568)
Vec2 rotate_clockwise(Vec2 v, float radians) { return rotate_counterclockwise(v, -radians); }

// Vector::signed_angle_to (zaru-linalg/src/vector.rs:568-573): -atan2(perp_dot, dot)
float signed_angle_to(Vec2 a, Vec2 b) {
    const float perp = a.x * b.y - a.y * b.x;       // cross().z, vector.rs:592-597,645-659
    const float dot = (0.f + a.x * b.x) + a.y * b.y;  // vector.rs:350-358
    return -std::atan2(perp, dot);
}

// crates/zaru/src/num.rs:6-8
float sigmoid(float v) { return 1.f / (1.f + std::exp(-v)); }

AspectRatio AspectRatio::of(uint32_t w, uint32_t h) {
    uint32_t a = w, b = h;
    while (b > 0) {
        uint32_t t = b;
        b = a % b;
        a = t;
    }
    return {w / a, h / a};
}

// rect.rs:49-62
bool Rect::bounding(const Vec2 *pts, size_t n, Rect &out) {
    if (n == 0) return false;
    Vec2 mn = pts[0], mx = pts[0];
    for (size_t i = 1; i < n; i++) {
        mn = vmin(mn, pts[i]);
        mx = vmax(mx, pts[i]);
    }
    out = span(mn.x, mn.y, mx.x, mx.y);
    return true;
}

// rect.rs:84-93
Rect Rect::grow_rel(float amount) const {
    const float left = width() * amount, right = width() * amount;
    const float top = height() * amount, bottom = height() * amount;
    return Rect(c_, {s_.x + left + right, s_.y + top + bottom});
}

// rect.rs:104-117
Rect Rect::grow_to_fit_aspect(AspectRatio a) const {
    Rect r = *this;
    const float target_width = height() * a.as_f32();
    if (target_width >= width()) {
        const float inc_w = target_width - width();
        r.s_.x += inc_w;
    } else {
        const float target_height = width() / a.as_f32();
        const float inc_h = target_height - height();
        r.s_.y += inc_h;
    }
    return r;
}

// rect.rs:193-201
bool Rect::intersection(const Rect &o, Rect &out) const {
    const Vec2 mn = vmax(top_left(), o.top_left());
    const Vec2 mx = vmin(top_left() + size(), o.top_left() + o.size());
    if (mn.x > mx.x || mn.y > mx.y) return false;
    const Vec2 pts[2] = {mn, mx};
    return bounding(pts, 2, out);
}

// rect.rs:203-214
float Rect::intersection_area(const Rect &o) const {
    Rect i;
    return intersection(o, i) ? i.area() : 0.f;
}

float Rect::iou(const Rect &o) const {
    const float inter = intersection_area(o);
    return inter / (area() + o.area() - inter);
}

// rect.rs:216-222
bool Rect::contains_point(Vec2 p) const {
    return x() <= p.x && y() <= p.y && x() + width() >= p.x && y() + height() >= p.y;
}

// rect.rs:287-325
bool RotatedRect::bounding(float radians, const Vec2 *pts, size_t n, size_t stride_floats,
                           RotatedRect &out) {
    if (n == 0) return false;
    const float c = std::cos(-radians), s = std::sin(-radians), neg_s = -s;
    Vec2 mn{3.40282347e38f, 3.40282347e38f}, mx{-3.40282347e38f, -3.40282347e38f};
    const float *f = reinterpret_cast<const float *>(pts);
    for (size_t i = 0; i < n; i++) {
        const Vec2 p{f[i * stride_floats], f[i * stride_floats + 1]};
        const Vec2 r{(0.f + c * p.x) + neg_s * p.y, (0.f + s * p.x) + c * p.y};
        mn = vmin(mn, r);
        mx = vmax(mx, r);
    }
    const Vec2 center = rotate_counterclockwise((mn + mx) * 0.5f, radians);
    const Vec2 size = mx - mn;
    out = RotatedRect(Rect::from_center(center.x, center.y, size.x, size.y), radians);
    return true;
}

// rect.rs:405-412
Vec2 RotatedRect::transform_in(Vec2 p) const {
    const Vec2 half = rect_.size() * 0.5f;
    const Vec2 pos = p - rect_.top_left() - half;
    return rotate_clockwise(pos, rad_) + half;
}

// rect.rs:417-423
Vec2 RotatedRect::transform_out(Vec2 p) const {
    const Vec2 half = rect_.size() * 0.5f;
    return rotate_counterclockwise(p - half, rad_) + half + rect_.top_left();
}

// rect.rs:395-400
bool RotatedRect::contains_point(Vec2 p) const {
    return rect_.move_to(0.f, 0.f).contains_point(transform_in(p));
}

// image/mod.rs:201-210
ViewData ViewData::view(const RotatedRect &child) const {
    const float radians = rect.rotation_radians() + child.rotation_radians();
    const Vec2 pos = rect.transform_out(child.rect().center()) - child.rect().size() * 0.5f;
    return {RotatedRect(child.rect().move_to(pos.x, pos.y), radians)};
}

}  // namespace zh
