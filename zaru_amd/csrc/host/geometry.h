// geometry.h -- f32 geometry of the reference, operation for operation.
//
// Mirrors crates/zaru-image/src/rect.rs (Rect, RotatedRect), the few zaru-linalg routines the
// hot path uses (Mat2::rotation_counterclockwise, Mat*Vec, signed_angle_to) and
// crates/zaru/src/num.rs::sigmoid.  Compiled with -ffp-contract=off: every result rounds
// exactly as the Rust code does (no FMA contraction, same evaluation order, glibc libm).
#pragma once
#include <cmath>
#include <cstdint>
#include <vector>

namespace zh {

struct Vec2 {
    float x = 0.f, y = 0.f;
};

inline Vec2 operator+(Vec2 a, Vec2 b) { return {a.x + b.x, a.y + b.y}; }
inline Vec2 operator-(Vec2 a, Vec2 b) { return {a.x - b.x, a.y - b.y}; }
inline Vec2 operator*(Vec2 a, float s) { return {a.x * s, a.y * s}; }
inline Vec2 operator*(Vec2 a, Vec2 b) { return {a.x * b.x, a.y * b.y}; }  // element-wise
inline Vec2 vmin(Vec2 a, Vec2 b) { return {std::fmin(a.x, b.x), std::fmin(a.y, b.y)}; }
inline Vec2 vmax(Vec2 a, Vec2 b) { return {std::fmax(a.x, b.x), std::fmax(a.y, b.y)}; }

// zaru-linalg: rotation matrices and Vector::{rotate_*, signed_angle_to}
Vec2 rotate_counterclockwise(Vec2 v, float radians);
Vec2 rotate_clockwise(Vec2 v, float radians);
float signed_angle_to(Vec2 a, Vec2 b);
float sigmoid(float v);

struct AspectRatio {
    uint32_t w = 1, h = 1;
    static AspectRatio of(uint32_t w, uint32_t h);  // reduced by gcd (resolution.rs:145-155)
    float as_f32() const { return (float)w / (float)h; }
};

class Rect {
  public:
    Rect() = default;
    static Rect from_center(float x, float y, float w, float h) { return Rect({x, y}, {w, h}); }
    static Rect from_top_left(float x, float y, float w, float h) {
        return from_center(x + w * 0.5f, y + h * 0.5f, w, h);
    }
    static Rect span(float x0, float y0, float x1, float y1) {
        return from_top_left(x0, y0, x1 - x0, y1 - y0);
    }
    static bool bounding(const Vec2 *pts, size_t n, Rect &out);

    Vec2 center() const { return c_; }
    Vec2 size() const { return s_; }
    float width() const { return s_.x; }
    float height() const { return s_.y; }
    Vec2 top_left() const { return c_ - s_ * 0.5f; }
    float x() const { return top_left().x; }
    float y() const { return top_left().y; }
    float area() const { return s_.x * s_.y; }

    Rect scale(float s) const { return Rect(c_, s_ * s); }
    Rect grow_rel(float amount) const;
    Rect grow_to_fit_aspect(AspectRatio a) const;
    Rect move_by(Vec2 off) const { return Rect(c_ + off, s_); }
    Rect move_to(float x, float y) const { return from_top_left(x, y, s_.x, s_.y); }
    bool intersection(const Rect &o, Rect &out) const;
    float intersection_area(const Rect &o) const;
    float iou(const Rect &o) const;
    bool contains_point(Vec2 p) const;

    bool operator==(const Rect &o) const {
        return c_.x == o.c_.x && c_.y == o.c_.y && s_.x == o.s_.x && s_.y == o.s_.y;
    }

  private:
    Rect(Vec2 c, Vec2 s) : c_(c), s_(s) {}
    Vec2 c_, s_;
};

class RotatedRect {
  public:
    RotatedRect() = default;
    RotatedRect(Rect r, float radians) : rect_(r), rad_(radians) {}
    static bool bounding(float radians, const Vec2 *pts, size_t n, size_t stride_floats,
                         RotatedRect &out);

    const Rect &rect() const { return rect_; }
    float rotation_radians() const { return rad_; }
    Vec2 center() const { return rect_.center(); }
    RotatedRect with_rect(Rect r) const { return RotatedRect(r, rad_); }
    RotatedRect grow_rel(float a) const { return with_rect(rect_.grow_rel(a)); }
    RotatedRect grow_to_fit_aspect(AspectRatio a) const { return with_rect(rect_.grow_to_fit_aspect(a)); }
    Vec2 transform_in(Vec2 p) const;
    Vec2 transform_out(Vec2 p) const;
    bool contains_point(Vec2 p) const;

  private:
    Rect rect_;
    float rad_ = 0.f;
};

// ViewData (crates/zaru/src/image/mod.rs:188-248): a view is one RotatedRect in
// root-image coordinates; nested views compose with ViewData::view.
struct ViewData {
    RotatedRect rect;
    static ViewData full(uint32_t w, uint32_t h) {
        return {RotatedRect(Rect::from_top_left(0.f, 0.f, (float)w, (float)h), 0.f)};
    }
    ViewData view(const RotatedRect &child) const;
    Rect local_rect() const {  // ImageView::rect(): origin-anchored size of the view
        return Rect::from_top_left(0.f, 0.f, rect.rect().width(), rect.rect().height());
    }
};

}  // namespace zh
