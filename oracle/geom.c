/*
 * geom.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * f32-exact restatement of the reference's geometry, preprocessing and post-processing.
 * Compiled with -ffp-contract=off: Rust never contracts a*b+c into an FMA, and every
 * expression below keeps the Rust evaluation order (left fold from 0.0 for Mat*Vec and
 * dot products, true division, glibc sinf/cosf/expf/atan2f).
 * Paths are relative to /root/reference.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ geometry */

/* crates/zaru-image/src/rect.rs:23-28 */
zo_rect zo_rect_from_center(float x, float y, float w, float h) {
    zo_rect r = {x, y, w, h};
    return r;
}

/* rect.rs:32-39 */
zo_rect zo_rect_from_top_left(float x, float y, float w, float h) {
    return zo_rect_from_center(x + w * 0.5f, y + h * 0.5f, w, h);
}

/* rect.rs:135-137: centre - size * 0.5 */
void zo_rect_top_left(const zo_rect *r, float out[2]) {
    out[0] = r->cx - r->w * 0.5f;
    out[1] = r->cy - r->h * 0.5f;
}

/* rect.rs:84-93 */
zo_rect zo_rect_grow_rel(zo_rect r, float amount) {
    float left = r.w * amount, right = r.w * amount;
    float top = r.h * amount, bottom = r.h * amount;
    r.w = r.w + left + right;
    r.h = r.h + top + bottom;
    return r;
}

static uint32_t gcd_u32(uint32_t a, uint32_t b) { /* resolution.rs:176-184 */
    while (b > 0) {
        uint32_t t = b;
        b = a % b;
        a = t;
    }
    return a;
}

/* rect.rs:104-117 with AspectRatio::as_f32 (resolution.rs:145-161) */
zo_rect zo_rect_grow_to_fit_aspect(zo_rect r, uint32_t aw, uint32_t ah) {
    uint32_t g = gcd_u32(aw, ah);
    float aspect = (float)(aw / g) / (float)(ah / g);
    float target_width = r.h * aspect;
    if (target_width >= r.w) {
        float inc_w = target_width - r.w;
        r.w += inc_w;
    } else {
        float target_height = r.w / aspect;
        float inc_h = target_height - r.h;
        r.h += inc_h;
    }
    return r;
}

/* rect.rs:64-68 span_inner via from_top_left */
static zo_rect span_inner(float x0, float y0, float x1, float y1) {
    return zo_rect_from_top_left(x0, y0, x1 - x0, y1 - y0);
}

/* rect.rs:193-201 */
int zo_rect_intersection(const zo_rect *a, const zo_rect *b, zo_rect *out) {
    float ta[2], tb[2];
    zo_rect_top_left(a, ta);
    zo_rect_top_left(b, tb);
    float mnx = fmaxf(ta[0], tb[0]), mny = fmaxf(ta[1], tb[1]);
    float mxx = fminf(ta[0] + a->w, tb[0] + b->w);
    float mxy = fminf(ta[1] + a->h, tb[1] + b->h);
    if (mnx > mxx || mny > mxy) return 0;
    /* Rect::bounding([min, max]) (rect.rs:49-62) */
    float bx0 = fminf(mnx, mxx), by0 = fminf(mny, mxy);
    float bx1 = fmaxf(mnx, mxx), by1 = fmaxf(mny, mxy);
    *out = span_inner(bx0, by0, bx1, by1);
    return 1;
}

/* rect.rs:203-214 */
float zo_rect_iou(const zo_rect *a, const zo_rect *b) {
    zo_rect i;
    float inter = zo_rect_intersection(a, b, &i) ? i.w * i.h : 0.0f;
    float uni = a->w * a->h + b->w * b->h - inter;
    return inter / uni;
}

/* Mat2::rotation_counterclockwise (zaru-linalg/src/matrix.rs:571-579) applied as
 * Mat * Vec (matrix/ops.rs:68-77): row r = (0 + m[r][0]*x) + m[r][1]*y. */
static void rot_ccw(float rad, float x, float y, float out[2]) {
    float c = cosf(rad), s = sinf(rad);
    float ns = -s;
    out[0] = (0.0f + c * x) + ns * y;
    out[1] = (0.0f + s * x) + c * y;
}

/* rotation_clockwise(r) = rotation_counterclockwise(-r) (matrix.rs:563-568) */
static void rot_cw(float rad, float x, float y, float out[2]) { rot_ccw(-rad, x, y, out); }

/* rect.rs:417-423 */
void zo_rrect_transform_out(const zo_rrect *r, float x, float y, float out[2]) {
    float chx = r->rect.w * 0.5f, chy = r->rect.h * 0.5f;
    float tl[2];
    zo_rect_top_left(&r->rect, tl);
    float v[2];
    rot_ccw(r->rad, x - chx, y - chy, v);
    out[0] = (v[0] + chx) + tl[0];
    out[1] = (v[1] + chy) + tl[1];
}

/* rect.rs:405-412 */
void zo_rrect_transform_in(const zo_rrect *r, float x, float y, float out[2]) {
    float chx = r->rect.w * 0.5f, chy = r->rect.h * 0.5f;
    float tl[2];
    zo_rect_top_left(&r->rect, tl);
    float px = (x - tl[0]) - chx, py = (y - tl[1]) - chy;
    float v[2];
    rot_cw(r->rad, px, py, v);
    out[0] = v[0] + chx;
    out[1] = v[1] + chy;
}

/* rect.rs:287-325 */
int zo_rrect_bounding(float rad, const float *pts, size_t n, size_t stride, zo_rrect *out) {
    if (n == 0) return 0;
    float c = cosf(-rad), s = sinf(-rad), ns = -s;
    float mnx = 3.40282347e38f, mny = 3.40282347e38f;
    float mxx = -3.40282347e38f, mxy = -3.40282347e38f;
    for (size_t i = 0; i < n; i++) {
        float x = pts[i * stride], y = pts[i * stride + 1];
        float px = (0.0f + c * x) + ns * y;
        float py = (0.0f + s * x) + c * y;
        mnx = fminf(mnx, px);
        mny = fminf(mny, py);
        mxx = fmaxf(mxx, px);
        mxy = fmaxf(mxy, py);
    }
    float cx = (mnx + mxx) * 0.5f, cy = (mny + mxy) * 0.5f;
    float ctr[2];
    rot_ccw(rad, cx, cy, ctr);
    out->rect = zo_rect_from_center(ctr[0], ctr[1], mxx - mnx, mxy - mny);
    out->rad = rad;
    return 1;
}

/* vector.rs:568-573, perp_dot 592-597 (cross 645-659), dot 350-358 */
float zo_signed_angle_to(float ax, float ay, float bx, float by) {
    float perp = ax * by - ay * bx;
    float dot = (0.0f + ax * bx) + ay * by;
    return -atan2f(perp, dot);
}

/* crates/zaru/src/num.rs:6-8 */
float zo_sigmoid(float v) { return 1.0f / (1.0f + expf(-v)); }

/* ------------------------------------------------------------------ image views */

/* image/mod.rs:195-199 with Image::rect (image/mod.rs:142-144) */
zo_rrect zo_view_full(uint32_t w, uint32_t h) {
    zo_rrect r;
    r.rect = zo_rect_from_top_left(0.0f, 0.0f, (float)w, (float)h);
    r.rad = 0.0f;
    return r;
}

/* image/mod.rs:201-210 */
zo_rrect zo_view_compose(const zo_rrect *parent, const zo_rrect *child) {
    float rad = parent->rad + child->rad;
    float p[2];
    zo_rrect_transform_out(parent, child->rect.cx, child->rect.cy, p);
    float px = p[0] - child->rect.w * 0.5f, py = p[1] - child->rect.h * 0.5f;
    zo_rrect out;
    out.rect = zo_rect_from_top_left(px, py, child->rect.w, child->rect.h); /* move_to */
    out.rad = rad;
    return out;
}

/* image/mod.rs:224-247 */
uint32_t zo_view_get(const uint8_t *rgba, uint32_t w, uint32_t h, size_t stride,
                     const zo_rrect *view, uint32_t x, uint32_t y) {
    float o[2];
    zo_rrect_transform_out(view, (float)x + 0.5f, (float)y + 0.5f, o);
    float fx = roundf(o[0] - 0.5f), fy = roundf(o[1] - 0.5f);
    if (fx < 0.0f || fy < 0.0f || ceilf(fx) >= 4294967296.0f || ceilf(fy) >= 4294967296.0f)
        return 0;
    uint32_t ix = (uint32_t)roundf(fx), iy = (uint32_t)roundf(fy);
    if (ix >= w || iy >= h) return 0;
    const uint8_t *p = rgba + (size_t)iy * stride + (size_t)ix * 4;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* Rust `f as u32`: saturating, NaN -> 0 */
static uint32_t sat_u32(float f) {
    if (!(f > 0.0f)) return 0;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

/* nn/mod.rs:54-67 (sample + NCHW image_map) and ColorMapper::map (nn/mod.rs:156-167) */
void zo_preproc(const uint8_t *rgba, uint32_t w, uint32_t h, size_t stride,
                const zo_rrect *view, uint32_t ow, uint32_t oh, float lo, float hi, float *out) {
    float vw = view->rect.w, vh = view->rect.h;
    float adjust = (hi - lo) / 255.0f;
    for (uint32_t c = 0; c < 3; c++) {
        for (uint32_t y = 0; y < oh; y++) {
            for (uint32_t x = 0; x < ow; x++) {
                float u = (float)x / (float)ow, v = (float)y / (float)oh;
                uint32_t sx = sat_u32(roundf(u * vw));
                uint32_t sy = sat_u32(roundf(v * vh));
                uint32_t col = zo_view_get(rgba, w, h, stride, view, sx, sy);
                uint32_t ch = (col >> (8 * c)) & 0xFF;
                out[(size_t)c * oh * ow + (size_t)y * ow + x] = (float)ch * adjust + lo;
            }
        }
    }
}

/* ------------------------------------------------------------------ SSD */

/* detection/ssd.rs:96-119 */
size_t zo_anchors(const uint32_t *layers, size_t nlayers, float *out_xy) {
    size_t n = 0;
    for (size_t l = 0; l < nlayers; l++) {
        uint32_t boxes = layers[3 * l], lw = layers[3 * l + 1], lh = layers[3 * l + 2];
        for (uint32_t y = 0; y < lh; y++)
            for (uint32_t x = 0; x < lw; x++)
                for (uint32_t b = 0; b < boxes; b++) {
                    if (out_xy) {
                        out_xy[2 * n] = ((float)x + 0.5f) / (float)lw;
                        out_xy[2 * n + 1] = ((float)y + 0.5f) / (float)lh;
                    }
                    n++;
                }
    }
    return n;
}

/* face/detection.rs:96-157 (kind 0 short range, kind 2 full range: the same
 * extract_outputs over different anchors) and hand/detection.rs:108-179 (kind 1) */
size_t zo_extract(int kind, const float *boxes, const float *confs, size_t nanchors,
                  const float *anchors_xy, uint32_t in_w, uint32_t in_h, float thresh,
                  zo_det *out, size_t cap) {
    const int face = kind != 1;
    size_t np = face ? 16 : 18, nkp = face ? 6 : 7, n = 0;
    float isx = (float)in_w, isy = (float)in_h;
    for (size_t i = 0; i < nanchors; i++) {
        float conf = zo_sigmoid(confs[i]);
        if (conf < thresh) continue;
        if (n >= cap) break;
        const float *b = boxes + i * np;
        zo_det *d = &out[n++];
        memset(d, 0, sizeof(*d));
        float cx = b[0] + anchors_xy[2 * i] * isx;
        float cy = b[1] + anchors_xy[2 * i + 1] * isy;
        d->conf = conf;
        d->anchor = (int32_t)i;
        d->rect = zo_rect_from_center(cx, cy, b[2], b[3]);
        d->nkp = (int32_t)nkp;
        for (size_t k = 0; k < nkp; k++) { /* quirk kept: offset is centre * input_size */
            d->kp[k][0] = b[4 + 2 * k] + cx * isx;
            d->kp[k][1] = b[5 + 2 * k] + cy * isy;
        }
        if (face) {
            float dx = d->kp[1][0] - d->kp[0][0], dy = d->kp[1][1] - d->kp[0][1];
            d->angle = zo_signed_angle_to(dx, dy, 1.0f, 0.0f);
        } else {
            float dx = d->kp[0][0] - d->kp[2][0], dy = d->kp[0][1] - d->kp[2][1];
            d->angle = zo_signed_angle_to(dx, dy, 0.0f, 1.0f);
        }
    }
    return n;
}

/* f32::total_cmp (zaru-image/src/num.rs:7-27) */
static int32_t total_key(float f) {
    int32_t i;
    memcpy(&i, &f, 4);
    return i ^ (int32_t)(((uint32_t)(i >> 31)) >> 1);
}

/* Tie rule: stable ascending sort (Rust's sort_unstable uses an insertion sort for
 * slices of <= 20 elements, which is stable); documented in DESIGN.md. */
static void sort_by_conf(zo_det *d, size_t n) {
    for (size_t i = 1; i < n; i++) {
        zo_det t = d[i];
        int32_t k = total_key(t.conf);
        size_t j = i;
        while (j > 0 && total_key(d[j - 1].conf) > k) {
            d[j] = d[j - 1];
            j--;
        }
        d[j] = t;
    }
}

/* detection/nms.rs:59-145 */
size_t zo_nms(zo_det *dets, size_t n, float iou_thresh, int mode, zo_det *out) {
    size_t nout = 0;
    zo_det *avg = (zo_det *)malloc(sizeof(zo_det) * (n ? n : 1));
    sort_by_conf(dets, n);
    while (n > 0) {
        zo_det seed = dets[--n];
        size_t keep = 0, navg = 0;
        if (mode == 0) {
            for (size_t i = 0; i < n; i++) {
                float iou = zo_rect_iou(&seed.rect, &dets[i].rect);
                if (iou < iou_thresh) dets[keep++] = dets[i];
            }
            n = keep;
            out[nout++] = seed;
            continue;
        }
        avg[navg++] = seed;
        for (size_t i = 0; i < n; i++) {
            float iou = zo_rect_iou(&seed.rect, &dets[i].rect);
            if (iou >= iou_thresh)
                avg[navg++] = dets[i];
            else
                dets[keep++] = dets[i];
        }
        n = keep;
        float ax = 0.0f, ay = 0.0f, aw = 0.0f, ah = 0.0f, aa = 0.0f, divisor = 0.0f;
        zo_det acc;
        memset(&acc, 0, sizeof(acc));
        acc.conf = seed.conf;
        acc.anchor = seed.anchor;
        for (size_t j = 0; j < navg; j++) {
            const zo_det *d = &avg[j];
            if (acc.nkp == 0 && d->nkp != 0) acc.nkp = d->nkp;
            float f = d->conf;
            divisor += f;
            for (int k = 0; k < acc.nkp; k++) {
                acc.kp[k][0] += d->kp[k][0] * f;
                acc.kp[k][1] += d->kp[k][1] * f;
            }
            ax += d->rect.cx * f;
            ay += d->rect.cy * f;
            aw += d->rect.w * f;
            ah += d->rect.h * f;
            aa += d->angle * f;
        }
        for (int k = 0; k < acc.nkp; k++) {
            acc.kp[k][0] /= divisor;
            acc.kp[k][1] /= divisor;
        }
        ax /= divisor;
        ay /= divisor;
        aw /= divisor;
        ah /= divisor;
        aa /= divisor;
        acc.rect = zo_rect_from_center(ax, ay, aw, ah);
        acc.angle = aa;
        out[nout++] = acc;
    }
    free(avg);
    return nout;
}

/* detection.rs:245-267 */
void zo_detector_map(zo_det *dets, size_t n, const zo_rect *rect, uint32_t in_w) {
    float scale = rect->w / (float)in_w;
    float tl[2];
    zo_rect_top_left(rect, tl);
    for (size_t i = 0; i < n; i++) {
        zo_det *d = &dets[i];
        d->rect = zo_rect_from_center(d->rect.cx * scale, d->rect.cy * scale, d->rect.w * scale,
                                      d->rect.h * scale);
        for (int k = 0; k < d->nkp; k++) {
            d->kp[k][0] *= scale;
            d->kp[k][1] *= scale;
        }
        d->rect.cx = d->rect.cx + tl[0];
        d->rect.cy = d->rect.cy + tl[1];
        for (int k = 0; k < d->nkp; k++) {
            d->kp[k][0] += tl[0];
            d->kp[k][1] += tl[1];
        }
    }
}

/* detection.rs:216-270 given the raw network outputs */
size_t zo_detect_post(int kind, const float *boxes, const float *confs, size_t nanchors,
                      uint32_t img_w, uint32_t img_h, uint32_t in_w, uint32_t in_h,
                      float thresh, float iou, zo_det *out, size_t cap) {
    return zo_detect_post_mode(kind, boxes, confs, nanchors, img_w, img_h, in_w, in_h, thresh, iou, 1, out, cap);
}

/* the same with SuppressionMode (nms.rs:154-163: 0 Remove, 1 Average) */
size_t zo_detect_post_mode(int kind, const float *boxes, const float *confs, size_t nanchors,
                           uint32_t img_w, uint32_t img_h, uint32_t in_w, uint32_t in_h,
                           float thresh, float iou, int mode, zo_det *out, size_t cap) {
    uint32_t face_layers[] = {2, 16, 16, 6, 8, 8};   /* face/detection.rs:53 */
    uint32_t palm_layers[] = {2, 24, 24, 6, 12, 12}; /* hand/detection.rs:117 */
    uint32_t full_layers[] = {1, 48, 48};            /* face/detection.rs:86-88 */
    const uint32_t *layers = kind == 0 ? face_layers : kind == 1 ? palm_layers : full_layers;
    const size_t nl = kind == 2 ? 1 : 2;
    size_t na = zo_anchors(layers, nl, NULL);
    if (na != nanchors) return 0;
    float *anchors = (float *)malloc(sizeof(float) * 2 * na);
    zo_anchors(layers, nl, anchors);
    zo_det *tmp = (zo_det *)malloc(sizeof(zo_det) * na);
    size_t n = zo_extract(kind, boxes, confs, na, anchors, in_w, in_h, thresh, tmp, na);
    zo_det *nms = (zo_det *)malloc(sizeof(zo_det) * (n ? n : 1));
    size_t m = zo_nms(tmp, n, iou, mode, nms);
    zo_rect full = zo_rect_from_top_left(0.0f, 0.0f, (float)img_w, (float)img_h);
    zo_rect rect = zo_rect_grow_to_fit_aspect(full, in_w, in_h);
    zo_detector_map(nms, m, &rect, in_w);
    if (m > cap) m = cap;
    memcpy(out, nms, sizeof(zo_det) * m);
    free(anchors);
    free(tmp);
    free(nms);
    return m;
}

/* landmark.rs:336-345 */
void zo_estimator_map(float *pos, size_t n, const zo_rect *rect, uint32_t in_w) {
    float scale = rect->w / (float)in_w;
    float tl[2];
    zo_rect_top_left(rect, tl);
    for (size_t i = 0; i < n; i++) {
        pos[3 * i] *= scale;
        pos[3 * i + 1] *= scale;
        pos[3 * i + 2] *= scale;
        pos[3 * i] += tl[0];
        pos[3 * i + 1] += tl[1];
    }
}

/* landmark.rs:479-494 */
int zo_tracker_update(float *pos, size_t n, const zo_rrect *view_rect, float roi_rad,
                      float est_angle, float padding, zo_rrect *updated, zo_rrect *next_roi) {
    float angle = roi_rad + est_angle;
    for (size_t i = 0; i < n; i++) {
        float o[2];
        zo_rrect_transform_out(view_rect, pos[3 * i], pos[3 * i + 1], o);
        pos[3 * i] = o[0];
        pos[3 * i + 1] = o[1];
    }
    if (!zo_rrect_bounding(angle, pos, n, 3, updated)) return 0;
    *next_roi = *updated;
    next_roi->rect = zo_rect_grow_rel(updated->rect, padding);
    return 1;
}

/* Estimate::angle_radians of the landmark networks, on view-local positions (n x 3):
 * FaceMesh V1 / V2 rotation_radians (mediapipe.rs:146-160, 407-421): (right_eye 263 -
 *   left_eye 33).signed_angle_to(X);
 * hand landmark rotation_radians (hand/landmark.rs:68-78): (wrist 0 - middle MCP 9)
 *   .signed_angle_to(Y). */
float zo_landmark_angle(int kind, const float *pos) {
    if (kind == 0) {
        float dx = pos[3 * 263] - pos[3 * 33], dy = pos[3 * 263 + 1] - pos[3 * 33 + 1];
        return zo_signed_angle_to(dx, dy, 1.0f, 0.0f);
    }
    float dx = pos[0] - pos[3 * 9], dy = pos[1] - pos[3 * 9 + 1];
    return zo_signed_angle_to(dx, dy, 0.0f, 1.0f);
}
