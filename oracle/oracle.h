/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference (placrosse/Zaru) hot path, used exclusively as
 * the checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * Nothing in zaru_amd/ links, loads or calls this code; the product path fails
 * loudly when its HIP extension is missing instead of falling back to it.
 *
 * Two halves:
 *   geom.c     f32-exact restatement (compiled with -ffp-contract=off, glibc libm) of
 *              view sampling, colour mapping, SSD anchors, BlazeFace/BlazePalm decode,
 *              weighted NMS and landmark/ROI mapping.  Each function cites the Rust
 *              it follows (paths relative to /root/reference).
 *   nnexec_*.c generic ONNX interpreter (NCHW, batch 1) in f64 and f32: a restatement of
 *              the standard ONNX operator definitions that ONNX Runtime 1.14.8 / tract
 *              0.20.7 implement for the reference (crates/zaru/src/nn/mod.rs:450-538).
 *              Parity of network outputs is tolerance-based.
 */
#ifndef ZARU_ORACLE_H
#define ZARU_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* rect.rs:15-18 -- a Rect is stored as (centre, size). */
typedef struct { float cx, cy, w, h; } zo_rect;
/* rect.rs:270-273 */
typedef struct { zo_rect rect; float rad; } zo_rrect;

#define ZO_MAX_KP 8
/* detection.rs:288-293 (+ the anchor index, used only for the documented tie rule) */
typedef struct {
    float conf, angle;
    zo_rect rect;
    int32_t nkp;
    int32_t anchor;
    float kp[ZO_MAX_KP][2];
} zo_det;

/* ---- geometry (crates/zaru-image/src/rect.rs, crates/zaru-linalg) ---- */
zo_rect zo_rect_from_top_left(float x, float y, float w, float h);
zo_rect zo_rect_from_center(float x, float y, float w, float h);
void zo_rect_top_left(const zo_rect *r, float out[2]);
zo_rect zo_rect_grow_rel(zo_rect r, float amount);
zo_rect zo_rect_grow_to_fit_aspect(zo_rect r, uint32_t aw, uint32_t ah);
int zo_rect_intersection(const zo_rect *a, const zo_rect *b, zo_rect *out);
float zo_rect_iou(const zo_rect *a, const zo_rect *b);
void zo_rrect_transform_out(const zo_rrect *r, float x, float y, float out[2]);
void zo_rrect_transform_in(const zo_rrect *r, float x, float y, float out[2]);
int zo_rrect_bounding(float rad, const float *pts, size_t n, size_t stride, zo_rrect *out);
float zo_signed_angle_to(float ax, float ay, float bx, float by);
float zo_sigmoid(float v);

/* ---- image views (crates/zaru/src/image/mod.rs) ---- */
zo_rrect zo_view_full(uint32_t w, uint32_t h);
zo_rrect zo_view_compose(const zo_rrect *parent, const zo_rrect *child);
/* returns packed RGBA (r in the low byte) or 0 for Color::NONE */
uint32_t zo_view_get(const uint8_t *rgba, uint32_t w, uint32_t h, size_t stride,
                     const zo_rrect *view, uint32_t x, uint32_t y);
/* Cnn::new image_map closure, NCHW: out[c*oh*ow + y*ow + x] */
void zo_preproc(const uint8_t *rgba, uint32_t w, uint32_t h, size_t stride,
                const zo_rrect *view, uint32_t ow, uint32_t oh, float lo, float hi, float *out);

/* ---- SSD / decode / NMS (crates/zaru/src/detection/, face/, hand/) ---- */
size_t zo_anchors(const uint32_t *layers /* {boxes,w,h}* */, size_t nlayers, float *out_xy);
size_t zo_extract(int kind /*0 face(16 params), 1 palm(18)*/, const float *boxes,
                  const float *confs, size_t nanchors, const float *anchors_xy,
                  uint32_t in_w, uint32_t in_h, float thresh, zo_det *out, size_t cap);
size_t zo_nms(zo_det *dets, size_t n, float iou_thresh, int mode /*0 remove,1 average*/,
              zo_det *out);
void zo_detector_map(zo_det *dets, size_t n, const zo_rect *rect, uint32_t in_w);

/* Detector::detect_impl end to end given raw outputs (detection.rs:216-270) */
size_t zo_detect_post(int kind, const float *boxes, const float *confs, size_t nanchors,
                      uint32_t img_w, uint32_t img_h, uint32_t in_w, uint32_t in_h,
                      float thresh, float iou, zo_det *out, size_t cap);
size_t zo_detect_post_mode(int kind, const float *boxes, const float *confs, size_t nanchors,
                           uint32_t img_w, uint32_t img_h, uint32_t in_w, uint32_t in_h,
                           float thresh, float iou, int mode, zo_det *out, size_t cap);

/* Estimator::estimate_impl map-out (landmark.rs:314-348): positions in place, n x 3 */
void zo_estimator_map(float *pos, size_t n, const zo_rect *view_local_rect, uint32_t in_w);
/* LandmarkTracker::track_impl steps 4-5 (landmark.rs:479-494) */
int zo_tracker_update(float *pos, size_t n, const zo_rrect *view_rect, float roi_rad,
                      float est_angle, float padding, zo_rrect *updated, zo_rrect *next_roi);
/* Estimate::angle_radians (kind 0 FaceMesh V1, mediapipe.rs:146-160; 1 hand,
 * hand/landmark.rs:68-78) of view-local positions (n x 3) */
float zo_landmark_angle(int kind, const float *pos);

/* ---- ONNX interpreter (nnexec) ---- */
typedef struct zo_net zo_net;
zo_net *zo_net_load(const uint8_t *bytes, size_t len, int f64);
void zo_net_free(zo_net *n);
size_t zo_net_num_outputs(const zo_net *n);
/* output shape of idx (after a run or from graph value_info); returns rank */
size_t zo_net_output_shape(const zo_net *n, size_t idx, int64_t *shape);
/* input: NCHW 1x3xHxW float; outputs: float arrays sized per output shape. 0 on success */
int zo_net_run(zo_net *n, const float *input, float *const *outputs);
const char *zo_net_error(void);
/* libjpeg-turbo's pixel stages (jpeg.c): quantised coefficients -> RGBA8 */
int zo_jpeg_pixels(const int16_t *coef, uint32_t width, uint32_t height, uint32_t ncomp,
                   uint32_t h_samp, uint32_t v_samp, const uint32_t *bw, const uint32_t *bh,
                   const uint32_t *qsel, const uint16_t *quant, uint8_t *rgba);
size_t zo_net_tensor(const zo_net *n, const char *name, double *out, size_t cap, int64_t *shape,
                     size_t *rank);

#ifdef __cplusplus
}
#endif
#endif
