// zr_track.h -- device-resident LandmarkTracker state shared by the track
// kernels (kernels/track.hip) and the runtime (session.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zr_kernels.h"

namespace zr {

// One tracked ROI (LandmarkTracker, crates/zaru/src/landmark.rs:354-501) kept in HBM between
// frames: the RoI the next estimate samples, the view geometry that estimate used (for the
// map-out) and the last result.  Layout mirrored by zr_track_state in include/zaru_hip.h.
struct TrackState {
    float roi[5];          // RotatedRect (cx, cy, w, h, rad) tracked next
    float view_rect[5];    // roi.grow_to_fit_aspect(aspect) of the pending estimate (landmark.rs:465)
    float local[3];        // Estimator map-out rect of that estimate: x, y (top left), w (landmark.rs:320-345)
    uint32_t active;       // 0 once lost (the reference sets roi = None, landmark.rs:475)
    uint32_t frame_w, frame_h;
    uint32_t tracked;      // last step: 1 tracked, 0 lost (or inactive)
    float confidence;      // last step's Confidence::confidence
    float updated[5];      // last step's updated_roi (RotatedRect::bounding, landmark.rs:488-491)
};

struct TrackParams {
    TrackState *state;
    ViewDesc *views;       // out: the next estimate's sampling view per ROI (the preprocessing input)
    const float *lm;       // landmark output 0 of the last estimate: n x L x 3 (n x 2L for kind 3)
    const float *flag;     // output 1: n x flag_stride (face_flag logit / presence); null: kind 2/3
    float *lm_out;         // out: frame-space landmarks, n x L x 3 (may be null)
    int n, L, flag_stride;
    int lm_stride;         // floats per image of output 0
    int kind;              // 0 FaceMesh (sigmoid flag, eyes 33->263 vs +X), 1 hand (presence, 0->9 vs +Y),
                           // 2 no confidence / no angle (eye), 3 as 2 with (x, y) relative pairs (68-point)
    int in_w, in_h;        // network input (map-out scale, kind 3 coordinate scale)
    int asp_w, asp_h;      // network aspect ratio, reduced
    float loss_thresh, padding;
    int seed;              // 1: only derive views from state.roi (no estimate to consume)
    int rpf;               // ROIs per frame: ROI i samples frame i / rpf
};

const char *launch_track(const TrackParams &p, hipStream_t s);

// Detector::detect_impl after inference (detpost.hip): extract, weighted NMS, map to frame px.
struct DetPostParams {
    const float *logits;    // [N][A] raw classificator logits
    const float *boxes;     // [N][A][D] raw regressors
    const float *anchors;   // [A][2] anchor centres (ssd.rs:96-119)
    const float *letterbox; // [N][4] the letterbox Rect (cx, cy, w, h) each frame was sampled with
    int N, A, D, nkp;       // frames, anchors, params per anchor, keypoints
    int face;               // 1: angle = eye line vs +X (BlazeFace); 0: wrist -> MCP vs +Y (palm)
    int in_w, in_h;         // detector input
    float thresh, iou;
    int mode;               // SuppressionMode: 0 Average (nms.rs:77-139), 1 Remove (nms.rs:70-76)
    int *count;             // [N] detections after NMS
    float *dets;            // [N][dcap][20] {conf, angle, cx, cy, w, h, 7 x (kx, ky)}, NMS order
    int dcap;
    float *rec;             // [N][2 + 20 rmax] all-gather records (may be null)
    int rmax;
    uint32_t first_id, id_stride;
    int *ties;              // [N][2] {candidates, candidates sharing their confidence} (may be null)
    // (both may be null) frame f < *nact writes slot map[f] of count / dets / rec / ties and uses
    // letterbox[map[f]]; frames >= *nact do nothing (the device HandTracker's due streams)
    const int *map, *nact;
};
const char *launch_det_post(const DetPostParams &p, hipStream_t s);
size_t det_post_lds(int anchors);

// Tracker seeding from detections (track.hip): ROI slot k < R of frame f is detection k
// (grow_rel + angle as configured), else -- when the frame has none -- forced ROI k, else idle.
struct SeedParams {
    const int *count;        // [N] (det_post)
    const float *dets;       // [N][dcap][20]
    int dcap;
    const float *forced;     // [N][R][5] (cx, cy, w, h, rad); may be null
    const int *nforced;      // [N]; may be null
    const uint32_t *fsize;   // [N][2] frame width, height
    int N, R;
    float roi_grow;
    int roi_use_angle;
    int asp_w, asp_h;
    TrackState *state;       // [N * R] out
    TrackState *seed_copy;   // [N * R] out, may be null: the seeds again (the update rewrites state)
    ViewDesc *views;         // [N * R] out
};
const char *launch_seed(const SeedParams &p, hipStream_t s);
// HandTracker::track's bookkeeping (crates/zaru/src/hand/tracking.rs:115-219) per video stream,
// on the device (track.hip): stream s owns hand slots [s * H, s * H + H) in hand order.  After
// the landmark update of the previous step: drop lost hands (retain, 116-127), filter the palm
// detections the previous step produced against the hands' ROIs (136-156), start a hand for
// every kept one (158-194), remove hands whose ROI overlaps an earlier hand's (swap_remove sweep,
// 196-208), and decide whether this step's palm detection counts (210-218).
struct HandManageParams {
    TrackState *state;       // [S * H] hand slots (the track update's output)
    uint64_t *ids;           // [S * H] HandId (tracking.rs:227, u64)
    float *hroi;             // [S * H][5] the hand's ROI (tracking.rs: TrackedHand::roi)
    int32_t *src;            // [S * H] out: slot of the hand before this call (-1: new hand)
    int32_t *nhands;         // [S]
    uint64_t *next_id;       // [S]
    int32_t *dropped;        // [S] out: kept palm detections this call found no free hand slot for
    double *next_det;        // [S] redetection clock (ms)
    int32_t *det_pending;    // [S] in: count/dets hold this stream's detections; out: this step's counts
    const int32_t *count;    // [S] detections (det_post)
    const float *dets;       // [S][dcap][20]
    const uint32_t *fsize;   // [S][2]
    ViewDesc *views;         // [S * H] out: the views this step's landmark estimate samples
    int S, H, dcap;
    float iou, grow;
    double now, interval;
    int init_clock;          // 1: next_det = now first (the reference starts the clock at construction)
    int asp_w, asp_h;
};
const char *launch_hand_manage(const HandManageParams &p, hipStream_t s);
// The streams whose detection hand_manage requested (det_pending[s] != 0), or -- lost_of != null
// -- whose tracker state holds no RoI (active == 0), in stream order: due[k] = s for k < *ndue,
// and due_views[k] = the template view with frame = s (one workgroup).
const char *launch_due_compact(const int32_t *det_pending, const TrackState *lost_of, int S, const ViewDesc &tmpl,
                               int32_t *due, int32_t *ndue, ViewDesc *due_views, uint64_t *total, hipStream_t s);
// The face video loop's re-seeding (examples/facemesh.rs:45-54): a stream without RoI takes the
// bounding rect of its most confident detection (the last of equal maxima) as its RoI.
struct ReseedParams {
    const int *count;        // [N] detections of this frame's detection (det_post, mapped)
    const float *dets;       // [N][dcap][20]
    int dcap;
    const uint32_t *fsize;   // [N][2] frame width, height
    int N;
    int asp_w, asp_h;        // landmark network aspect ratio
    TrackState *state;       // [N] in / out
    ViewDesc *views;         // [N] out: the next estimate's view of a re-seeded stream
    uint64_t *reseeded;      // running count of re-seeded streams (may be null)
};
const char *launch_reseed(const ReseedParams &p, hipStream_t s);

// fn: 0 sinf, 1 cosf, 2 expf, 3 atanf, 4 atan2f(a, b) -- glibc_math.h on the device
const char *launch_glibc_math(int fn, const float *a, const float *b, float *out, int64_t n, hipStream_t s);

}  // namespace zr
