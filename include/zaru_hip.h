/*
 * zaru_hip.h -- C ABI of the MI355X (gfx950) CNN runner for Zaru's detection/landmark path.
 *
 * This is the drop-in boundary of SURVEY.md §8b: a fourth `Session` variant behind
 * `ZARU_ONNX_BACKEND=hip`.  Every entry point names the reference interface it replaces
 * (paths relative to placrosse/Zaru).  Conventions:
 *   - every call returns ZR_OK (0) or a negative error class and sets a thread-local message
 *     readable with zr_last_error() (reference: anyhow::Error from Loader::load /
 *     NeuralNetwork::estimate, crates/zaru/src/nn/mod.rs:259, 450);
 *   - no C++ exception or abort crosses this boundary: every entry point catches at the
 *     boundary (host out-of-memory -> ZR_ERR_DEVICE, anything else -> ZR_ERR_INTERNAL);
 *   - a session is safe to use from several threads at once (NeuralNetwork is Clone + Send +
 *     Sync and HandTracker workers call estimate(&self) concurrently,
 *     crates/zaru/src/hand/tracking.rs:165-181);
 *   - tensors are f32, row-major, batch in dim 0 replacing the reference's fixed 1
 *     (crates/zaru/src/nn/tensor.rs:19-34).
 * The host side of the reference (Detector, Estimator, LandmarkTracker, ...) stays as is;
 * INTEGRATION.md shows the Rust binding.
 */
#ifndef ZARU_HIP_H
#define ZARU_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZR_OK 0
#define ZR_ERR_INVALID_ARGUMENT (-1)
#define ZR_ERR_MODEL (-2)       /* malformed ONNX, or an operator/pattern with no HIP lowering */
#define ZR_ERR_DEVICE (-3)      /* HIP runtime failure (no GPU, out of memory, ...) */
#define ZR_ERR_SHAPE (-4)       /* tensor count or shape mismatch */
#define ZR_ERR_INTERNAL (-5)    /* unexpected internal failure (caught at the boundary) */

typedef struct zr_session zr_session; /* = Arc<NeuralNetworkImpl> (crates/zaru/src/nn/mod.rs:369-375) */

/* A view of an image: RotatedRect in root-image coordinates (crates/zaru/src/image/mod.rs:
 * 188-192), stored as the reference stores it: centre, size, clockwise radians. */
typedef struct {
    float cx, cy, w, h, rad;
} zr_view;

/* An RGBA8 frame (crates/zaru/src/image/mod.rs:47-51), r in the lowest byte. */
typedef struct {
    const uint8_t *rgba;
    uint32_t width, height;
    uint64_t row_stride; /* bytes */
} zr_frame;

/* NeuralNetwork::from_onnx(bytes)[.with_output_selection(sel)].load()
 * (crates/zaru/src/nn/mod.rs:411, 247, 259-362).  `onnx` is only borrowed; weights are
 * copied to the device.  n_sel == 0 selects every graph output. */
int zr_session_create(const uint8_t *onnx, size_t len, const uint32_t *out_sel, size_t n_sel,
                      int device, zr_session **out);

/* Last Arc drop. */
void zr_session_destroy(zr_session *s);

/* num_inputs() / num_outputs() (crates/zaru/src/nn/mod.rs:416-423) */
int zr_session_num_io(const zr_session *s, int is_output, size_t *n);

/* inputs() / outputs() descriptors (crates/zaru/src/nn/mod.rs:428-443).  `shape` receives up
 * to 8 dims with the batch dim = 1; `name` stays valid for the session's lifetime. */
int zr_session_io(const zr_session *s, int is_output, size_t idx, const char **name,
                  int64_t *shape, size_t *rank);

/* NeuralNetwork::estimate (crates/zaru/src/nn/mod.rs:450-538), batched: `inputs[0]` is a
 * host [batch,C,H,W] tensor, `outputs[i]` host buffers sized batch * per-image numel of
 * output i.  Synchronous: returns with the outputs written. */
int zr_session_run(zr_session *s, size_t batch, const float *const *inputs, size_t n_in,
                   float *const *outputs, size_t n_out);

/* Device-resident variant: `d_input` already in HBM ([batch,C,H,W]); outputs are device
 * buffers; work is enqueued on `hip_stream` (NULL = default stream) and the call returns
 * without waiting. */
int zr_session_run_async(zr_session *s, size_t batch, const float *d_input, float *const *d_outputs,
                         size_t n_out, void *hip_stream);

/* Cnn::estimate (crates/zaru/src/nn/mod.rs:118-126) batched over views of one host RGBA8
 * image: the image->tensor map (nn/mod.rs:54-73, ColorMapper::linear(lo..=hi)) runs on the
 * GPU, bit-exact, and feeds the network directly.  Host outputs, synchronous. */
int zr_cnn_estimate_views(zr_session *s, const uint8_t *rgba, uint32_t w, uint32_t h,
                          size_t row_stride, const zr_view *views, size_t n_views, float lo,
                          float hi, float *const *outputs);

/* Device-resident variant over several frames already in HBM: view v samples frame
 * view_frame[v].  `frames` is a host array whose rgba pointers are device pointers. */
int zr_cnn_estimate_views_async(zr_session *s, const zr_frame *frames, size_t n_frames,
                                const zr_view *views, const uint32_t *view_frame, size_t n_views,
                                float lo, float hi, float *const *d_outputs, void *hip_stream);

/* The preprocessing alone (K1), into `d_out` as [n_views,3,oh,ow] f32 (device). */
int zr_preprocess_views_async(const zr_frame *frames, size_t n_frames, const zr_view *views,
                              const uint32_t *view_frame, size_t n_views, uint32_t ow,
                              uint32_t oh, float lo, float hi, float *d_out, void *hip_stream);

/* Detector candidate compaction (device): per image, every anchor whose raw logit is
 * >= logit_min is written as {anchor index bits, logit, params[0..D)} into d_rec
 * ([n][cap][2+D]) and counted in d_count[n] (may exceed cap).  The exact sigmoid /
 * threshold / decode / NMS then runs on the host (face/detection.rs:96-157, nms.rs:59-145). */
int zr_detection_candidates_async(const float *d_logits, const float *d_boxes, uint32_t n,
                                  uint32_t anchors, uint32_t params, float logit_min,
                                  uint32_t cap, int32_t *d_count, float *d_rec, void *hip_stream);

/* ---- Detector::detect_impl after inference, on the device ----------------------------------
 * extract_outputs + NMS + map into frame pixels (crates/zaru/src/detection.rs:231-267,
 * face/detection.rs:96-157, hand/detection.rs:108-179, detection/nms.rs:59-145), one wave per
 * frame, bit-exact with the host restatement (glibc expf / atan2f restated on the device; NMS ties
 * in anchor order).  Per frame: d_count[f] = detections after NMS (exact, whatever dcap is), the
 * first dcap of them in d_dets [n][dcap][20] = {conf, angle, cx, cy, w, h, 7 x (kx, ky)} (frame
 * px, keypoints past the network's zero; dcap = anchors keeps every detection), and when d_records
 * is not NULL the all-gather record [n][2 + 20 rmax] = {frame id first_id + f * id_stride (u32
 * bits), count (u32 bits), the first rmax detections, zeros}.  d_ties (may be NULL):
 * [n][2] = {candidates (conf >= thresh), candidates whose confidence another candidate shares};
 * ties are ordered by anchor index, which is Rust's sort_unstable order only up to 20
 * candidates (nms.rs:66), so a frame with more than 20 candidates and a tie is not pinned by the
 * reference. */
typedef struct {
    int face;               /* 1 BlazeFace (angle: eye line vs +X), 0 BlazePalm (wrist -> MCP vs +Y) */
    int anchors, params, keypoints;  /* A, values per anchor (16 / 18), keypoints (6 / 7) */
    int in_w, in_h;         /* detector input */
    float thresh, iou;      /* Detector threshold (0.5), NMS IoU threshold (0.3) */
    int mode;               /* SuppressionMode (nms.rs:154-163): 0 Average (default), 1 Remove */
} zr_detpost_cfg;
int zr_detect_post_async(const float *d_logits, const float *d_boxes, const float *d_anchors,
                         const float *d_letterbox, size_t n, const zr_detpost_cfg *cfg,
                         int32_t *d_count, float *d_dets, size_t dcap, float *d_records, size_t rmax,
                         uint32_t first_id, uint32_t id_stride, int32_t *d_ties, void *hip_stream);

/* The same over a device-resident frame subset: frame f < *d_nframes (f < n) is the logits /
 * boxes row f, and its count / detections / tie counts / letterbox go to slot d_map[f]; slots of
 * other frames are left as they are (the device HandTracker's palm detection over the streams
 * due for it, hand/tracking.rs:210-218). */
int zr_detect_post_mapped_async(const float *d_logits, const float *d_boxes, const float *d_anchors,
                                const float *d_letterbox, size_t n, const int32_t *d_map, const int32_t *d_nframes,
                                const zr_detpost_cfg *cfg, int32_t *d_count, float *d_dets, size_t dcap,
                                int32_t *d_ties, void *hip_stream);

/* ---- the one collective of the multi-GPU path ------------------------------
 * A communicator over the node's ranks (one process per GPU) for the all-gather of the detection
 * records (RCCL over xGMI).  The reference has no multi-device code; this is the build's own
 * exchange, issued on a HIP stream so it overlaps the next step's kernels.  zr_comm_unique_id
 * runs on one rank; its 128 bytes reach the others by any side channel (the benchmark uses the
 * gloo control group).  zr_comm_create blocks until every rank joined. */
typedef struct zr_comm zr_comm;
int zr_comm_unique_id(uint8_t id[128]);
int zr_comm_create(const uint8_t id[128], int nranks, int rank, int device, zr_comm **out);
void zr_comm_destroy(zr_comm *c);
/* the communicator's rank count (what an all-gather writes nranks * bytes for) */
int zr_comm_size(const zr_comm *c, int *nranks);
/* recv (nranks * bytes, rank-major) <- every rank's send (bytes), enqueued on hip_stream (not NULL:
 * the legacy default stream is refused with ZR_ERR_INVALID_ARGUMENT).
 * Every zr_comm_* call first takes the thread's pending HIP error (hipGetLastError) and, if one
 * is set, returns ZR_ERR_DEVICE naming it without calling RCCL; after an RCCL call it clears
 * only the status RCCL itself left. */
int zr_comm_all_gather_async(zr_comm *c, const void *d_send, void *d_recv, size_t bytes, void *hip_stream);

/* ---- LandmarkTracker state on the device ------------------------------
 * A video loop of LandmarkTracker::track (crates/zaru/src/landmark.rs:463-501) over n streams
 * without a host round trip per frame: the tracker state lives in HBM, the landmark network
 * samples views that the previous update wrote (zr_cnn_estimate_device_views_async), and
 * zr_track_update_async consumes that estimate: loss check, map-out, angle, transform_out,
 * RotatedRect::bounding, grow_rel(padding), and the next view.  ROI i is evaluated on frame i
 * of each step's frame array.  Geometry follows the host restatement operation for operation
 * (f32, no contraction) with glibc 2.35's own sinf/cosf/expf/atan2f restated on the device
 * (verified over every f32 input), so the update and the view table are bit-identical to the
 * host path given the same network outputs. */
typedef struct {
    float roi[5];       /* RotatedRect {cx, cy, w, h, rad} tracked next (LandmarkTracker::roi) */
    float view_rect[5]; /* roi.grow_to_fit_aspect(aspect) of the pending estimate */
    float local[3];     /* Estimator map-out rect of that estimate: x, y, w */
    uint32_t active;    /* 0 once lost (roi = None) */
    uint32_t frame_w, frame_h;
    uint32_t tracked;   /* last step: 1 tracked, 0 lost / inactive */
    float confidence;   /* last step's Confidence::confidence */
    float updated[5];   /* last step's updated_roi */
} zr_track_state;

/* One view of the preprocessing's view table (the sampling parameters of a zr_view). */
typedef struct {
    float half_w, half_h, tl_x, tl_y, view_w, view_h, cos_r, sin_r;
    uint32_t frame, pad;
} zr_view_desc;

typedef struct {
    int kind;           /* 0 FaceMesh V1/V2 (face_flag = sigmoid(out1), eyes 33->263 vs +X),
                           1 hand (presence = out1, wrist 0 -> MCP 9 vs +Y),
                           2 no confidence / angle (EyeNetwork), 3 as 2 with relative (x, y)
                           pairs (68-point networks) */
    int num_landmarks;
    int in_w, in_h;     /* network input */
    int aspect_w, aspect_h;
    float loss_thresh, padding;
    int rois_per_frame; /* ROI i samples frame i / rois_per_frame (0 = 1) */
} zr_track_cfg;

/* Derive every state's first view from state.roi (LandmarkTracker::set_roi); no estimate. */
int zr_track_seed_async(zr_track_state *d_state, size_t n, const zr_track_cfg *cfg,
                        zr_view_desc *d_views, void *hip_stream);
/* Consume the estimate made on d_views (landmark output 0 with lm_stride floats per image, and
 * output 1 with flag_stride floats per image for kinds 0/1 -- the flag -- and kind 2 -- the 5
 * iris points, which come first), update the states, write frame-space landmarks to d_lm_out
 * (n x L x 3, may be NULL; rows of ROIs not tracked this step are NaN) and the next views.
 * lm_stride must cover what the kind's extract reads (3L; 2L for kind 3; 3(L-5) for kind 2). */
int zr_track_update_async(zr_track_state *d_state, size_t n, const zr_track_cfg *cfg,
                          const float *d_landmarks, size_t lm_stride, const float *d_flag,
                          size_t flag_stride, float *d_lm_out, zr_view_desc *d_views, void *hip_stream);
/* The sampling parameters the preprocessing derives from each zr_view: glibc cosf/sinf of the
 * angle (rect.rs:135-137,417-423), so a caller can build or check a device view table.  A view
 * whose frame index is past the call's frame table samples Color::NONE everywhere. */
int zr_view_describe(const zr_view *views, size_t n, uint32_t frame, zr_view_desc *out);
/* Seed trackers from device detections (the pipeline's ROI step, pipeline.cpp /
 * examples/facemesh.rs:49-54, hand/tracking.rs:136-159): ROI slot k of frame f (i = f * R + k,
 * R = cfg->rois_per_frame) is RotatedRect(det_k.rect[.grow_rel(roi_grow)], roi_use_angle ?
 * det_k.angle : 0) for the frame's first R detections (NMS order), else -- when the frame has no
 * detection -- its forced ROI k (d_forced [n][R][5], d_nforced [n]; both may be NULL), else the
 * slot is idle (active = 0).  Writes the states, optionally a copy of them (d_seed_copy, may be
 * NULL: the update rewrites the states), and their first views (frame f). */
int zr_track_seed_detections_async(const int32_t *d_count, const float *d_dets, size_t dcap,
                                   const float *d_forced, const int32_t *d_nforced,
                                   const uint32_t *d_frame_size, size_t n, const zr_track_cfg *cfg,
                                   float roi_grow, int roi_use_angle, zr_track_state *d_state,
                                   zr_track_state *d_seed_copy, zr_view_desc *d_views, void *hip_stream);
/* HandTracker::track's bookkeeping (crates/zaru/src/hand/tracking.rs:115-219) for n video
 * streams with their hands in HBM: stream s owns the hand slots [s * H, s * H + H) of d_state /
 * d_ids / d_hroi (the hand's ROI, {cx, cy, w, h, rad}).  Called after zr_track_update_async has
 * consumed the previous step's hand landmark estimate: drops lost hands (tracking.rs:116-127);
 * when d_det_pending[s], filters stream s's palm detections (d_count / d_dets as
 * zr_detect_post_async writes them, frame px) against the hands' ROIs (136-156) and starts a hand
 * for each kept one, ROI = RotatedRect(det.rect.grow_rel(palm_grow), det.angle) (158-194, u64 HandIds
 * from d_next_id; a kept detection finding no free slot of the H is counted in d_dropped[s], may be
 * NULL -- the reference's Vec grows instead); removes hands whose ROI overlaps an earlier
 * hand's with the reference's swap_remove sweep (196-208); and sets d_det_pending[s] when no hand
 * is left or now_ms reached d_next_det[s] (advanced by interval_ms) -- this step's palm detection
 * then counts at the next call (210-218).  Writes every slot's view (idle slots: an empty view),
 * the hand counts and, per slot, the slot the hand had before the call (d_src, -1: new), so the
 * caller can pair hands with the landmarks the update wrote.  Geometry as the host restatement
 * (f32, no contraction): the same decisions as the host HandTracker given the same inputs. */
typedef struct {
    int slots;              /* H: hand slots per stream */
    float iou_thresh;       /* tracking.rs:38 (0.3) */
    float palm_grow;        /* tracking.rs:136 (1.5) */
    double interval_ms;     /* redetection interval, tracking.rs:41 (300 ms) */
    int aspect_w, aspect_h; /* the hand landmark network's aspect ratio */
} zr_hand_cfg;
int zr_hand_manage_async(zr_track_state *d_state, uint64_t *d_ids, float *d_hroi, int32_t *d_src,
                         int32_t *d_nhands, uint64_t *d_next_id, double *d_next_det, int32_t *d_det_pending,
                         const int32_t *d_count, const float *d_dets, size_t dcap,
                         const uint32_t *d_frame_size, size_t n, const zr_hand_cfg *cfg, double now_ms,
                         int init_clock, zr_view_desc *d_views, int32_t *d_dropped, void *hip_stream);
/* Cnn::estimate (nn/mod.rs:118-126) with a device-resident view table (frames: host array). */
int zr_cnn_estimate_device_views_async(zr_session *s, const zr_frame *frames, size_t n_frames,
                                       const zr_view_desc *d_views, size_t n_views, float lo,
                                       float hi, float *const *d_outputs, void *hip_stream);
/* The same when only the first *d_count (device int, <= n_views) views are needed: the launches
 * skip the work of images at and past it, whose outputs are then undefined.  The count is read
 * by the kernels, so no host decision sits between the step that writes it and this one. */
int zr_cnn_estimate_device_views_count_async(zr_session *s, const zr_frame *frames, size_t n_frames,
                                             const zr_view_desc *d_views, size_t n_views, const int32_t *d_count,
                                             float lo, float hi, float *const *d_outputs, void *hip_stream);
/* The streams zr_hand_manage_async asked to detect on (d_det_pending[s] != 0) compacted in stream
 * order: d_due[k] = s and d_due_views[k] = *view_template with its frame index set to s, for
 * k < *d_ndue (one workgroup, on the stream; hand/tracking.rs:210-218's schedule on the device).
 * d_total (may be NULL): *d_total += *d_ndue, a running count of the detections run. */
int zr_due_compact_async(const int32_t *d_det_pending, size_t n, const zr_view_desc *view_template, int32_t *d_due,
                         int32_t *d_ndue, zr_view_desc *d_due_views, uint64_t *d_total, void *hip_stream);
/* The face video loop of the reference's demo (crates/zaru/examples/facemesh.rs:35-56: track, and
 * on loss detect on the same frame and re-seed the tracker from the most confident detection) on
 * the device, in two calls around a mapped detection (zr_cnn_estimate_device_views_count_async +
 * zr_detect_post_mapped_async).  zr_track_lost_compact_async: as zr_due_compact_async, with the
 * streams whose state holds no RoI (active == 0: lost by this step's zr_track_update_async or
 * never seeded, LandmarkTracker::roi() == None) as the due streams.  zr_track_reseed_best_async:
 * every stream without RoI whose detection found a face (d_count / d_dets as the mapped
 * post-processing wrote its slot) gets RoI = RotatedRect(best.rect, 0) for best =
 * max_by_key(TotalF32(confidence)) (the last of equal maxima; LandmarkTracker::set_roi,
 * landmark.rs:434-436), active = 1, and its next view in d_views; other streams are untouched.
 * d_reseeded (may be NULL): += the streams re-seeded. */
int zr_track_lost_compact_async(const zr_track_state *d_state, size_t n, const zr_view_desc *view_template,
                                int32_t *d_due, int32_t *d_ndue, zr_view_desc *d_due_views, uint64_t *d_total,
                                void *hip_stream);
int zr_track_reseed_best_async(const int32_t *d_count, const float *d_dets, size_t dcap, const uint32_t *d_frame_size,
                               size_t n, const zr_track_cfg *cfg, zr_track_state *d_state, zr_view_desc *d_views,
                               uint64_t *d_reseeded, void *hip_stream);

/* ---- JPEG frame source --------------------------------------------------
 * Replaces decode_jpeg (crates/zaru-image/src/jpeg.rs:107-182) for its libjpeg-turbo backend
 * (turbojpeg 0.5.3: accurate integer IDCT, fancy upsampling, TJPF_RGBA output): the frame is
 * decoded straight into an RGBA8 device buffer, byte-identical to libjpeg-turbo.  Streams with
 * restart intervals (DRI, >= 8 intervals, each 64-interval range within a workgroup's LDS) are
 * Huffman-decoded on the device, one lane per interval; the others on the calling thread.
 * Dequantisation, IDCT, upsampling and colour conversion are enqueued on `hip_stream`.  Baseline
 * 8-bit JPEG, 1 or 3 components, 4:4:4 / 4:2:2 / 4:2:0, one interleaved scan, restart markers.
 * A decoder may be reused; calls on one decoder are serialised (its staging is reused once the
 * previous upload completed). */
typedef struct zr_jpeg_decoder zr_jpeg_decoder;
int zr_jpeg_decoder_create(int device, zr_jpeg_decoder **out);
void zr_jpeg_decoder_destroy(zr_jpeg_decoder *d);
int zr_jpeg_info(const uint8_t *jpeg, size_t len, uint32_t *width, uint32_t *height);
int zr_jpeg_decode_async(zr_jpeg_decoder *d, const uint8_t *jpeg, size_t len, uint8_t *d_rgba,
                         size_t row_stride, void *hip_stream);
/* n frames (<= 4096) in one call: frame i from jpegs[i] (lens[i] bytes) into d_rgba[i].  Every
 * frame is parsed before anything is enqueued (an error names the frame); the device-decodable
 * frames share one set of Huffman launches, so a multi-camera ingest fills the GPU with one call
 * instead of one small launch per frame.  zr_jpeg_decode_async is the n = 1 case.  Huffman
 * decoding runs on the device for streams with restart intervals (one lane per interval) and
 * for streams without them (self-synchronising decoding, one lane per 4096-bit segment, round 4)
 * unless their scan averages > 600 bits per block (near-lossless noise: those sync too slowly)
 * or ZARU_JPEG_SYNC=0; the rest, and every frame under ZARU_JPEG_HOST_ENTROPY=1, on the host. */
int zr_jpeg_decode_batch_async(zr_jpeg_decoder *d, size_t n, const uint8_t *const *jpegs, const size_t *lens,
                               uint8_t *const *d_rgba, const size_t *row_strides, void *hip_stream);
/* Host-only half (no GPU): the frame's block layout and, when `coef` is given, its quantised
 * coefficients ([component][by][bx][64], natural order; cap_blocks >= layout->total_blocks). */
typedef struct {
    uint32_t width, height, ncomp, h_samp, v_samp, total_blocks;
    uint32_t bw[3], bh[3], qsel[3];
    uint16_t quant[4][64]; /* natural order */
} zr_jpeg_layout;
/* Frames decoded so far whose Huffman stage ran on the device and on the host; *corrupt (may be
 * NULL; waits for the last call) is 1 when a frame of the LAST call held an invalid Huffman code or
 * AC index.  Error contract: a frame decoded on the host with corrupt data fails the call
 * (ZR_ERR_INVALID_ARGUMENT, frame named); on the device it cannot fail the already-returned call,
 * so the block holding the bad code and the rest of its interval (a stream without restart
 * intervals: every block from the bad one to the end of the frame) decode as all-zero blocks
 * (libjpeg-turbo's insufficient-data behaviour) and the frame's flag is set --
 * zr_jpeg_frame_errors names the frames.  A valid stream without restart intervals whose device
 * sync passes do not converge is finished by a serial decode on the device: never flagged. */
int zr_jpeg_decoder_status(zr_jpeg_decoder *d, uint64_t *gpu_entropy, uint64_t *host_entropy, int *corrupt);
/* per frame of the last call: 1 = corrupt entropy data (waits for that call); *n = its frame count */
int zr_jpeg_frame_errors(zr_jpeg_decoder *d, int32_t *flags, size_t cap, size_t *n);
int zr_jpeg_coefficients(const uint8_t *jpeg, size_t len, int16_t *coef, size_t cap_blocks,
                         zr_jpeg_layout *layout);

/* Roofline accounting of the compiled plan: algorithmic bytes and FLOPs per image, number
 * of kernel launches per run. */
int zr_session_stats(const zr_session *s, double *bytes_per_image, double *flops_per_image,
                     size_t *launches);

/* Per-launch profiling with HIP events recorded on the launching stream around every kernel
 * of this session (preprocessing included).  zr_profile_read returns and clears the
 * aggregate, one line per kernel symbol: "<kernel> <launches> <total_ms> <bytes> <flops>"
 * where bytes/flops are the algorithmic traffic/work of those launches. */
int zr_profile_enable(zr_session *s, int enable);
int zr_profile_read(zr_session *s, char *buf, size_t cap, size_t *needed);

/* Compile a model without a GPU and describe the fused launch plan as text, one launch per
 * line (for tests and diagnostics).  Writes at most `cap` bytes incl. the NUL terminator;
 * `*needed` receives the full length + 1. */
int zr_plan_describe(const uint8_t *onnx, size_t len, const uint32_t *out_sel, size_t n_sel,
                     char *buf, size_t cap, size_t *needed);

/* Test hook: evaluate the device restatement of glibc's sinf (fn 0), cosf (1), expf (2),
 * atanf (3) or atan2f(a, b) (4) on n device floats (kernels/glibc_math.h). */
int zr_debug_glibc_math(int fn, const float *d_a, const float *d_b, float *d_out, size_t n, void *hip_stream);

/* Thread-local text of the last error (anyhow::Error text). */
const char *zr_last_error(void);

/* Minimal device-memory helpers so host code needs no HIP headers. kind: 0 H2D, 1 D2H, 2 D2D */
int zr_device_count(int *n);
int zr_malloc(void **p, size_t bytes);
int zr_free(void *p);
int zr_host_alloc(void **p, size_t bytes); /* page-locked host memory (truly async copies) */
int zr_host_free(void *p);
int zr_memcpy_async(void *dst, const void *src, size_t bytes, int kind, void *hip_stream);
/* height rows of width bytes, row pitches dpitch / spitch */
int zr_memcpy2d_async(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height,
                      int kind, void *hip_stream);
int zr_stream_create(void **stream);
int zr_stream_destroy(void *stream);
int zr_stream_synchronize(void *stream);
int zr_event_create(void **event);
int zr_event_create_timing(void **event); /* an event zr_event_elapsed can read */
int zr_event_elapsed(float *ms, void *start, void *end);
int zr_stream_wait_event(void *stream, void *event);
int zr_event_destroy(void *event);
int zr_event_record(void *event, void *stream);
int zr_event_synchronize(void *event);
int zr_event_query(void *event); /* ZR_OK when complete, 1 while pending */

#ifdef __cplusplus
}
#endif
#endif /* ZARU_HIP_H */
