// pipeline.h -- batched detect -> track pipelines over frames resident in HBM.
//
// One `run` = the reference's per-frame call chain for a whole batch of frames:
//   Detector::detect (detection.rs:216-270) on every frame, then for each detection a
//   one-shot LandmarkTracker seeded from it (examples/facemesh.rs:49-54 for faces,
//   hand/tracking.rs:136-194 for hands) -> Estimator::estimate (landmark.rs:314-348) ->
//   tracker update (landmark.rs:463-501).
// The GPU runs preprocessing + both networks as two batched launches sequences (all frames'
// letterbox views, then all ROIs); the host runs the bit-exact decode/NMS and the landmark
// mapping on a thread pool.  Frames with no detection can be given explicit ROIs
// ("forced-ROI mode") so that synthetic frames exercise the full path.
#pragma once
#include <atomic>
#include <chrono>
#include <functional>
#include <memory>
#include <thread>
#include <vector>

#include "detection.h"
#include "device_tracker.h"
#include "landmark.h"

namespace zh {

class ThreadPool {
  public:
    explicit ThreadPool(int n);
    ~ThreadPool();
    void parallel_for(size_t n, const std::function<void(size_t)> &fn);
    int size() const { return (int)workers_.size() + 1; }

  private:
    struct Impl;
    std::unique_ptr<Impl> impl_;
    std::vector<std::thread> workers_;
};

struct RoiResult {
    uint32_t frame = 0;
    bool from_detection = false;
    bool tracked = false;  // false: confidence below the loss threshold
    float confidence = 0.f;  // the estimate's Confidence (face_flag / hand presence), always set
    RotatedRect roi;       // ROI the tracker was seeded with
    // tracked: landmarks in frame coordinates, view/updated ROI.  Lost: the reference returns
    // None (landmark.rs:468-477), so only view_rect is set and the estimate stays empty.
    TrackingResult result;
    RotatedRect next_roi;  // valid when tracked
};

// Mirrors Detector::timers / Estimator::timers (detection.rs:273-275, landmark.rs:289-291).
// Host mode: the host's waits for each GPU stage and its own decode / map work.  Device mode:
// HIP-event spans of each stage on the sub-batch streams, summed over the sub-batches (they run
// concurrently, so the sum may exceed the wall time): detector inference, decode + NMS + map + ROI
// seeding, landmark inference, tracker update; host_wait_ms is the host's wait for the steps.
struct StageTimes {
    double detect_gpu_ms = 0, decode_nms_ms = 0, landmark_gpu_ms = 0, map_ms = 0, total_ms = 0;
    double host_wait_ms = 0;
    size_t frames = 0, detections = 0, rois = 0, tracked = 0;
    // detections past PipelineConfig::det_cap (device mode; 0 with the default cap, which keeps
    // the detector's whole output)
    size_t dropped_detections = 0;
    // NMS candidates (conf >= threshold), those sharing their exact confidence with another, and
    // frames with > 20 candidates and a tie: the reference's sort_unstable order is not pinned
    // there (nms.rs:66), this build's is anchor order
    size_t nms_candidates = 0, nms_tied = 0, nms_unpinned_frames = 0;
};

struct PipelineConfig {
    DetectorNetwork detector = DetectorNetwork::short_range_face();
    LandmarkNetwork landmarker = LandmarkNetwork::face_mesh_v1();
    float det_threshold = Detector::DEFAULT_THRESHOLD;
    float nms_iou = NonMaxSuppression::DEFAULT_IOU_THRESH;
    SuppressionMode nms_mode = SuppressionMode::Average;  // Detector::nms_mut().set_mode
    // ROI from a detection: RotatedRect(det.rect.grow_rel(roi_grow), use_det_angle ? angle : 0)
    float roi_grow = 0.f;
    bool roi_use_angle = false;
    float roi_padding = LandmarkTracker::DEFAULT_ROI_PADDING;
    float loss_threshold = LandmarkTracker::DEFAULT_LOSS_THRESHOLD;
    uint32_t max_rois_per_frame = 8;
    uint32_t candidate_cap = 64;  // device compaction slots per frame (overflow -> full copy)
    // the batch runs as this many sub-batches on their own streams, software-pipelined so
    // that the host decode / mapping of one overlaps the GPU work of the next
    uint32_t sub_batches = 2;
    // give each sub-batch its own HIP stream (kernels of different sub-batches may then run
    // concurrently on the GPU); false = one stream, kernels strictly back to back
    bool stream_per_sub_batch = true;
    // decode + NMS + map, the ROI seeding and the tracker update on the device
    // (zr_detect_post_async -> zr_track_seed_detections_async -> landmarks ->
    // zr_track_update_async, one stream per sub-batch, no host step in between); false = the
    // host restatement (decode/NMS/map and the tracker update on the thread pool).  Both give
    // the same bits.  det_cap: detections kept per frame on the device; 0 = the detector's anchor
    // count, the most NMS can return, so nothing is ever dropped (the reference's Detections is a
    // Vec, detection.rs:44-111).  A smaller cap counts what it drops in StageTimes.
    bool device_post = true;
    uint32_t det_cap = 0;
    static PipelineConfig face();  // BlazeFace -> FaceMesh V1 (config 3)
    static PipelineConfig hand();  // BlazePalm lite -> hand landmark lite (config 4)
};

class DetectTrackPipeline {
  public:
    DetectTrackPipeline(PipelineConfig cfg, int device = 0, int threads = 8);
    ~DetectTrackPipeline();

    // frames: device-resident RGBA8.  forced[f]: ROIs to track on frame f when it has no
    // detection (may be empty).  Synchronous; results valid until the next run.
    void run(const std::vector<Image> &frames, const std::vector<std::vector<RotatedRect>> &forced);

    const std::vector<std::vector<Detection>> &detections() const {
        materialize();
        return dets_;
    }
    const std::vector<RoiResult> &rois() const {
        materialize();
        return rois_;
    }
    const StageTimes &times() const { return times_; }
    const PipelineConfig &config() const { return cfg_; }
    double detector_bytes_per_image() const;
    double landmarker_bytes_per_image() const;
    double detector_flops_per_image() const;
    double landmarker_flops_per_image() const;
    void *stream() const { return stream_; }
    // per-launch HIP-event profiling of both networks' sessions (zr_profile_*)
    void profile(bool on);
    std::string profile_read();  // "<net>/<kernel> <launches> <total_ms> <bytes> <flops>" lines

    // keep a frame set (and its forced ROIs) resident in the pipeline, so repeated runs over
    // the same device frames pay no per-call argument conversion
    void set_frames(std::vector<Image> frames, std::vector<std::vector<RotatedRect>> forced);
    void run_frames() { run(frames_, forced_); }
    // `steps` consecutive runs over the resident frames, software-pipelined across run
    // boundaries: the next run's detections are enqueued behind this run's landmark launches,
    // before this run's landmark mapping, so the GPU never waits for the host between runs.
    // Results are the last run's; times() sums all runs.
    void run_frames_repeated(int steps);
    // The same, one step at a time, so a caller can act between steps (the multi-GPU
    // all-gather of each step's detections): begin_steps() enqueues the first detections,
    // each step(more) finishes one run over the resident frames -- with more = true the next
    // run's detections are enqueued before this run's landmark mapping -- and leaves its
    // results readable until the next step.  Every begun sequence ends with step(false).
    void begin_steps();
    void step(bool more);

    // every step's per-frame detection records ([B][2 + 20 rmax] f32: frame id
    // first_id + f * id_stride, count, the first rmax detections) written on the device by the
    // post-processing itself, and -- with a communicator -- all-gathered over the node's ranks on
    // the pipeline's own stream, overlapping the next step.  No host copy on that path.
    void enable_records(uint32_t rmax, uint32_t first_id, uint32_t id_stride, zr_comm *comm = nullptr,
                        int world = 1);
    uint32_t record_width() const { return 2 + 20 * rec_rmax_; }
    // the last finished step's records of this rank (host copy, waits for them) ...
    std::vector<float> records();
    // ... and the gathered records of every rank ([world][B][W], needs a communicator)
    std::vector<float> gathered();

  private:
    // one software-pipeline slot: a contiguous range of frames with its own stream/buffers
    struct Slot {
        size_t f0 = 0, nf = 0;
        void *stream = nullptr;
        void *ev_det = nullptr, *ev_lm = nullptr;  // stage-1 / stage-3 outputs on the host
        // device mode: timing events around the stages (detector, post + seed, landmarks,
        // update) and the event after this step's records were written
        void *ev_t[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
        void *ev_rec = nullptr;
        bool timed = false;
        DeviceArray<float> d_boxes, d_logits, d_rec, d_lm[4];
        DeviceArray<int32_t> d_count;
        PinnedArray<float> h_rec, h_lm[4];
        PinnedArray<int32_t> h_count;
        std::vector<zr_frame> zf;
        std::vector<Rect> letterbox, local_rect;
        std::vector<zr_view> rv;
        std::vector<uint32_t> rf;
        size_t roi0 = 0, nroi = 0;
        // device post-processing (PipelineConfig::device_post): per-frame inputs (uploaded once
        // per frame set) ...
        DeviceArray<float> d_lbox, d_forced;
        DeviceArray<uint32_t> d_fsize;
        DeviceArray<int32_t> d_nforced;
        DeviceArray<zr_view_desc> d_views;
        PinnedArray<float> h_lbox, h_forced;
        PinnedArray<uint32_t> h_fsize;
        PinnedArray<int32_t> h_nforced;
        bool inputs_ok = false;
        // ... and two result sets on the device: a step writes one while the last finished
        // step's stays readable.  Only the summary (tracker states, seeds, detection counts: one
        // copy) comes to the host each step; detections and landmarks on demand (materialize)
        struct Results {
            DeviceArray<uint8_t> sum;  // [state: nv][seed: nv] zr_track_state, [count: n] int32
            DeviceArray<float> dets, lmout, lm[4];
            PinnedArray<uint8_t> h_sum;
        } res[2];
        int wr = 0;    // the set the enqueued step writes
        int done = 0;  // the set of the last finished step
    };
    void stage_device_post(Slot &s, const std::vector<Image> &frames,
                           const std::vector<std::vector<RotatedRect>> &forced);
    void finish_device(Slot &s);  // the slot's step completed: counts; results readable
    void unpack_device(Slot &s) const;
    void materialize() const;
    zr_track_cfg track_cfg() const;
    void stage_detect(Slot &s, const std::vector<Image> &frames);
    void stage_decode_and_rois(Slot &s, const std::vector<Image> &frames,
                               const std::vector<std::vector<RotatedRect>> &forced);
    void stage_map(Slot &s);
    void enqueue_gather();  // after every active slot enqueued a step (records on)
    size_t det_cap() const;

    PipelineConfig cfg_;
    int device_;
    std::shared_ptr<const Cnn> det_cnn_, lm_cnn_;
    DeviceArray<float> d_anchors_;  // [A][2], device post-processing
    NonMaxSuppression nms_;
    ThreadPool pool_;
    void *stream_ = nullptr;
    std::vector<std::unique_ptr<Slot>> slots_;
    mutable std::vector<std::vector<Detection>> dets_;
    std::vector<NonMaxSuppression::TieCount> ties_;  // host mode: per frame of the step
    void add_ties(const NonMaxSuppression::TieCount &t) {
        times_.nms_candidates += (size_t)t.candidates;
        times_.nms_tied += (size_t)t.tied;
        times_.nms_unpinned_frames += t.unpinned() ? 1 : 0;
    }
    mutable std::vector<RoiResult> rois_;
    mutable bool stale_ = false;  // device mode: dets_ / rois_ not yet built from the last step
    StageTimes times_;
    std::vector<Image> frames_;
    std::vector<std::vector<RotatedRect>> forced_;
    size_t active_slots_ = 0;
    std::chrono::steady_clock::time_point steps_t0_;
    // records (enable_records): two sets, step t writes set t & 1
    uint32_t rec_rmax_ = 0, rec_first_ = 0, rec_stride_ = 1;
    zr_comm *comm_ = nullptr;
    int world_ = 1;
    DeviceArray<float> d_rec_[2], d_gath_[2];
    void *gstream_ = nullptr, *ev_gath_[2] = {nullptr, nullptr};
    bool gath_used_[2] = {false, false};
    uint64_t enq_steps_ = 0, done_steps_ = 0;
};

}  // namespace zh
