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
    RotatedRect roi;       // ROI the tracker was seeded with
    TrackingResult result; // valid when tracked
    RotatedRect next_roi;
};

struct StageTimes {  // mirrors Detector::timers / Estimator::timers (detection.rs:273-275)
    double detect_gpu_ms = 0, decode_nms_ms = 0, landmark_gpu_ms = 0, map_ms = 0, total_ms = 0;
    size_t frames = 0, detections = 0, rois = 0, tracked = 0;
};

struct PipelineConfig {
    DetectorNetwork detector = DetectorNetwork::short_range_face();
    LandmarkNetwork landmarker = LandmarkNetwork::face_mesh_v1();
    float det_threshold = Detector::DEFAULT_THRESHOLD;
    float nms_iou = NonMaxSuppression::DEFAULT_IOU_THRESH;
    // ROI from a detection: RotatedRect(det.rect.grow_rel(roi_grow), use_det_angle ? angle : 0)
    float roi_grow = 0.f;
    bool roi_use_angle = false;
    float roi_padding = LandmarkTracker::DEFAULT_ROI_PADDING;
    float loss_threshold = LandmarkTracker::DEFAULT_LOSS_THRESHOLD;
    uint32_t max_rois_per_frame = 8;
    uint32_t candidate_cap = 64;  // device compaction slots per frame (overflow -> full copy)
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

    const std::vector<std::vector<Detection>> &detections() const { return dets_; }
    const std::vector<RoiResult> &rois() const { return rois_; }
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

  private:
    PipelineConfig cfg_;
    int device_;
    std::shared_ptr<const Cnn> det_cnn_, lm_cnn_;
    NonMaxSuppression nms_;
    ThreadPool pool_;
    void *stream_ = nullptr;
    DeviceArray<float> d_boxes_, d_logits_, d_rec_, d_lm_[4];
    DeviceArray<int32_t> d_count_;
    std::vector<float> h_rec_, h_lm_[4];
    std::vector<int32_t> h_count_;
    std::vector<std::vector<Detection>> dets_;
    std::vector<RoiResult> rois_;
    StageTimes times_;
};

}  // namespace zh
