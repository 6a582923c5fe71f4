// hand_tracker.h -- crates/zaru/src/hand/tracking.rs (HandTracker) on the HIP backend.
//
// Same state machine as the reference, call for call:
//   1. finish last frame's per-hand landmark work; drop hands whose tracking was lost
//      (tracking.rs:116-127);
//   2. take the palm detections if the detection started earlier has finished, without
//      blocking (tracking.rs:129-134);
//   3. drop detections whose grown box overlaps a tracked ROI, start a tracker for every other
//      one with ROI = RotatedRect(det.rect.grow_rel(1.5), det.angle), padding 0.4
//      (tracking.rs:136-194);
//   4. remove hands whose ROIs overlap an earlier hand's (tracking.rs:196-208);
//   5. start a palm detection when no hand is tracked or the redetect interval elapsed, and
//      none is running (tracking.rs:210-218).
// MI355X-native difference: the reference runs one OS worker thread per hand, each calling
// Cnn::estimate on its own crop, and palm detection on another worker.  Here every tracked
// hand of a frame is one view of ONE batched landmark launch sequence on the GPU, and palm
// detection runs asynchronously on its own HIP stream; "worker finished" is a HIP event.
// Determinism: the reference's steps 3/4 read each hand's ROI while its worker may already be
// processing the new frame (a race resolved by timing).  This tracker always uses the ROI
// produced by the previous frame's result, i.e. the reference's outcome when the worker has
// not yet finished the new frame.
#pragma once
#include <cstdint>
#include <memory>
#include <optional>
#include <vector>

#include "detection.h"
#include "landmark.h"

namespace zh {

class HandTracker {
  public:
    static constexpr float DEFAULT_IOU_THRESH = 0.3f;             // tracking.rs:38
    static constexpr double DEFAULT_REDETECT_INTERVAL_MS = 300.0;  // tracking.rs:41
    static constexpr float ROI_PADDING = 0.4f;                    // tracking.rs:34
    static constexpr float PALM_GROW = 1.5f;                      // tracking.rs:136

    explicit HandTracker(int device = 0);
    ~HandTracker();
    HandTracker(const HandTracker &) = delete;
    HandTracker &operator=(const HandTracker &) = delete;

    void set_redetect_interval(double ms) { det_interval_ms_ = ms; }
    void set_iou_thresh(float t) { iou_ = t; }
    // Not in the reference API (its LandmarkTracker keeps the default 0.5): lets tests keep
    // tracking alive on synthetic frames.
    void set_loss_threshold(float t) { loss_ = t; }

    // HandTracker::track(Arc<Image>).  `now_ms` stands for Instant::now(); the redetect clock
    // starts at the first call (the reference starts it at construction).  The image is copied
    // into a tracker-owned device buffer, so the caller may reuse its buffer at once.
    void track(const Image &img, double now_ms);
    void track(const Image &img);

    struct HandData {  // tracking.rs:237-262
        uint64_t id;
        Estimate landmarks;     // global image coordinates
        RotatedRect view_rect;  // the hand's ROI (updated_roi of its last result)
    };
    // HandTracker::hands(): the hands that have a result from the previous `track` call.
    std::vector<HandData> hands() const;

    // Test hooks (no reference counterpart).  `wait_detection` blocks until a running palm
    // detection has finished, so the next `track` takes its result (the reference's
    // `!handle.will_block()`).  `inject_detections` hands detections to the next `track`
    // call as if the palm detector had produced them.
    void wait_detection();
    void inject_detections(std::vector<Detection> dets);
    bool detection_running() const { return det_running_; }
    size_t num_tracked() const { return hands_.size(); }

    // Steps 3 and 4 as pure functions of the ROIs (CPU-testable).
    // keep[i]: detection i overlaps no ROI (IoU with its grown box < thresh).
    static std::vector<bool> filter_detections(const std::vector<Rect> &rois,
                                               const std::vector<Detection> &dets, float iou_thresh);
    // The Vec::swap_remove sweep of tracking.rs:197-208; returns the surviving indices into
    // `rois` in their resulting order.
    static std::vector<size_t> dedupe_rois(const std::vector<Rect> &rois, float iou_thresh);

  private:
    struct Hand {
        uint64_t id = 0;
        RotatedRect roi;             // roi_arc: last updated_roi, or the seeding ROI
        RotatedRect tracker_roi;     // the hand's LandmarkTracker ROI (padded)
        std::optional<Estimate> lm;  // result of the previous frame
        bool pending = false;        // has a view in the in-flight landmark batch
        size_t slot = 0;             // its index in that batch
        RotatedRect view_rect;       // view of the in-flight estimate (landmark.rs:465)
        Rect local_rect;             // its map-out rect (landmark.rs:320-323)
    };
    struct FrameBuf;

    FrameBuf *upload(const Image &img);
    void finish_landmarks();
    void collect_detection(std::vector<Detection> &out);
    void launch_landmarks(FrameBuf *fb);
    void launch_detection(FrameBuf *fb);

    std::shared_ptr<const Cnn> palm_, hand_;
    DetectorNetwork palm_net_ = DetectorNetwork::palm_lite();
    LandmarkNetwork hand_net_ = LandmarkNetwork::hand_lite();
    NonMaxSuppression nms_;
    float iou_ = DEFAULT_IOU_THRESH, loss_ = LandmarkTracker::DEFAULT_LOSS_THRESHOLD;
    double det_interval_ms_ = DEFAULT_REDETECT_INTERVAL_MS;
    std::optional<double> next_det_ms_;
    uint64_t next_id_ = 0;
    std::vector<Hand> hands_;
    std::vector<Detection> injected_;

    void *lm_stream_ = nullptr, *det_stream_ = nullptr;
    void *lm_done_ = nullptr, *det_done_ = nullptr;
    std::vector<std::unique_ptr<FrameBuf>> bufs_;
    FrameBuf *lm_frame_ = nullptr, *det_frame_ = nullptr;  // frames the in-flight work reads
    bool lm_running_ = false, det_running_ = false;
    Rect det_letterbox_;
    DeviceArray<float> d_lm_[4], d_boxes_, d_logits_;
    PinnedArray<float> h_lm_[4], h_boxes_, h_logits_;
};

}  // namespace zh
