// device_face_loop.h -- the face video loop of the reference's demo
// (crates/zaru/examples/facemesh.rs:35-56) over n camera streams with every tracker's state in
// HBM.  Per frame the reference runs
//     if let Some(r) = tracker.track(&image) { ... }            // LandmarkTracker::track_impl
//     else { detections = detector.detect(&image);               // only when tracking is lost
//            tracker.set_roi(max_by_key(confidence).bounding_rect()) }
// Each step here enqueues, on one HIP stream and with no host decision between frames:
//   1. the landmark network on every stream's view (written by the previous step),
//   2. the tracker update (zr_track_update_async: loss check, map-out, bounding, next view),
//   3. the streams left without RoI compacted into a list + device count
//      (zr_track_lost_compact_async),
//   4. the detector on those streams' letterboxed frames only (the launches skip images past the
//      count: zr_cnn_estimate_device_views_count_async) and its post-processing into each
//      stream's slot (zr_detect_post_mapped_async),
//   5. the re-seeding of those streams from their most confident detection
//      (zr_track_reseed_best_async), which writes the view the next frame's estimate samples.
// A stream with no RoI at construction detects on its first frame, as the demo starts.
#pragma once
#include <memory>
#include <utility>
#include <vector>

#include "detection.h"
#include "landmark.h"

namespace zh {

class DeviceFaceLoop {
  public:
    DeviceFaceLoop(DetectorNetwork detector, LandmarkNetwork landmarker, size_t streams, int device = 0,
                   float padding = LandmarkTracker::DEFAULT_ROI_PADDING,
                   float loss_thresh = LandmarkTracker::DEFAULT_LOSS_THRESHOLD,
                   float det_thresh = Detector::DEFAULT_THRESHOLD);
    ~DeviceFaceLoop();
    DeviceFaceLoop(const DeviceFaceLoop &) = delete;
    DeviceFaceLoop &operator=(const DeviceFaceLoop &) = delete;

    // LandmarkTracker::set_roi for stream s before its next frame (test / warm-start hook)
    void set_roi(size_t s, const RotatedRect &roi);
    // one device-resident frame per stream (all of one size); enqueue only
    void step(const std::vector<Image> &frames);
    void synchronize();
    size_t streams() const { return n_; }
    const LandmarkNetwork &landmarker() const { return lm_net_; }

    // after synchronize():
    std::vector<zr_track_state> states();       // tracked = this frame's track() returned Some
    std::vector<float> landmarks();             // this frame, frame px, n x L x 3 (NaN: not tracked)
    std::vector<int32_t> detected();            // per stream: 1 if this frame ran the detector
    std::vector<int32_t> detection_counts();    // per stream: faces this frame's detection found
    uint64_t detections_run();                  // detector images summed over the steps
    uint64_t reacquisitions();                  // streams re-seeded from a detection, summed

  private:
    void frame_size(uint32_t W, uint32_t H);
    std::shared_ptr<const Cnn> det_, lm_;
    DetectorNetwork det_net_;
    LandmarkNetwork lm_net_;
    zr_track_cfg tcfg_{};
    zr_detpost_cfg pcfg_{};
    size_t n_ = 0, dcap_ = 0;
    void *stream_ = nullptr;
    uint32_t fw_ = 0, fh_ = 0;
    zr_view_desc det_tmpl_{};  // the letterboxed detector view (frame index set per stream)
    std::vector<std::pair<size_t, RotatedRect>> pending_rois_;
    DeviceArray<zr_track_state> state_;
    DeviceArray<zr_view_desc> views_, due_views_;
    DeviceArray<float> lm_outs_[4], lm_out_, det_boxes_, det_logits_, anchors_, lbox_, dets_;
    DeviceArray<uint32_t> fsize_;
    DeviceArray<int32_t> due_, ndue_, count_;
    DeviceArray<uint64_t> due_total_, reseeded_;
};

}  // namespace zh
