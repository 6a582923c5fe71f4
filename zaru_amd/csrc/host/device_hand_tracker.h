// device_hand_tracker.h -- HandTracker (crates/zaru/src/hand/tracking.rs:115-219) over n video
// streams with every hand's state in HBM: each step runs, on one HIP stream,
//   1. the LandmarkTracker update of every hand slot from the previous step's estimate
//      (zr_track_update_async, kind "hand"),
//   2. the bookkeeping -- drop lost hands, filter the previous step's palm detections against
//      the hands' ROIs, start new hands, the swap_remove de-duplication, the redetection
//      schedule (zr_hand_manage_async),
//   3. the hand landmark network on every slot's view of this step's frame, and
//   4. BlazePalm with its device post-processing on the streams step 2 asked to detect on
//      (tracking.rs:210-218: no hand tracked, or the redetection interval elapsed): step 2's
//      request flags are compacted on the device into a stream list + count
//      (zr_due_compact_async), the palm launches skip the images past that count
//      (zr_cnn_estimate_device_views_count_async) and the post-processing writes each due stream's
//      slot (zr_detect_post_mapped_async); step 2 consumes them at the next step.
// The host enqueues only: no host round trip per frame.  Stream s owns `slots` hand slots.
// Schedule: a palm detection requested at step t is taken at step t + 1 -- the host HandTracker's
// schedule when every detection finishes within one frame (HandTracker::wait_detection before
// each track call), against which tests/test_gpu_device_hand_tracker.py checks it.
#pragma once
#include <memory>
#include <vector>

#include "detection.h"
#include "landmark.h"

namespace zh {

class DeviceHandTracker {
  public:
    DeviceHandTracker(size_t streams, int slots = 4, int device = 0);
    ~DeviceHandTracker();
    DeviceHandTracker(const DeviceHandTracker &) = delete;
    DeviceHandTracker &operator=(const DeviceHandTracker &) = delete;

    void set_redetect_interval(double ms) { cfg_.interval_ms = ms; }
    void set_iou_thresh(float t) { cfg_.iou_thresh = t; }
    void set_loss_threshold(float t) { tcfg_.loss_thresh = t; }
    // A/B switch: BlazePalm on every stream's frame each step (the round-3 schedule; results of
    // streams that did not ask are discarded) instead of on the due streams only
    void set_palm_every_frame(bool on) { palm_every_ = on; }
    // frames BlazePalm ran on so far (every_frame: all streams each step; else the due streams,
    // counted from the device list after synchronize())
    uint64_t palm_frames();
    // detections handed to stream s's next step as if its palm detection had produced them (test
    // hook, the host HandTracker's inject_detections); replaces that step's palm result
    void inject_detections(size_t s, const std::vector<Detection> &dets);
    // one device-resident frame per stream; `now_ms` stands for Instant::now()
    void step(const std::vector<Image> &frames, double now_ms);
    void synchronize();
    size_t streams() const { return n_; }
    int slots() const { return cfg_.slots; }

    struct HandData {  // tracking.rs:237-262
        uint64_t id;  // HandId(u64), tracking.rs:227
        std::vector<float> landmarks;  // 21 x 3, frame px (the previous step's estimate)
        RotatedRect view_rect;         // the hand's ROI
    };
    // after synchronize(): stream s's hands that have a result (HandTracker::hands)
    std::vector<HandData> hands(size_t s);
    std::vector<int32_t> hand_counts();  // every stream's hands, tracked or new
    std::vector<int32_t> detection_pending();  // streams whose palm detection of the last step counts
    // per stream, the last step's new hands that found no free slot of the `slots` (the reference's
    // hand list is unbounded, tracking.rs:158-194; here capacity is fixed and its overflow reported)
    std::vector<int32_t> dropped_hands();
    // per stream, palm detections of the last palm pass past the detection capacity (0: the
    // capacity is the detector's anchor count, the most NMS can return)
    std::vector<int32_t> dropped_detections();
    size_t detection_capacity() const { return dcap_; }

  private:
    std::shared_ptr<const Cnn> palm_, hand_;
    DetectorNetwork palm_net_ = DetectorNetwork::palm_lite();
    LandmarkNetwork hand_net_ = LandmarkNetwork::hand_lite();
    zr_hand_cfg cfg_{};
    zr_track_cfg tcfg_{};
    zr_detpost_cfg pcfg_{};
    size_t n_ = 0, dcap_ = 0;  // dcap_: every NMS output (the palm detector's anchor count)
    uint64_t steps_ = 0;
    void *stream_ = nullptr;
    uint32_t fw_ = 0, fh_ = 0;  // frame size the letterbox table was built for
    DeviceArray<zr_track_state> state_;
    DeviceArray<uint64_t> ids_, next_id_;
    DeviceArray<uint32_t> fsize_;
    DeviceArray<float> hroi_, lm_out_, outs_[4], palm_boxes_, palm_logits_, anchors_, lbox_, dets_;
    DeviceArray<int32_t> src_, nhands_, det_pending_, count_, dropped_;
    DeviceArray<double> next_det_;
    DeviceArray<zr_view_desc> views_, due_views_;
    DeviceArray<int32_t> due_, ndue_;  // the due streams of a step and their count
    zr_view_desc palm_tmpl_{};         // the letterboxed palm view (frame index set per stream)
    bool palm_every_ = false;
    uint64_t palm_frames_ = 0;         // every-frame mode
    DeviceArray<uint64_t> due_total_;  // due streams summed over the steps (device)
    std::vector<std::vector<Detection>> injected_;
    std::vector<Rect> letterbox_;
};

}  // namespace zh
