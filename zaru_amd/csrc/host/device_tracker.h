// device_tracker.h -- LandmarkTracker (crates/zaru/src/landmark.rs:354-501) over n video
// streams with its state in HBM: each step runs the landmark network on
// views the previous step's update wrote, then the update kernel, all enqueued on one HIP
// stream; the host touches nothing between frames.  ROI i follows stream i.
#pragma once
#include <memory>
#include <utility>
#include <vector>

#include "landmark.h"

namespace zh {

// the track kernel's extract / angle kind of a landmark network (zr_track_cfg::kind)
int track_kind(NetworkKind k);

class DeviceTracker {
  public:
    DeviceTracker(LandmarkNetwork net, int device = 0, float padding = LandmarkTracker::DEFAULT_ROI_PADDING,
                  float loss_thresh = LandmarkTracker::DEFAULT_LOSS_THRESHOLD);
    ~DeviceTracker();
    DeviceTracker(const DeviceTracker &) = delete;
    DeviceTracker &operator=(const DeviceTracker &) = delete;

    // LandmarkTracker::set_roi for every stream, with each stream's frame size
    void set_rois(const std::vector<RotatedRect> &rois, const std::vector<std::pair<uint32_t, uint32_t>> &sizes);
    // one device-resident frame per stream (frames[i] -> ROI i): estimate + update, enqueue only
    void step(const std::vector<Image> &frames);
    void synchronize();
    size_t size() const { return n_; }
    const LandmarkNetwork &network() const { return net_; }
    std::vector<zr_track_state> states();      // after synchronize()
    std::vector<float> landmarks();            // last step, frame px, n x L x 3 (NaN rows: not tracked)
    std::vector<zr_view_desc> views();         // the view table the next step samples
    // the view the host path (pipeline.cpp / Estimator) derives from `roi`, for parity checks
    zr_view_desc host_view(const RotatedRect &roi, uint32_t frame_w, uint32_t frame_h, uint32_t frame) const;
    void *stream() const { return stream_; }

  private:
    LandmarkNetwork net_;
    std::shared_ptr<const Cnn> cnn_;
    zr_track_cfg cfg_{};
    size_t n_ = 0;
    void *stream_ = nullptr;
    DeviceArray<zr_track_state> state_;
    DeviceArray<zr_view_desc> views_;
    DeviceArray<float> outs_[4], lm_out_;
};

}  // namespace zh
