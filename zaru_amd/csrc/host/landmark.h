// landmark.h -- crates/zaru/src/landmark.rs (Estimator, LandmarkTracker) with the two
// hot-path landmark networks: FaceMeshV1 (face/landmark/mediapipe.rs:41-272) and the hand
// landmark LiteNetwork (hand/landmark.rs:244-322).
#pragma once
#include <memory>
#include <optional>
#include <vector>

#include "geometry.h"
#include "networks.h"

namespace zh {

struct LandmarkNetwork {
    NetworkKind kind;
    int num_landmarks;  // 468 / 478 / 21
    static LandmarkNetwork face_mesh_v1();
    static LandmarkNetwork face_mesh_v2();  // mediapipe.rs:81-116
    static LandmarkNetwork eye();           // face/eye.rs:29-64 (76 points: 5 iris + 71 contour)
    static LandmarkNetwork face_onnx_68();  // multipie68.rs:83-118
    static LandmarkNetwork peppa_68();      // multipie68.rs:46-81
    static LandmarkNetwork hand_lite();
};

// One estimate (LandmarkResultV1 / hand LandmarkResult): positions n x 3 plus flags.
struct Estimate {
    std::vector<float> positions;  // n * 3
    float confidence = 0.f;        // face_flag (sigmoid) / hand presence (Confidence trait)
    float raw_handedness = 0.f;    // hand only
    float tongue_out = 0.f;        // FaceMesh V2 blendshape (sigmoid inside the graph)
    std::vector<float> world;      // hand metric landmarks (Identity_3), n * 3
    size_t size() const { return positions.size() / 3; }
    Vec2 xy(size_t i) const { return {positions[3 * i], positions[3 * i + 1]}; }
};

// extract() of each network from one image's raw outputs (mediapipe.rs:59-71,
// hand/landmark.rs:298-322, eye.rs:47-64, multipie68.rs:71-80,108-117).  `outs[i]` points at
// that image's slice of output i; in_w / in_h: the network input resolution (the 68-point nets
// emit coordinates relative to it).  Networks whose reference Output has no Confidence (eye,
// 68-point) report confidence 1.
void extract_landmarks(const LandmarkNetwork &net, const float *const *outs, Estimate &e,
                       uint32_t in_w = 0, uint32_t in_h = 0);

// Estimate::angle_radians: FaceMesh eye corners 33 -> 263 against +X (mediapipe.rs:146-160);
// hand wrist - middle MCP against +Y (hand/landmark.rs:68-78); none for the eye / 68-point
// networks (the trait default, landmark.rs:217-219) -- 0, which LandmarkTracker adds exactly as
// `unwrap_or(0.0)` does (landmark.rs:479).
float estimate_angle(const LandmarkNetwork &net, const Estimate &e);

// Estimator::estimate_impl map-out (landmark.rs:336-345)
void map_estimate(Estimate &e, const Rect &rect, uint32_t in_w);

class Estimator {  // landmark.rs:256-349
  public:
    Estimator(LandmarkNetwork net, int device = 0);
    const LandmarkNetwork &network() const { return net_; }
    const Cnn &cnn() const { return *cnn_; }
    uint32_t input_width() const { return cnn_->input_width(); }
    AspectRatio aspect() const { return cnn_->aspect(); }
    // estimate on a view of a host image; landmarks in the view's coordinates
    Estimate &estimate(const Image &img, const ViewData &view);
    // the view actually sampled and the rect used for map-out (landmark.rs:320-323)
    ViewData network_view(const ViewData &view, Rect *rect_out) const;

  private:
    LandmarkNetwork net_;
    std::shared_ptr<const Cnn> cnn_;
    Estimate est_;
};

struct TrackingResult {  // landmark.rs:504-529
    RotatedRect view_rect;
    RotatedRect updated_roi;
    Estimate estimate;  // landmarks in full-image coordinates
};

// LandmarkTracker::track_impl after the estimate (landmark.rs:468-494); returns false when
// tracking is lost (confidence below the loss threshold), true with `res`/`next_roi` otherwise.
bool tracker_update(const LandmarkNetwork &net, const RotatedRect &roi, const RotatedRect &view_rect,
                    float loss_thresh, float padding, Estimate &est, TrackingResult &res,
                    RotatedRect &next_roi);

class LandmarkTracker {  // landmark.rs:361-502
  public:
    static constexpr float DEFAULT_LOSS_THRESHOLD = 0.5f;
    static constexpr float DEFAULT_ROI_PADDING = 0.3f;
    explicit LandmarkTracker(Estimator est);
    void set_loss_threshold(float t) { loss_ = t; }
    void set_roi_padding(float p);
    void set_roi(const RotatedRect &r) { roi_ = r; }
    const std::optional<RotatedRect> &roi() const { return roi_; }
    Estimator &estimator() { return est_; }
    float loss_threshold() const { return loss_; }
    float roi_padding() const { return pad_; }
    // nullopt when no ROI is set or tracking was lost
    std::optional<TrackingResult> track(const Image &full);

  private:
    Estimator est_;
    std::optional<RotatedRect> roi_;
    float loss_ = DEFAULT_LOSS_THRESHOLD, pad_ = DEFAULT_ROI_PADDING;
};

}  // namespace zh
