// detection.h -- crates/zaru/src/detection{.rs,/ssd.rs,/nms.rs}, face/detection.rs and
// hand/detection.rs: SSD anchors, BlazeFace / BlazePalm decode, weighted NMS and the generic
// Detector driver.  Bit-exact with the reference given the same raw network outputs.
#pragma once
#include <memory>
#include <vector>

#include "geometry.h"
#include "networks.h"

namespace zh {

struct Detection {  // detection.rs:288-293
    float confidence = 0.f;
    float angle = 0.f;
    Rect rect;
    std::vector<Vec2> keypoints;
    int32_t anchor = -1;  // anchor index (documented NMS tie rule)
};

struct LayerInfo {  // ssd.rs:43-64
    uint32_t boxes_per_cell, width, height;
};

// ssd.rs:96-119 -- centres only; boxes_per_cell repeats the centre
std::vector<Vec2> calculate_anchors(const std::vector<LayerInfo> &layers);

enum class SuppressionMode { Remove, Average };

class NonMaxSuppression {  // nms.rs:18-146
  public:
    static constexpr float DEFAULT_IOU_THRESH = 0.3f;
    void set_iou_thresh(float t) { iou_ = t; }
    void set_mode(SuppressionMode m) { mode_ = m; }
    float iou_thresh() const { return iou_; }
    SuppressionMode mode() const { return mode_; }
    // Sorts `dets` ascending by confidence (stable: ties keep input order, as Rust's
    // sort_unstable does for <= 20 elements) and returns the suppressed/averaged list.
    // `ties` (optional): the candidate count and how many of them share their confidence with
    // another candidate.  Above 20 candidates Rust's sort_unstable (ipnsort) is not stable, so a
    // frame with more than 20 candidates and a tie has an order the reference does not pin.
    struct TieCount {
        int candidates = 0, tied = 0;
        bool unpinned() const { return candidates > 20 && tied > 0; }
    };
    std::vector<Detection> process(std::vector<Detection> &dets, TieCount *ties = nullptr) const;

  private:
    float iou_ = DEFAULT_IOU_THRESH;
    SuppressionMode mode_ = SuppressionMode::Average;
};

// A detection network (detection.rs:21-40) with its decode (extract).
struct DetectorNetwork {
    NetworkKind kind;
    std::vector<LayerInfo> layers;
    int params;    // 16 face / 18 palm
    int keypoints;  // 6 / 7
    static DetectorNetwork short_range_face();  // face/detection.rs:30-59
    static DetectorNetwork full_range_face();   // face/detection.rs:61-94
    static DetectorNetwork palm_lite();         // hand/detection.rs:49-75
    const std::vector<Vec2> &anchors() const;
    // extract_detection (face/detection.rs:124-157, hand/detection.rs:144-179)
    Detection decode(uint32_t anchor, const float *box_params, float confidence, uint32_t in_w,
                     uint32_t in_h) const;
    // extract_outputs over a full [A][params] / [A] pair (face/detection.rs:96-122)
    void extract(const float *boxes, const float *logits, float thresh, uint32_t in_w,
                 uint32_t in_h, std::vector<Detection> &out) const;

  private:
    mutable std::shared_ptr<std::vector<Vec2>> anchors_;
};

// Detector::detect_impl steps after inference (detection.rs:245-267)
void map_detections(std::vector<Detection> &dets, const Rect &letterbox, uint32_t in_w);

// Fixed-size detection records, the payload of the multi-GPU all-gather: per
// frame {frame id (u32 bits), count (u32 bits)} then `rmax` x {conf, angle, cx, cy, w, h,
// 7 x (kx, ky)} (20 f32 each, zero-padded; detections beyond rmax are dropped, count is not).
constexpr uint32_t DET_RECORD_FIELDS = 20;
inline uint32_t det_record_width(uint32_t rmax) { return 2 + DET_RECORD_FIELDS * rmax; }
void pack_detection_records(const std::vector<std::vector<Detection>> &dets,
                            const std::vector<uint32_t> &frame_ids, uint32_t rmax, float *out);

class Detector {  // detection.rs:152-276
  public:
    static constexpr float DEFAULT_THRESHOLD = 0.5f;
    Detector(DetectorNetwork net, int device = 0);
    void set_threshold(float t) { thresh_ = t; }
    float threshold() const { return thresh_; }
    NonMaxSuppression &nms_mut() { return nms_; }
    uint32_t input_width() const { return cnn_->input_width(); }
    const std::vector<Detection> &detect(const Image &img);
    const DetectorNetwork &network() const { return net_; }
    const Cnn &cnn() const { return *cnn_; }

  private:
    DetectorNetwork net_;
    std::shared_ptr<const Cnn> cnn_;
    float thresh_ = DEFAULT_THRESHOLD;
    NonMaxSuppression nms_;
    std::vector<Detection> dets_;
};

// The letterboxed view a detector samples from a w x h image (detection.rs:224-227).
ViewData letterbox_view(uint32_t w, uint32_t h, AspectRatio in_aspect, Rect *rect_out = nullptr);

// Conservative raw-logit bound below which sigmoid(logit) < thresh for sure; used by the
// device candidate compaction so that the exact host decode sees every anchor it could keep.
float candidate_logit_floor(float thresh);

}  // namespace zh
