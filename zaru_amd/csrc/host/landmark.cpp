// landmark.cpp -- see landmark.h.
#include "landmark.h"

#include <algorithm>

namespace zh {

LandmarkNetwork LandmarkNetwork::face_mesh_v1() { return {NetworkKind::FaceMeshV1, 468}; }
LandmarkNetwork LandmarkNetwork::face_mesh_v2() { return {NetworkKind::FaceMeshV2, 478}; }
LandmarkNetwork LandmarkNetwork::eye() { return {NetworkKind::IrisLandmark, 76}; }
LandmarkNetwork LandmarkNetwork::face_onnx_68() { return {NetworkKind::FaceOnnx68, 68}; }
LandmarkNetwork LandmarkNetwork::peppa_68() { return {NetworkKind::PeppaFacialLandmark68, 68}; }
LandmarkNetwork LandmarkNetwork::hand_lite() { return {NetworkKind::HandLandmarkLite, 21}; }

void extract_landmarks(const LandmarkNetwork &net, const float *const *outs, Estimate &e,
                       uint32_t in_w, uint32_t in_h) {
    const size_t n = (size_t)net.num_landmarks;
    if (net.kind == NetworkKind::IrisLandmark) {
        // iris (5 x 3, output 1) first, then the eye contour (71 x 3, output 0) (eye.rs:47-64)
        e.positions.resize(3 * n);
        std::copy(outs[1], outs[1] + 15, e.positions.begin());
        std::copy(outs[0], outs[0] + 3 * (n - 5), e.positions.begin() + 15);
        e.confidence = 1.f;
        return;
    }
    if (net.kind == NetworkKind::FaceOnnx68 || net.kind == NetworkKind::PeppaFacialLandmark68) {
        // (x, y) pairs relative to the input resolution, z = 0 (multipie68.rs:71-80)
        e.positions.assign(3 * n, 0.f);
        for (size_t i = 0; i < n; i++) {
            e.positions[3 * i] = outs[0][2 * i] * (float)in_w;
            e.positions[3 * i + 1] = outs[0][2 * i + 1] * (float)in_h;
        }
        e.confidence = 1.f;
        return;
    }
    e.positions.assign(outs[0], outs[0] + 3 * n);
    if (net.kind == NetworkKind::FaceMeshV1) {
        e.confidence = sigmoid(outs[1][0]);  // face_flag, mediapipe.rs:60
    } else if (net.kind == NetworkKind::FaceMeshV2) {
        e.confidence = sigmoid(outs[1][0]);  // face_flag, mediapipe.rs:100
        e.tongue_out = outs[2][0];           // mediapipe.rs:103
    } else {
        e.confidence = outs[1][0];  // presence (sigmoid inside the graph)
        e.raw_handedness = outs[2][0];
        e.world.assign(outs[3], outs[3] + 3 * n);
    }
}

float estimate_angle(const LandmarkNetwork &net, const Estimate &e) {
    if (is_face_mesh(net.kind)) return signed_angle_to(e.xy(263) - e.xy(33), Vec2{1.f, 0.f});
    if (net.kind != NetworkKind::HandLandmarkLite) return 0.f;
    return signed_angle_to(e.xy(0) - e.xy(9), Vec2{0.f, 1.f});
}

void map_estimate(Estimate &e, const Rect &rect, uint32_t in_w) {
    const float scale = rect.width() / (float)in_w;
    const float x = rect.x(), y = rect.y();
    for (size_t i = 0; i < e.size(); i++) {
        float *p = &e.positions[3 * i];
        p[0] = p[0] * scale;
        p[1] = p[1] * scale;
        p[2] = p[2] * scale;
        p[0] += x;
        p[1] += y;
    }
}

Estimator::Estimator(LandmarkNetwork net, int device)
    : net_(net), cnn_(network_cnn(net.kind, device)) {}

ViewData Estimator::network_view(const ViewData &view, Rect *rect_out) const {
    const Rect rect = view.local_rect().grow_to_fit_aspect(cnn_->aspect());
    if (rect_out) *rect_out = rect;
    return view.view(RotatedRect(rect, 0.f));
}

Estimate &Estimator::estimate(const Image &img, const ViewData &view) {
    Rect rect;
    const ViewData v = network_view(view, &rect);
    auto outs = cnn_->estimate(img, {v});
    std::vector<const float *> ptrs;
    for (auto &o : outs) ptrs.push_back(o.data());
    extract_landmarks(net_, ptrs.data(), est_, cnn_->input_width(), cnn_->input_height());
    // the default LandmarkFilter is a no-op (landmark.rs:151-158)
    map_estimate(est_, rect, cnn_->input_width());
    return est_;
}

bool tracker_update(const LandmarkNetwork &net, const RotatedRect &roi, const RotatedRect &view_rect,
                    float loss_thresh, float padding, Estimate &est, TrackingResult &res,
                    RotatedRect &next_roi) {
    if (est.confidence < loss_thresh) return false;
    const float angle = roi.rotation_radians() + estimate_angle(net, est);
    for (size_t i = 0; i < est.size(); i++) {
        const Vec2 o = view_rect.transform_out(est.xy(i));
        est.positions[3 * i] = o.x;
        est.positions[3 * i + 1] = o.y;
    }
    RotatedRect updated;
    RotatedRect::bounding(angle, reinterpret_cast<const Vec2 *>(est.positions.data()), est.size(), 3,
                          updated);
    next_roi = updated.grow_rel(padding);
    res.view_rect = view_rect;
    res.updated_roi = updated;
    res.estimate = est;
    return true;
}

LandmarkTracker::LandmarkTracker(Estimator est) : est_(std::move(est)) {}

void LandmarkTracker::set_roi_padding(float p) {
    if (!(p >= 0.f)) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "roi padding must be >= 0");
    pad_ = p;
}

std::optional<TrackingResult> LandmarkTracker::track(const Image &full) {
    if (!roi_) return std::nullopt;
    const RotatedRect roi = *roi_;
    const RotatedRect view_rect = roi.grow_to_fit_aspect(est_.aspect());
    const ViewData view = ViewData::full(full.width, full.height).view(view_rect);
    Estimate &e = est_.estimate(full, view);
    TrackingResult res;
    RotatedRect next;
    if (!tracker_update(est_.network(), roi, view_rect, loss_, pad_, e, res, next)) {
        roi_.reset();
        return std::nullopt;
    }
    roi_ = next;
    return res;
}

}  // namespace zh
