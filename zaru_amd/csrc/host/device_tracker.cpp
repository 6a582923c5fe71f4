// device_tracker.cpp -- see device_tracker.h.
#include "device_tracker.h"

namespace zh {

int track_kind(NetworkKind k) {
    if (is_face_mesh(k)) return 0;  // face_flag = sigmoid(out1), eye line 33 -> 263
    if (k == NetworkKind::HandLandmarkLite) return 1;
    if (k == NetworkKind::IrisLandmark) return 2;
    if (k == NetworkKind::FaceOnnx68 || k == NetworkKind::PeppaFacialLandmark68) return 3;
    throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "not a landmark network");
}

DeviceTracker::DeviceTracker(LandmarkNetwork net, int device, float padding, float loss_thresh)
    : net_(net), cnn_(network_cnn(net.kind, device)) {
    if (!(padding >= 0.f)) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "roi padding must be >= 0");
    const AspectRatio a = cnn_->aspect();
    cfg_.kind = track_kind(net.kind);
    cfg_.num_landmarks = net.num_landmarks;
    cfg_.in_w = (int)cnn_->input_width();
    cfg_.in_h = (int)cnn_->input_height();
    cfg_.aspect_w = (int)a.w;
    cfg_.aspect_h = (int)a.h;
    cfg_.loss_thresh = loss_thresh;
    cfg_.padding = padding;
    check(zr_stream_create(&stream_));
}

DeviceTracker::~DeviceTracker() {
    if (stream_) {
        (void)zr_stream_synchronize(stream_);
        (void)zr_stream_destroy(stream_);
    }
}

void DeviceTracker::set_rois(const std::vector<RotatedRect> &rois,
                             const std::vector<std::pair<uint32_t, uint32_t>> &sizes) {
    if (rois.size() != sizes.size() || rois.empty())
        throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "one frame size per ROI, at least one ROI");
    synchronize();
    n_ = rois.size();
    std::vector<zr_track_state> h(n_);
    for (size_t i = 0; i < n_; i++) {
        const Rect &r = rois[i].rect();
        h[i] = zr_track_state{};
        h[i].roi[0] = r.center().x;
        h[i].roi[1] = r.center().y;
        h[i].roi[2] = r.width();
        h[i].roi[3] = r.height();
        h[i].roi[4] = rois[i].rotation_radians();
        h[i].active = 1;
        h[i].frame_w = sizes[i].first;
        h[i].frame_h = sizes[i].second;
    }
    state_.resize(n_);
    views_.resize(n_);
    const NeuralNetwork &nn = cnn_->nn();
    for (size_t k = 0; k < nn.num_outputs() && k < 4; k++) outs_[k].resize((size_t)nn.output_per_image(k) * n_);
    lm_out_.resize(n_ * (size_t)net_.num_landmarks * 3);
    check(zr_memcpy_async(state_.ptr, h.data(), n_ * sizeof(zr_track_state), 0, stream_));
    check(zr_track_seed_async(state_.ptr, n_, &cfg_, views_.ptr, stream_));
    check(zr_stream_synchronize(stream_));  // `h` is pageable and goes out of scope
}

void DeviceTracker::step(const std::vector<Image> &frames) {
    if (frames.size() != n_ || n_ == 0) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "one frame per tracked ROI");
    std::vector<zr_frame> zf(n_);
    for (size_t i = 0; i < n_; i++) {
        if (!frames[i].on_device) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "tracker frames must be device-resident");
        zf[i] = zr_frame{frames[i].rgba, frames[i].width, frames[i].height, frames[i].row_stride};
    }
    const NeuralNetwork &nn = cnn_->nn();
    float *outs[4] = {outs_[0].ptr, outs_[1].ptr, outs_[2].ptr, outs_[3].ptr};
    const ColorMapper cm = cnn_->color_mapper();
    // the frame table is staged (pinned) inside the call, so zf may die after it returns
    check(zr_cnn_estimate_device_views_async(nn.handle(), zf.data(), n_, views_.ptr, n_, cm.lo, cm.hi, outs, stream_));
    const bool flagged = cfg_.kind <= 2;  // flag output, or (kind 2) the iris output
    check(zr_track_update_async(state_.ptr, n_, &cfg_, outs_[0].ptr, (size_t)nn.output_per_image(0),
                                flagged ? outs_[1].ptr : nullptr, flagged ? (size_t)nn.output_per_image(1) : 0,
                                lm_out_.ptr, views_.ptr, stream_));
}

void DeviceTracker::synchronize() {
    if (stream_) check(zr_stream_synchronize(stream_));
}

std::vector<zr_track_state> DeviceTracker::states() {
    std::vector<zr_track_state> h(n_);
    if (n_) {
        check(zr_memcpy_async(h.data(), state_.ptr, n_ * sizeof(zr_track_state), 1, stream_));
        synchronize();
    }
    return h;
}

std::vector<zr_view_desc> DeviceTracker::views() {
    std::vector<zr_view_desc> h(n_);
    if (n_) {
        check(zr_memcpy_async(h.data(), views_.ptr, n_ * sizeof(zr_view_desc), 1, stream_));
        synchronize();
    }
    return h;
}

zr_view_desc DeviceTracker::host_view(const RotatedRect &roi, uint32_t frame_w, uint32_t frame_h,
                                      uint32_t frame) const {
    // LandmarkTracker::track_impl's view (landmark.rs:465-467) + Estimator's aspect fit
    // (landmark.rs:320-323), as the host pipeline builds it (pipeline.cpp)
    const AspectRatio a = cnn_->aspect();
    const ViewData view = ViewData::full(frame_w, frame_h).view(roi.grow_to_fit_aspect(a));
    const ViewData net = view.view(RotatedRect(view.local_rect().grow_to_fit_aspect(a), 0.f));
    const zr_view z = to_zr_view(net);
    zr_view_desc d{};
    check(zr_view_describe(&z, 1, frame, &d));
    return d;
}

std::vector<float> DeviceTracker::landmarks() {
    std::vector<float> h(n_ * (size_t)net_.num_landmarks * 3);
    if (!h.empty()) {
        check(zr_memcpy_async(h.data(), lm_out_.ptr, h.size() * 4, 1, stream_));
        synchronize();
    }
    return h;
}

}  // namespace zh
