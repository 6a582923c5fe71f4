// device_face_loop.cpp -- see device_face_loop.h.
#include "device_face_loop.h"

#include "device_tracker.h"

namespace zh {

DeviceFaceLoop::DeviceFaceLoop(DetectorNetwork detector, LandmarkNetwork landmarker, size_t streams, int device,
                               float padding, float loss_thresh, float det_thresh)
    : det_(network_cnn(detector.kind, device)), lm_(network_cnn(landmarker.kind, device)), det_net_(detector),
      lm_net_(landmarker) {
    if (streams == 0 || streams > (1u << 20)) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "bad stream count");
    if (!is_face_detector(detector.kind) || !is_face_mesh(landmarker.kind))
        throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "the face loop pairs a face detector with a face mesh network");
    if (!(padding >= 0.f)) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "roi padding must be >= 0");
    n_ = streams;
    const AspectRatio a = lm_->aspect();
    tcfg_.kind = track_kind(landmarker.kind);
    tcfg_.num_landmarks = landmarker.num_landmarks;
    tcfg_.in_w = (int)lm_->input_width();
    tcfg_.in_h = (int)lm_->input_height();
    tcfg_.aspect_w = (int)a.w;
    tcfg_.aspect_h = (int)a.h;
    tcfg_.loss_thresh = loss_thresh;
    tcfg_.padding = padding;
    pcfg_.face = 1;
    pcfg_.anchors = (int)det_net_.anchors().size();
    pcfg_.params = det_net_.params;
    pcfg_.keypoints = det_net_.keypoints;
    pcfg_.in_w = (int)det_->input_width();
    pcfg_.in_h = (int)det_->input_height();
    pcfg_.thresh = det_thresh;
    pcfg_.iou = NonMaxSuppression::DEFAULT_IOU_THRESH;
    dcap_ = det_net_.anchors().size();  // every NMS output: max_by_key sees them all
    check(zr_stream_create(&stream_));
    state_.resize(n_);
    views_.resize(n_);
    due_views_.resize(n_);
    const NeuralNetwork &ln = lm_->nn();
    for (size_t k = 0; k < ln.num_outputs() && k < 4; k++) lm_outs_[k].resize((size_t)ln.output_per_image(k) * n_);
    lm_out_.resize(n_ * (size_t)lm_net_.num_landmarks * 3);
    det_boxes_.resize(n_ * (size_t)pcfg_.anchors * pcfg_.params);
    det_logits_.resize(n_ * (size_t)pcfg_.anchors);
    dets_.resize(n_ * dcap_ * 20);
    lbox_.resize(4 * n_);
    fsize_.resize(2 * n_);
    due_.resize(n_);
    ndue_.resize(1);
    count_.resize(n_);
    due_total_.resize(1);
    reseeded_.resize(1);
    const auto &an = det_net_.anchors();
    anchors_.resize(2 * an.size());
    check(zr_memcpy_async(anchors_.ptr, an.data(), an.size() * sizeof(Vec2), 0, stream_));
    const std::vector<int32_t> zi(n_, 0);
    const uint64_t z = 0;
    check(zr_memcpy_async(count_.ptr, zi.data(), n_ * 4, 0, stream_));
    check(zr_memcpy_async(ndue_.ptr, zi.data(), 4, 0, stream_));
    check(zr_memcpy_async(due_total_.ptr, &z, 8, 0, stream_));
    check(zr_memcpy_async(reseeded_.ptr, &z, 8, 0, stream_));
    check(zr_stream_synchronize(stream_));  // the host vectors are pageable and go out of scope
}

DeviceFaceLoop::~DeviceFaceLoop() {
    if (stream_) {
        (void)zr_stream_synchronize(stream_);
        (void)zr_stream_destroy(stream_);
    }
}

void DeviceFaceLoop::set_roi(size_t s, const RotatedRect &roi) {
    if (s >= n_) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "stream index out of range");
    pending_rois_.emplace_back(s, roi);
}

// (Re)initialise for a frame size: every stream without RoI, each view a valid letterbox view of
// its own frame (the landmark network samples every stream's view each step), the detector's
// letterbox table and the frame sizes.
void DeviceFaceLoop::frame_size(uint32_t W, uint32_t H) {
    fw_ = W;
    fh_ = H;
    Rect lb;
    const ViewData lv = letterbox_view(W, H, det_->aspect(), &lb);
    const zr_view zv = to_zr_view(lv);
    check(zr_view_describe(&zv, 1, 0, &det_tmpl_));
    std::vector<float> l(4 * n_);
    std::vector<uint32_t> fs(2 * n_);
    std::vector<zr_view_desc> v(n_, det_tmpl_);
    std::vector<zr_track_state> st(n_, zr_track_state{});
    for (size_t i = 0; i < n_; i++) {
        l[4 * i] = lb.center().x;
        l[4 * i + 1] = lb.center().y;
        l[4 * i + 2] = lb.width();
        l[4 * i + 3] = lb.height();
        fs[2 * i] = W;
        fs[2 * i + 1] = H;
        v[i].frame = (uint32_t)i;
        st[i].frame_w = W;
        st[i].frame_h = H;
    }
    check(zr_memcpy_async(lbox_.ptr, l.data(), l.size() * 4, 0, stream_));
    check(zr_memcpy_async(fsize_.ptr, fs.data(), fs.size() * 4, 0, stream_));
    check(zr_memcpy_async(views_.ptr, v.data(), n_ * sizeof(zr_view_desc), 0, stream_));
    check(zr_memcpy_async(state_.ptr, st.data(), n_ * sizeof(zr_track_state), 0, stream_));
    check(zr_stream_synchronize(stream_));
}

void DeviceFaceLoop::step(const std::vector<Image> &frames) {
    if (frames.size() != n_) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "one frame per stream");
    std::vector<zr_frame> zf(n_);
    for (size_t i = 0; i < n_; i++) {
        const Image &f = frames[i];
        if (!f.on_device) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "face loop frames must be device-resident");
        if (f.width != frames[0].width || f.height != frames[0].height)
            throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "all streams share one frame size");
        zf[i] = zr_frame{f.rgba, f.width, f.height, f.row_stride};
    }
    if (frames[0].width != fw_ || frames[0].height != fh_) frame_size(frames[0].width, frames[0].height);
    if (!pending_rois_.empty()) {  // LandmarkTracker::set_roi: the state's RoI + its view
        check(zr_stream_synchronize(stream_));
        std::vector<zr_track_state> st(n_);
        check(zr_memcpy_async(st.data(), state_.ptr, n_ * sizeof(zr_track_state), 1, stream_));
        check(zr_stream_synchronize(stream_));
        for (const auto &[s, roi] : pending_rois_) {
            const Rect &r = roi.rect();
            st[s].roi[0] = r.center().x;
            st[s].roi[1] = r.center().y;
            st[s].roi[2] = r.width();
            st[s].roi[3] = r.height();
            st[s].roi[4] = roi.rotation_radians();
            st[s].active = 1;
        }
        pending_rois_.clear();
        // the seed pass derives every active state's view from its RoI; inactive ones keep theirs
        check(zr_memcpy_async(state_.ptr, st.data(), n_ * sizeof(zr_track_state), 0, stream_));
        std::vector<zr_view_desc> v(n_);
        check(zr_memcpy_async(v.data(), views_.ptr, n_ * sizeof(zr_view_desc), 1, stream_));
        check(zr_track_seed_async(state_.ptr, n_, &tcfg_, views_.ptr, stream_));
        check(zr_stream_synchronize(stream_));
        std::vector<zr_view_desc> seeded(n_);
        check(zr_memcpy_async(seeded.data(), views_.ptr, n_ * sizeof(zr_view_desc), 1, stream_));
        check(zr_stream_synchronize(stream_));
        for (size_t i = 0; i < n_; i++)
            if (!st[i].active) seeded[i] = v[i];
        check(zr_memcpy_async(views_.ptr, seeded.data(), n_ * sizeof(zr_view_desc), 0, stream_));
        check(zr_stream_synchronize(stream_));
    }
    // 1-2: tracker.track on every stream (LandmarkTracker::track_impl, landmark.rs:463-501)
    const NeuralNetwork &ln = lm_->nn();
    float *louts[4] = {lm_outs_[0].ptr, lm_outs_[1].ptr, lm_outs_[2].ptr, lm_outs_[3].ptr};
    const ColorMapper lc = lm_->color_mapper();
    check(zr_cnn_estimate_device_views_async(ln.handle(), zf.data(), n_, views_.ptr, n_, lc.lo, lc.hi, louts, stream_));
    check(zr_track_update_async(state_.ptr, n_, &tcfg_, lm_outs_[0].ptr, (size_t)ln.output_per_image(0),
                                lm_outs_[1].ptr, (size_t)ln.output_per_image(1), lm_out_.ptr, views_.ptr, stream_));
    // 3-4: detector.detect on the streams whose track returned None (facemesh.rs:43-47)
    check(zr_track_lost_compact_async(state_.ptr, n_, &det_tmpl_, due_.ptr, ndue_.ptr, due_views_.ptr,
                                      due_total_.ptr, stream_));
    float *douts[2] = {det_boxes_.ptr, det_logits_.ptr};
    const ColorMapper dc = det_->color_mapper();
    check(zr_cnn_estimate_device_views_count_async(det_->nn().handle(), zf.data(), n_, due_views_.ptr, n_, ndue_.ptr,
                                                   dc.lo, dc.hi, douts, stream_));
    check(zr_detect_post_mapped_async(det_logits_.ptr, det_boxes_.ptr, anchors_.ptr, lbox_.ptr, n_, due_.ptr,
                                      ndue_.ptr, &pcfg_, count_.ptr, dets_.ptr, dcap_, nullptr, stream_));
    // 5: tracker.set_roi(best.bounding_rect()) (facemesh.rs:49-54)
    check(zr_track_reseed_best_async(count_.ptr, dets_.ptr, dcap_, fsize_.ptr, n_, &tcfg_, state_.ptr, views_.ptr,
                                     reseeded_.ptr, stream_));
}

void DeviceFaceLoop::synchronize() {
    if (stream_) check(zr_stream_synchronize(stream_));
}

std::vector<zr_track_state> DeviceFaceLoop::states() {
    std::vector<zr_track_state> h(n_);
    check(zr_memcpy_async(h.data(), state_.ptr, n_ * sizeof(zr_track_state), 1, stream_));
    synchronize();
    return h;
}

std::vector<float> DeviceFaceLoop::landmarks() {
    std::vector<float> h(n_ * (size_t)lm_net_.num_landmarks * 3);
    check(zr_memcpy_async(h.data(), lm_out_.ptr, h.size() * 4, 1, stream_));
    synchronize();
    return h;
}

std::vector<int32_t> DeviceFaceLoop::detected() {
    int32_t nd = 0;
    std::vector<int32_t> due(n_), out(n_, 0);
    check(zr_memcpy_async(&nd, ndue_.ptr, 4, 1, stream_));
    check(zr_memcpy_async(due.data(), due_.ptr, n_ * 4, 1, stream_));
    synchronize();
    for (int32_t k = 0; k < nd && k < (int32_t)n_; k++) out[due[k]] = 1;
    return out;
}

std::vector<int32_t> DeviceFaceLoop::detection_counts() {
    std::vector<int32_t> ran = detected(), cnt(n_);
    check(zr_memcpy_async(cnt.data(), count_.ptr, n_ * 4, 1, stream_));
    synchronize();
    for (size_t s = 0; s < n_; s++)
        if (!ran[s]) cnt[s] = -1;
    return cnt;
}

uint64_t DeviceFaceLoop::reacquisitions() {
    uint64_t t = 0;
    check(zr_memcpy_async(&t, reseeded_.ptr, 8, 1, stream_));
    synchronize();
    return t;
}

uint64_t DeviceFaceLoop::detections_run() {
    uint64_t t = 0;
    check(zr_memcpy_async(&t, due_total_.ptr, 8, 1, stream_));
    synchronize();
    return t;
}

}  // namespace zh
