// device_hand_tracker.cpp -- see device_hand_tracker.h.
#include "device_hand_tracker.h"

#include <algorithm>

#include "device_tracker.h"
#include "hand_tracker.h"

namespace zh {

DeviceHandTracker::DeviceHandTracker(size_t streams, int slots, int device)
    : palm_(network_cnn(NetworkKind::PalmDetectionLite, device)),
      hand_(network_cnn(NetworkKind::HandLandmarkLite, device)) {
    if (streams == 0 || slots <= 0 || slots > 64) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "bad stream / slot count");
    n_ = streams;
    const AspectRatio a = hand_->aspect();
    cfg_.slots = slots;
    cfg_.iou_thresh = HandTracker::DEFAULT_IOU_THRESH;
    cfg_.palm_grow = HandTracker::PALM_GROW;
    cfg_.interval_ms = HandTracker::DEFAULT_REDETECT_INTERVAL_MS;
    cfg_.aspect_w = (int)a.w;
    cfg_.aspect_h = (int)a.h;
    tcfg_.kind = track_kind(hand_net_.kind);
    tcfg_.num_landmarks = hand_net_.num_landmarks;
    tcfg_.in_w = (int)hand_->input_width();
    tcfg_.in_h = (int)hand_->input_height();
    tcfg_.aspect_w = (int)a.w;
    tcfg_.aspect_h = (int)a.h;
    tcfg_.loss_thresh = LandmarkTracker::DEFAULT_LOSS_THRESHOLD;
    tcfg_.padding = HandTracker::ROI_PADDING;
    tcfg_.rois_per_frame = slots;
    pcfg_.face = 0;
    pcfg_.anchors = (int)palm_net_.anchors().size();
    pcfg_.params = palm_net_.params;
    pcfg_.keypoints = palm_net_.keypoints;
    pcfg_.in_w = (int)palm_->input_width();
    pcfg_.in_h = (int)palm_->input_height();
    pcfg_.thresh = Detector::DEFAULT_THRESHOLD;
    pcfg_.iou = NonMaxSuppression::DEFAULT_IOU_THRESH;
    dcap_ = palm_net_.anchors().size();
    check(zr_stream_create(&stream_));
    const size_t nv = n_ * (size_t)slots;
    state_.resize(nv);
    ids_.resize(nv);
    hroi_.resize(nv * 5);
    src_.resize(nv);
    views_.resize(nv);
    lm_out_.resize(nv * (size_t)hand_net_.num_landmarks * 3);
    nhands_.resize(n_);
    due_.resize(n_);
    due_views_.resize(n_);
    ndue_.resize(1);
    due_total_.resize(1);
    next_id_.resize(n_);
    next_det_.resize(n_);
    det_pending_.resize(n_);
    count_.resize(n_);
    dropped_.resize(n_);
    fsize_.resize(2 * n_);
    lbox_.resize(4 * n_);
    dets_.resize(n_ * dcap_ * 20);
    const NeuralNetwork &hn = hand_->nn();
    for (size_t k = 0; k < hn.num_outputs() && k < 4; k++) outs_[k].resize((size_t)hn.output_per_image(k) * nv);
    palm_boxes_.resize(n_ * (size_t)pcfg_.anchors * pcfg_.params);
    palm_logits_.resize(n_ * (size_t)pcfg_.anchors);
    const auto &an = palm_net_.anchors();
    anchors_.resize(2 * an.size());
    check(zr_memcpy_async(anchors_.ptr, an.data(), an.size() * sizeof(Vec2), 0, stream_));
    // no hands, no pending detection, ids from 0 (the state's `active` flags all clear)
    const std::vector<zr_track_state> zs(nv, zr_track_state{});
    check(zr_memcpy_async(state_.ptr, zs.data(), nv * sizeof(zr_track_state), 0, stream_));
    const std::vector<int32_t> zi(n_, 0);
    const std::vector<uint64_t> zl(n_, 0);
    check(zr_memcpy_async(nhands_.ptr, zi.data(), n_ * 4, 0, stream_));
    check(zr_memcpy_async(next_id_.ptr, zl.data(), n_ * 8, 0, stream_));
    check(zr_memcpy_async(det_pending_.ptr, zi.data(), n_ * 4, 0, stream_));
    check(zr_memcpy_async(count_.ptr, zi.data(), n_ * 4, 0, stream_));
    check(zr_memcpy_async(dropped_.ptr, zi.data(), n_ * 4, 0, stream_));
    check(zr_memcpy_async(due_total_.ptr, zl.data(), 8, 0, stream_));
    check(zr_stream_synchronize(stream_));  // the host vectors are pageable and go out of scope
    injected_.resize(n_);
}

DeviceHandTracker::~DeviceHandTracker() {
    if (stream_) {
        (void)zr_stream_synchronize(stream_);
        (void)zr_stream_destroy(stream_);
    }
}

void DeviceHandTracker::inject_detections(size_t s, const std::vector<Detection> &dets) {
    if (s >= n_) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "stream index out of range");
    for (const Detection &d : dets) injected_[s].push_back(d);
}

void DeviceHandTracker::step(const std::vector<Image> &frames, double now_ms) {
    if (frames.size() != n_) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "one frame per stream");
    std::vector<zr_frame> zf(n_);
    for (size_t i = 0; i < n_; i++) {
        const Image &f = frames[i];
        if (!f.on_device) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "tracker frames must be device-resident");
        if (i > 0 && (f.width != frames[0].width || f.height != frames[0].height))
            throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "all streams share one frame size");
        zf[i] = zr_frame{f.rgba, f.width, f.height, f.row_stride};
    }
    const uint32_t W = frames[0].width, H = frames[0].height;
    if (W != fw_ || H != fh_) {  // the letterbox views and frame sizes of this frame size
        fw_ = W;
        fh_ = H;
        Rect lb;
        (void)letterbox_view(W, H, palm_->aspect(), &lb);
        letterbox_.assign(n_, lb);
        std::vector<float> l(4 * n_);
        std::vector<uint32_t> fs(2 * n_);
        for (size_t i = 0; i < n_; i++) {
            l[4 * i] = lb.center().x;
            l[4 * i + 1] = lb.center().y;
            l[4 * i + 2] = lb.width();
            l[4 * i + 3] = lb.height();
            fs[2 * i] = W;
            fs[2 * i + 1] = H;
        }
        check(zr_memcpy_async(lbox_.ptr, l.data(), l.size() * 4, 0, stream_));
        check(zr_memcpy_async(fsize_.ptr, fs.data(), fs.size() * 4, 0, stream_));
        check(zr_stream_synchronize(stream_));
        const zr_view pv = to_zr_view(letterbox_view(W, H, palm_->aspect()));
        check(zr_view_describe(&pv, 1, 0, &palm_tmpl_));
        // every entry of the due-view table holds a valid view from the start (stream i's
        // letterbox): due_compact writes only the first ndue, and a palm preprocessing that does
        // not honour the device count (an unfused plan) samples all n_ entries
        std::vector<zr_view_desc> dv(n_, palm_tmpl_);
        for (size_t i = 0; i < n_; i++) dv[i].frame = (uint32_t)i;
        check(zr_memcpy_async(due_views_.ptr, dv.data(), n_ * sizeof(zr_view_desc), 0, stream_));
        check(zr_stream_synchronize(stream_));
    }
    // injected detections replace the palm result this step consumes (test hook)
    bool any = false;
    for (auto &v : injected_) any = any || !v.empty();
    if (any) {
        check(zr_stream_synchronize(stream_));
        std::vector<int32_t> cnt(n_), pend(n_);
        std::vector<float> d(n_ * dcap_ * 20, 0.f);
        check(zr_memcpy_async(cnt.data(), count_.ptr, n_ * 4, 1, stream_));
        check(zr_memcpy_async(pend.data(), det_pending_.ptr, n_ * 4, 1, stream_));
        check(zr_memcpy_async(d.data(), dets_.ptr, d.size() * 4, 1, stream_));
        check(zr_stream_synchronize(stream_));
        for (size_t s = 0; s < n_; s++) {
            if (injected_[s].empty()) continue;
            // the host tracker's order: the injected detections, then the finished palm result
            std::vector<float> palm;
            const int np = pend[s] ? std::min(cnt[s], (int32_t)dcap_) : 0;
            palm.assign(d.begin() + s * dcap_ * 20, d.begin() + (s * dcap_ + np) * 20);
            cnt[s] = 0;
            pend[s] = 1;
            for (const Detection &det : injected_[s]) {
                if ((size_t)cnt[s] >= dcap_) break;
                float *r = d.data() + (s * dcap_ + cnt[s]) * 20;
                std::fill(r, r + 20, 0.f);
                r[0] = det.confidence;
                r[1] = det.angle;
                r[2] = det.rect.center().x;
                r[3] = det.rect.center().y;
                r[4] = det.rect.width();
                r[5] = det.rect.height();
                cnt[s]++;
            }
            for (int k = 0; k < np && (size_t)cnt[s] < dcap_; k++, cnt[s]++)
                std::copy(palm.begin() + k * 20, palm.begin() + (k + 1) * 20, d.begin() + (s * dcap_ + cnt[s]) * 20);
            injected_[s].clear();
        }
        check(zr_memcpy_async(count_.ptr, cnt.data(), n_ * 4, 0, stream_));
        check(zr_memcpy_async(det_pending_.ptr, pend.data(), n_ * 4, 0, stream_));
        check(zr_memcpy_async(dets_.ptr, d.data(), d.size() * 4, 0, stream_));
        check(zr_stream_synchronize(stream_));
    }
    const size_t nv = n_ * (size_t)cfg_.slots;
    const NeuralNetwork &hn = hand_->nn();
    // 1. the previous step's estimates (tracking.rs:116-127: the workers' results)
    if (steps_ > 0)
        check(zr_track_update_async(state_.ptr, nv, &tcfg_, outs_[0].ptr, (size_t)hn.output_per_image(0), outs_[1].ptr,
                                    (size_t)hn.output_per_image(1), lm_out_.ptr, views_.ptr, stream_));
    // 2. bookkeeping (tracking.rs:129-218)
    check(zr_hand_manage_async(state_.ptr, ids_.ptr, hroi_.ptr, src_.ptr, nhands_.ptr, next_id_.ptr, next_det_.ptr,
                               det_pending_.ptr, count_.ptr, dets_.ptr, dcap_, fsize_.ptr, n_, &cfg_, now_ms,
                               steps_ == 0 ? 1 : 0, views_.ptr, dropped_.ptr, stream_));
    // 3. the hand landmark network on every slot's view of this frame
    float *outs[4] = {outs_[0].ptr, outs_[1].ptr, outs_[2].ptr, outs_[3].ptr};
    const ColorMapper hc = hand_->color_mapper();
    check(zr_cnn_estimate_device_views_async(hn.handle(), zf.data(), n_, views_.ptr, nv, hc.lo, hc.hi, outs, stream_));
    // 4. BlazePalm (Detector::detect_impl, detection.rs:224-267) on the streams step 2 asked to
    // detect on, taken next step: their list and count stay on the device
    float *pd[2] = {palm_boxes_.ptr, palm_logits_.ptr};
    if (palm_every_) {
        std::vector<zr_view> pv(n_);
        for (size_t i = 0; i < n_; i++) pv[i] = to_zr_view(letterbox_view(W, H, palm_->aspect()));
        std::vector<uint32_t> pvf(n_);
        for (size_t i = 0; i < n_; i++) pvf[i] = (uint32_t)i;
        palm_->estimate_async(std::vector<zr_frame>(zf.begin(), zf.end()), pv, pvf, pd, stream_);
        check(zr_detect_post_async(palm_logits_.ptr, palm_boxes_.ptr, anchors_.ptr, lbox_.ptr, n_, &pcfg_, count_.ptr,
                                   dets_.ptr, dcap_, nullptr, 0, 0, 1, nullptr, stream_));
        palm_frames_ += n_;
    } else {
        check(zr_due_compact_async(det_pending_.ptr, n_, &palm_tmpl_, due_.ptr, ndue_.ptr, due_views_.ptr, due_total_.ptr,
                                   stream_));
        const ColorMapper pc = palm_->color_mapper();
        check(zr_cnn_estimate_device_views_count_async(palm_->nn().handle(), zf.data(), n_, due_views_.ptr, n_, ndue_.ptr,
                                                       pc.lo, pc.hi, pd, stream_));
        check(zr_detect_post_mapped_async(palm_logits_.ptr, palm_boxes_.ptr, anchors_.ptr, lbox_.ptr, n_, due_.ptr,
                                          ndue_.ptr, &pcfg_, count_.ptr, dets_.ptr, dcap_, nullptr, stream_));
    }
    steps_++;
}

uint64_t DeviceHandTracker::palm_frames() {
    uint64_t due = 0;
    check(zr_memcpy_async(&due, due_total_.ptr, 8, 1, stream_));
    synchronize();
    return palm_frames_ + due;
}

void DeviceHandTracker::synchronize() {
    if (stream_) check(zr_stream_synchronize(stream_));
}

std::vector<int32_t> DeviceHandTracker::hand_counts() {
    std::vector<int32_t> h(n_);
    check(zr_memcpy_async(h.data(), nhands_.ptr, n_ * 4, 1, stream_));
    synchronize();
    return h;
}

std::vector<int32_t> DeviceHandTracker::dropped_hands() {
    std::vector<int32_t> h(n_);
    check(zr_memcpy_async(h.data(), dropped_.ptr, n_ * 4, 1, stream_));
    synchronize();
    return h;
}

std::vector<int32_t> DeviceHandTracker::dropped_detections() {
    std::vector<int32_t> h(n_);
    check(zr_memcpy_async(h.data(), count_.ptr, n_ * 4, 1, stream_));
    synchronize();
    for (auto &c : h) c = c > (int32_t)dcap_ ? c - (int32_t)dcap_ : 0;
    return h;
}

std::vector<int32_t> DeviceHandTracker::detection_pending() {
    std::vector<int32_t> h(n_);
    check(zr_memcpy_async(h.data(), det_pending_.ptr, n_ * 4, 1, stream_));
    synchronize();
    return h;
}

std::vector<DeviceHandTracker::HandData> DeviceHandTracker::hands(size_t s) {
    if (s >= n_) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "stream index out of range");
    const int H = cfg_.slots, L = hand_net_.num_landmarks;
    int32_t nh = 0;
    std::vector<uint64_t> ids(H);
    std::vector<int32_t> src(H);
    std::vector<float> roi(5 * H), lm((size_t)H * L * 3);
    std::vector<zr_track_state> st(H);
    check(zr_memcpy_async(&nh, nhands_.ptr + s, 4, 1, stream_));
    check(zr_memcpy_async(ids.data(), ids_.ptr + s * H, 8 * H, 1, stream_));
    check(zr_memcpy_async(src.data(), src_.ptr + s * H, 4 * H, 1, stream_));
    check(zr_memcpy_async(roi.data(), hroi_.ptr + s * H * 5, 20 * H, 1, stream_));
    check(zr_memcpy_async(lm.data(), lm_out_.ptr + (size_t)s * H * L * 3, lm.size() * 4, 1, stream_));
    synchronize();
    std::vector<HandData> out;
    for (int j = 0; j < nh; j++) {
        if (src[j] < 0) continue;  // started this step: no result yet (hand.lm is None)
        HandData d;
        d.id = ids[j];
        d.landmarks.assign(lm.begin() + (size_t)src[j] * L * 3, lm.begin() + (size_t)(src[j] + 1) * L * 3);
        d.view_rect = RotatedRect(Rect::from_center(roi[5 * j], roi[5 * j + 1], roi[5 * j + 2], roi[5 * j + 3]),
                                  roi[5 * j + 4]);
        out.push_back(std::move(d));
    }
    return out;
}

}  // namespace zh
