// hand_tracker.cpp -- see hand_tracker.h.
#include "hand_tracker.h"

#include <chrono>
#include <numeric>

namespace zh {

struct HandTracker::FrameBuf {
    DeviceArray<uint8_t> rgba;
    uint32_t w = 0, h = 0;
    int users = 0;  // in-flight launches that read it
};

namespace {
double steady_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}
}  // namespace

HandTracker::HandTracker(int device)
    : palm_(network_cnn(NetworkKind::PalmDetectionLite, device)),
      hand_(network_cnn(NetworkKind::HandLandmarkLite, device)) {
    check(zr_stream_create(&lm_stream_));
    check(zr_stream_create(&det_stream_));
    check(zr_event_create(&lm_done_));
    check(zr_event_create(&det_done_));
}

HandTracker::~HandTracker() {
    if (lm_stream_) zr_stream_synchronize(lm_stream_);
    if (det_stream_) zr_stream_synchronize(det_stream_);
    if (lm_done_) zr_event_destroy(lm_done_);
    if (det_done_) zr_event_destroy(det_done_);
    if (lm_stream_) zr_stream_destroy(lm_stream_);
    if (det_stream_) zr_stream_destroy(det_stream_);
}

std::vector<bool> HandTracker::filter_detections(const std::vector<Rect> &rois,
                                                 const std::vector<Detection> &dets, float t) {
    std::vector<bool> keep(dets.size(), true);
    for (size_t i = 0; i < dets.size(); i++) {
        const Rect grown = dets[i].rect.grow_rel(PALM_GROW);
        for (const Rect &r : rois)
            if (r.iou(grown) >= t) {  // hand.roi.rect().iou(&det.grow_rel(1.5)) (tracking.rs:142-148)
                keep[i] = false;
                break;
            }
    }
    return keep;
}

std::vector<size_t> HandTracker::dedupe_rois(const std::vector<Rect> &rois, float t) {
    std::vector<size_t> idx(rois.size());
    std::iota(idx.begin(), idx.end(), 0);
    // for i in (0..len).rev(): the range is fixed before the loop; swap_remove(i) moves the
    // last element into slot i, which the sweep does not revisit (tracking.rs:197-208)
    for (size_t i = rois.size(); i-- > 0;) {
        const Rect &roi = rois[idx[i]];
        for (size_t j = 0; j < i; j++)
            if (roi.iou(rois[idx[j]]) >= t) {
                idx[i] = idx.back();
                idx.pop_back();
                break;
            }
    }
    return idx;
}

HandTracker::FrameBuf *HandTracker::upload(const Image &img) {
    FrameBuf *fb = nullptr;
    for (auto &b : bufs_)
        if (b->users == 0) {
            fb = b.get();
            break;
        }
    if (!fb) {
        bufs_.push_back(std::make_unique<FrameBuf>());
        fb = bufs_.back().get();
    }
    const size_t row = (size_t)img.width * 4, bytes = row * img.height;
    fb->rgba.resize(bytes ? bytes : 4);
    fb->w = img.width;
    fb->h = img.height;
    const int kind = img.on_device ? 2 : 0;
    if (img.row_stride == row) {
        check(zr_memcpy_async(fb->rgba.ptr, img.rgba, bytes, kind, lm_stream_));
    } else {
        for (uint32_t y = 0; y < img.height; y++)
            check(zr_memcpy_async(fb->rgba.ptr + y * row, img.rgba + y * img.row_stride, row, kind, lm_stream_));
    }
    check(zr_stream_synchronize(lm_stream_));
    return fb;
}

void HandTracker::track(const Image &img) { track(img, steady_ms()); }

void HandTracker::track(const Image &img, double now) {
    if (!next_det_ms_) next_det_ms_ = now;
    // 1. results of the previous frame (PromiseHandle::block per hand)
    finish_landmarks();
    FrameBuf *fb = upload(img);
    // 2. finished palm detections, if any
    std::vector<Detection> dets = std::move(injected_);
    injected_.clear();
    if (det_running_ && zr_event_query(det_done_) == ZR_OK) collect_detection(dets);
    // 3. new hands from detections that overlap no tracked ROI
    std::vector<Rect> rois;
    for (const Hand &h : hands_) rois.push_back(h.roi.rect());
    const std::vector<bool> keep = filter_detections(rois, dets, iou_);
    for (size_t i = 0; i < dets.size(); i++) {
        if (!keep[i]) continue;
        Hand h;
        h.id = next_id_++;
        h.roi = RotatedRect(dets[i].rect.grow_rel(PALM_GROW), dets[i].angle);
        h.tracker_roi = h.roi;  // LandmarkTracker::set_roi, no padding (landmark.rs:438-440)
        hands_.push_back(std::move(h));
    }
    // 4. tracked regions that started to overlap
    rois.clear();
    for (const Hand &h : hands_) rois.push_back(h.roi.rect());
    std::vector<Hand> kept;
    for (size_t i : dedupe_rois(rois, iou_)) kept.push_back(std::move(hands_[i]));
    hands_.swap(kept);
    // 5. (re)detection
    if ((hands_.empty() || now >= *next_det_ms_) && !det_running_) {
        launch_detection(fb);
        *next_det_ms_ += det_interval_ms_;
    }
    // every tracked hand on this frame: one batched landmark launch sequence
    launch_landmarks(fb);
}

void HandTracker::finish_landmarks() {
    if (!lm_running_) return;
    check(zr_event_synchronize(lm_done_));
    lm_running_ = false;
    if (lm_frame_) {
        lm_frame_->users--;
        lm_frame_ = nullptr;
    }
    const uint32_t in_w = hand_->input_width();
    const size_t nout = hand_->nn().num_outputs();
    std::vector<Hand> kept;
    for (Hand &h : hands_) {
        if (!h.pending) {
            kept.push_back(std::move(h));
            continue;
        }
        h.pending = false;
        const float *outs[4] = {nullptr, nullptr, nullptr, nullptr};
        for (size_t k = 0; k < nout && k < 4; k++) outs[k] = h_lm_[k].ptr + h.slot * hand_->nn().output_per_image(k);
        // the hand worker's LandmarkTracker::track (tracking.rs:167-180, landmark.rs:463-501)
        Estimate e;
        extract_landmarks(hand_net_, outs, e);
        map_estimate(e, h.local_rect, in_w);
        TrackingResult res;
        RotatedRect next;
        if (!tracker_update(hand_net_, h.tracker_roi, h.view_rect, loss_, ROI_PADDING, e, res, next))
            continue;  // tracking lost: the hand is dropped
        h.roi = res.updated_roi;
        h.tracker_roi = next;
        h.lm = std::move(res.estimate);
        kept.push_back(std::move(h));
    }
    hands_.swap(kept);
}

void HandTracker::launch_landmarks(FrameBuf *fb) {
    if (hands_.empty()) return;
    const AspectRatio a = hand_->aspect();
    const ViewData full = ViewData::full(fb->w, fb->h);
    std::vector<zr_view> views;
    std::vector<uint32_t> vf;
    for (size_t i = 0; i < hands_.size(); i++) {
        Hand &h = hands_[i];
        h.view_rect = h.tracker_roi.grow_to_fit_aspect(a);  // landmark.rs:465-466
        const ViewData view = full.view(h.view_rect);
        h.local_rect = view.local_rect().grow_to_fit_aspect(a);  // landmark.rs:320-323
        views.push_back(to_zr_view(view.view(RotatedRect(h.local_rect, 0.f))));
        vf.push_back(0);
        h.slot = i;
        h.pending = true;
    }
    const size_t n = views.size(), nout = hand_->nn().num_outputs();
    std::vector<float *> d(nout);
    for (size_t k = 0; k < nout; k++) {
        const size_t cnt = (size_t)hand_->nn().output_per_image(k) * n;
        d_lm_[k].resize(cnt);
        h_lm_[k].resize(cnt);
        d[k] = d_lm_[k].ptr;
    }
    const std::vector<zr_frame> fr{zr_frame{fb->rgba.ptr, fb->w, fb->h, (uint64_t)fb->w * 4}};
    hand_->estimate_async(fr, views, vf, d.data(), lm_stream_);
    for (size_t k = 0; k < nout; k++)
        check(zr_memcpy_async(h_lm_[k].ptr, d[k], (size_t)hand_->nn().output_per_image(k) * n * 4, 1, lm_stream_));
    check(zr_event_record(lm_done_, lm_stream_));
    lm_running_ = true;
    lm_frame_ = fb;
    fb->users++;
}

void HandTracker::launch_detection(FrameBuf *fb) {
    const size_t A = palm_net_.anchors().size(), D = (size_t)palm_net_.params;
    d_boxes_.resize(A * D);
    d_logits_.resize(A);
    h_boxes_.resize(A * D);
    h_logits_.resize(A);
    const std::vector<zr_frame> fr{zr_frame{fb->rgba.ptr, fb->w, fb->h, (uint64_t)fb->w * 4}};
    // Detector::detect_impl's letterbox view (detection.rs:224-227)
    const std::vector<zr_view> v{to_zr_view(letterbox_view(fb->w, fb->h, palm_->aspect(), &det_letterbox_))};
    const std::vector<uint32_t> vf{0};
    float *d[2] = {d_boxes_.ptr, d_logits_.ptr};
    palm_->estimate_async(fr, v, vf, d, det_stream_);
    check(zr_memcpy_async(h_boxes_.ptr, d_boxes_.ptr, A * D * 4, 1, det_stream_));
    check(zr_memcpy_async(h_logits_.ptr, d_logits_.ptr, A * 4, 1, det_stream_));
    check(zr_event_record(det_done_, det_stream_));
    det_running_ = true;
    det_frame_ = fb;
    fb->users++;
}

void HandTracker::collect_detection(std::vector<Detection> &out) {
    check(zr_event_synchronize(det_done_));
    det_running_ = false;
    if (det_frame_) {
        det_frame_->users--;
        det_frame_ = nullptr;
    }
    // the palm worker's Detector::detect (detection.rs:231-267)
    std::vector<Detection> raw;
    palm_net_.extract(h_boxes_.ptr, h_logits_.ptr, Detector::DEFAULT_THRESHOLD, palm_->input_width(),
                      palm_->input_height(), raw);
    std::vector<Detection> dets = nms_.process(raw);
    map_detections(dets, det_letterbox_, palm_->input_width());
    for (auto &d : dets) out.push_back(std::move(d));
}

void HandTracker::wait_detection() {
    if (det_running_) check(zr_event_synchronize(det_done_));
}

void HandTracker::inject_detections(std::vector<Detection> dets) {
    for (auto &d : dets) injected_.push_back(std::move(d));
}

std::vector<HandTracker::HandData> HandTracker::hands() const {
    std::vector<HandData> out;
    for (const Hand &h : hands_)
        if (h.lm) out.push_back({h.id, *h.lm, h.roi});
    return out;
}

}  // namespace zh
