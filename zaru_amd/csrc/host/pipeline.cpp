// pipeline.cpp -- see pipeline.h.
#include "pipeline.h"

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>

namespace zh {

// ---------------------------------------------------------------- thread pool
struct ThreadPool::Impl {
    std::mutex mu;
    std::condition_variable cv, done_cv;
    const std::function<void(size_t)> *fn = nullptr;
    size_t n = 0;
    std::atomic<size_t> next{0};
    uint64_t generation = 0;
    int busy = 0;
    bool stop = false;

    void work() {
        for (;;) {
            size_t i = next.fetch_add(1);
            if (i >= n) break;
            (*fn)(i);
        }
    }
};

ThreadPool::ThreadPool(int n) : impl_(new Impl) {
    for (int t = 1; t < std::max(1, n); t++)
        workers_.emplace_back([this] {
            Impl &I = *impl_;
            uint64_t seen = 0;
            for (;;) {
                {
                    std::unique_lock<std::mutex> lk(I.mu);
                    I.cv.wait(lk, [&] { return I.stop || I.generation != seen; });
                    if (I.stop) return;
                    seen = I.generation;
                    I.busy++;
                }
                I.work();
                {
                    std::lock_guard<std::mutex> lk(I.mu);
                    if (--I.busy == 0) I.done_cv.notify_all();
                }
            }
        });
}

ThreadPool::~ThreadPool() {
    {
        std::lock_guard<std::mutex> lk(impl_->mu);
        impl_->stop = true;
    }
    impl_->cv.notify_all();
    for (auto &t : workers_) t.join();
}

void ThreadPool::parallel_for(size_t n, const std::function<void(size_t)> &fn) {
    if (n == 0) return;
    Impl &I = *impl_;
    if (workers_.empty() || n == 1) {
        for (size_t i = 0; i < n; i++) fn(i);
        return;
    }
    {
        std::lock_guard<std::mutex> lk(I.mu);
        I.fn = &fn;
        I.n = n;
        I.next = 0;
        I.generation++;
    }
    I.cv.notify_all();
    I.work();
    std::unique_lock<std::mutex> lk(I.mu);
    I.done_cv.wait(lk, [&] { return I.busy == 0 && I.next.load() >= I.n; });
    I.fn = nullptr;
}

// ---------------------------------------------------------------- pipeline
PipelineConfig PipelineConfig::face() {
    PipelineConfig c;
    c.detector = DetectorNetwork::short_range_face();
    c.landmarker = LandmarkNetwork::face_mesh_v1();
    c.roi_grow = 0.f;        // tracker.set_roi(detection.bounding_rect()) (examples/facemesh.rs:49-54)
    c.roi_use_angle = false;
    c.roi_padding = LandmarkTracker::DEFAULT_ROI_PADDING;
    return c;
}

PipelineConfig PipelineConfig::hand() {
    PipelineConfig c;
    c.detector = DetectorNetwork::palm_lite();
    c.landmarker = LandmarkNetwork::hand_lite();
    c.roi_grow = 1.5f;       // palm -> hand (hand/tracking.rs:136,159)
    c.roi_use_angle = true;
    c.roi_padding = 0.4f;    // hand/tracking.rs:34
    return c;
}

DetectTrackPipeline::DetectTrackPipeline(PipelineConfig cfg, int device, int threads)
    : cfg_(std::move(cfg)), device_(device), det_cnn_(network_cnn(cfg_.detector.kind, device)),
      lm_cnn_(network_cnn(cfg_.landmarker.kind, device)), pool_(threads) {
    nms_.set_iou_thresh(cfg_.nms_iou);
    check(zr_stream_create(&stream_));
}

DetectTrackPipeline::~DetectTrackPipeline() {
    if (stream_) zr_stream_destroy(stream_);
}

static double session_stat(const Cnn &c, bool flops) {
    double b = 0, f = 0;
    size_t n = 0;
    check(zr_session_stats(c.nn().handle(), &b, &f, &n));
    return flops ? f : b;
}
double DetectTrackPipeline::detector_bytes_per_image() const { return session_stat(*det_cnn_, false); }
double DetectTrackPipeline::landmarker_bytes_per_image() const { return session_stat(*lm_cnn_, false); }
double DetectTrackPipeline::detector_flops_per_image() const { return session_stat(*det_cnn_, true); }
double DetectTrackPipeline::landmarker_flops_per_image() const { return session_stat(*lm_cnn_, true); }

void DetectTrackPipeline::profile(bool on) {
    check(zr_profile_enable(det_cnn_->nn().handle(), on ? 1 : 0));
    check(zr_profile_enable(lm_cnn_->nn().handle(), on ? 1 : 0));
}

std::string DetectTrackPipeline::profile_read() {
    std::string out;
    const std::pair<const char *, const Cnn *> nets[2] = {{"detector", det_cnn_.get()}, {"landmarker", lm_cnn_.get()}};
    std::vector<char> buf(1 << 16);
    for (auto &nc : nets) {
        // reading clears the records, so read once into a generous buffer
        size_t need = 0;
        check(zr_profile_read(nc.second->nn().handle(), buf.data(), buf.size(), &need));
        const std::string txt(buf.data());
        size_t pos = 0;
        while (pos < txt.size()) {
            size_t e = txt.find('\n', pos);
            if (e == std::string::npos) e = txt.size();
            if (e > pos) out += std::string(nc.first) + "/" + txt.substr(pos, e - pos) + "\n";
            pos = e + 1;
        }
    }
    return out;
}

namespace {
using clk = std::chrono::steady_clock;
double ms_since(clk::time_point t) {
    return std::chrono::duration<double, std::milli>(clk::now() - t).count();
}
}  // namespace

void DetectTrackPipeline::run(const std::vector<Image> &frames,
                              const std::vector<std::vector<RotatedRect>> &forced) {
    const auto t0 = clk::now();
    const size_t B = frames.size();
    times_ = StageTimes{};
    times_.frames = B;
    dets_.assign(B, {});
    rois_.clear();
    if (B == 0) return;

    const Cnn &dc = *det_cnn_;
    const uint32_t din_w = dc.input_width(), din_h = dc.input_height();
    const auto &anchors = cfg_.detector.anchors();
    const uint32_t A = (uint32_t)anchors.size(), D = (uint32_t)cfg_.detector.params;
    const uint32_t cap = cfg_.candidate_cap, rec_w = 2 + D;

    // ---- stage 1: letterbox views of every frame -> detector (one batched launch chain)
    std::vector<zr_frame> zf(B);
    std::vector<zr_view> zv(B);
    std::vector<uint32_t> vf(B);
    std::vector<Rect> letterbox(B);
    for (size_t f = 0; f < B; f++) {
        if (!frames[f].on_device) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "pipeline frames must be device-resident");
        zf[f] = zr_frame{frames[f].rgba, frames[f].width, frames[f].height, frames[f].row_stride};
        zv[f] = to_zr_view(letterbox_view(frames[f].width, frames[f].height, dc.aspect(), &letterbox[f]));
        vf[f] = (uint32_t)f;
    }
    d_boxes_.resize((size_t)B * A * D);
    d_logits_.resize((size_t)B * A);
    d_count_.resize(B);
    d_rec_.resize((size_t)B * cap * rec_w);
    float *douts[2] = {d_boxes_.ptr, d_logits_.ptr};
    dc.estimate_async(zf, zv, vf, douts, stream_);
    const float floor = candidate_logit_floor(cfg_.det_threshold);
    check(zr_detection_candidates_async(d_logits_.ptr, d_boxes_.ptr, (uint32_t)B, A, D, floor, cap,
                                        d_count_.ptr, d_rec_.ptr, stream_));
    h_count_.resize(B);
    h_rec_.resize((size_t)B * cap * rec_w);
    check(zr_memcpy_async(h_count_.data(), d_count_.ptr, B * sizeof(int32_t), 1, stream_));
    check(zr_memcpy_async(h_rec_.data(), d_rec_.ptr, h_rec_.size() * sizeof(float), 1, stream_));
    check(zr_stream_synchronize(stream_));
    times_.detect_gpu_ms = ms_since(t0);

    // ---- stage 2: exact decode + NMS + map to image coordinates (host, per frame)
    const auto t1 = clk::now();
    std::vector<size_t> overflow;
    for (size_t f = 0; f < B; f++)
        if ((uint32_t)h_count_[f] > cap) overflow.push_back(f);
    std::vector<std::vector<float>> full_boxes(B), full_logits(B);
    for (size_t f : overflow) {  // rare: more candidates than slots -> copy that frame whole
        full_boxes[f].resize((size_t)A * D);
        full_logits[f].resize(A);
        check(zr_memcpy_async(full_boxes[f].data(), d_boxes_.ptr + f * A * D, (size_t)A * D * 4, 1, stream_));
        check(zr_memcpy_async(full_logits[f].data(), d_logits_.ptr + f * A, (size_t)A * 4, 1, stream_));
    }
    if (!overflow.empty()) check(zr_stream_synchronize(stream_));
    const float thresh = cfg_.det_threshold;
    pool_.parallel_for(B, [&](size_t f) {
        std::vector<Detection> raw;
        if (!full_logits[f].empty()) {
            cfg_.detector.extract(full_boxes[f].data(), full_logits[f].data(), thresh, din_w, din_h, raw);
        } else {
            const int n = h_count_[f];
            const float *rec = &h_rec_[f * cap * rec_w];
            std::vector<std::pair<uint32_t, int>> order;  // restore anchor order
            for (int i = 0; i < n; i++) {
                uint32_t a;
                std::memcpy(&a, &rec[i * rec_w], 4);
                order.push_back({a, i});
            }
            std::sort(order.begin(), order.end());
            for (auto &o : order) {
                const float *r = &rec[o.second * rec_w];
                const float conf = sigmoid(r[1]);
                if (conf < thresh) continue;
                raw.push_back(cfg_.detector.decode(o.first, r + 2, conf, din_w, din_h));
            }
        }
        dets_[f] = nms_.process(raw);
        map_detections(dets_[f], letterbox[f], din_w);
    });
    times_.decode_nms_ms = ms_since(t1);

    // ---- stage 3: ROIs -> landmark network (one batched launch chain over all ROIs)
    const auto t2 = clk::now();
    const Cnn &lc = *lm_cnn_;
    const AspectRatio la = lc.aspect();
    std::vector<zr_view> rv;
    std::vector<uint32_t> rf;
    std::vector<Rect> local_rect;
    for (size_t f = 0; f < B; f++) {
        std::vector<std::pair<RotatedRect, bool>> seeds;
        for (const auto &d : dets_[f]) {
            if (seeds.size() >= cfg_.max_rois_per_frame) break;
            seeds.push_back({RotatedRect(cfg_.roi_grow > 0.f ? d.rect.grow_rel(cfg_.roi_grow) : d.rect,
                                         cfg_.roi_use_angle ? d.angle : 0.f), true});
        }
        if (seeds.empty() && f < forced.size())
            for (const auto &r : forced[f]) {
                if (seeds.size() >= cfg_.max_rois_per_frame) break;
                seeds.push_back({r, false});
            }
        const ViewData full = ViewData::full(frames[f].width, frames[f].height);
        for (const auto &s : seeds) {
            RoiResult r;
            r.frame = (uint32_t)f;
            r.from_detection = s.second;
            r.roi = s.first;
            // LandmarkTracker::track_impl (landmark.rs:465-467) + Estimator (landmark.rs:320-323)
            r.result.view_rect = s.first.grow_to_fit_aspect(la);
            const ViewData view = full.view(r.result.view_rect);
            const Rect rect = view.local_rect().grow_to_fit_aspect(la);
            rv.push_back(to_zr_view(view.view(RotatedRect(rect, 0.f))));
            rf.push_back((uint32_t)f);
            local_rect.push_back(rect);
            rois_.push_back(r);
        }
    }
    const size_t R = rois_.size();
    times_.rois = R;
    for (auto &d : dets_) times_.detections += d.size();
    const size_t nout = lc.nn().num_outputs();
    if (R > 0) {
        std::vector<float *> lptr(nout);
        for (size_t i = 0; i < nout; i++) {
            d_lm_[i].resize((size_t)lc.nn().output_per_image(i) * R);
            lptr[i] = d_lm_[i].ptr;
        }
        lc.estimate_async(zf, rv, rf, lptr.data(), stream_);
        for (size_t i = 0; i < nout; i++) {
            h_lm_[i].resize((size_t)lc.nn().output_per_image(i) * R);
            check(zr_memcpy_async(h_lm_[i].data(), lptr[i], h_lm_[i].size() * 4, 1, stream_));
        }
        check(zr_stream_synchronize(stream_));
    }
    times_.landmark_gpu_ms = ms_since(t2);

    // ---- stage 4: extract + Estimator map-out + tracker update (host, per ROI)
    const auto t3 = clk::now();
    const uint32_t lin_w = lc.input_width();
    std::atomic<size_t> tracked{0};
    pool_.parallel_for(R, [&](size_t i) {
        RoiResult &r = rois_[i];
        const float *outs[4];
        for (size_t k = 0; k < nout; k++) outs[k] = &h_lm_[k][i * lc.nn().output_per_image(k)];
        Estimate e;
        extract_landmarks(cfg_.landmarker, outs, e);
        map_estimate(e, local_rect[i], lin_w);
        r.tracked = tracker_update(cfg_.landmarker, r.roi, r.result.view_rect, cfg_.loss_threshold,
                                   cfg_.roi_padding, e, r.result, r.next_roi);
        if (!r.tracked) r.result.estimate = std::move(e);
        else tracked++;
    });
    times_.tracked = tracked.load();
    times_.map_ms = ms_since(t3);
    times_.total_ms = ms_since(t0);
}

}  // namespace zh
