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
    nms_.set_mode(cfg_.nms_mode);
    if (cfg_.device_post) {
        // 0: the detector's anchor count, the most NMS can return (nothing dropped)
        if (cfg_.det_cap == 0) cfg_.det_cap = (uint32_t)cfg_.detector.anchors().size();
        if (cfg_.det_cap < cfg_.max_rois_per_frame) cfg_.det_cap = cfg_.max_rois_per_frame;
        const auto &a = cfg_.detector.anchors();
        d_anchors_.resize(2 * a.size());
        check(zr_memcpy_async(d_anchors_.ptr, a.data(), a.size() * sizeof(Vec2), 0, nullptr));
        check(zr_stream_synchronize(nullptr));
    }
    check(zr_stream_create(&stream_));
    // every slot enqueues on the one pipeline stream (the GPU runs the kernels back to back,
    // so per-kernel timings stay clean); the host waits on per-slot events instead
    for (uint32_t i = 0; i < std::max(1u, cfg_.sub_batches); i++) {
        slots_.push_back(std::make_unique<Slot>());
        Slot &s = *slots_.back();
        if (cfg_.stream_per_sub_batch && i > 0) check(zr_stream_create(&s.stream));
        else s.stream = stream_;
        check(zr_event_create(&s.ev_det));
        check(zr_event_create(&s.ev_lm));
        check(zr_event_create(&s.ev_rec));
        for (auto &e : s.ev_t) check(zr_event_create_timing(&e));
    }
}

DetectTrackPipeline::~DetectTrackPipeline() {
    for (auto &s : slots_) {
        if (s->stream) zr_stream_synchronize(s->stream);
        if (s->stream && s->stream != stream_) zr_stream_destroy(s->stream);
        if (s->ev_det) zr_event_destroy(s->ev_det);
        if (s->ev_lm) zr_event_destroy(s->ev_lm);
        if (s->ev_rec) zr_event_destroy(s->ev_rec);
        for (auto e : s->ev_t)
            if (e) zr_event_destroy(e);
    }
    if (gstream_) {
        zr_stream_synchronize(gstream_);
        zr_stream_destroy(gstream_);
    }
    for (auto e : ev_gath_)
        if (e) zr_event_destroy(e);
    if (stream_) zr_stream_destroy(stream_);
}

size_t DetectTrackPipeline::det_cap() const { return cfg_.det_cap; }

void DetectTrackPipeline::enable_records(uint32_t rmax, uint32_t first_id, uint32_t id_stride, zr_comm *comm,
                                         int world) {
    if (!cfg_.device_post) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "device records need device post-processing");
    if (rmax == 0 || rmax > 64 || world < 1) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "bad record configuration");
    if (comm) {
        // the all-gather writes the communicator's nranks * bytes into a world-sized block
        int nranks = 0;
        check(zr_comm_size(comm, &nranks));
        if (nranks != world)
            throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "world (" + std::to_string(world) + ") is not the communicator's rank count (" +
                                                         std::to_string(nranks) + ")");
    }
    if (gstream_) check(zr_stream_synchronize(gstream_));
    rec_rmax_ = rmax;
    rec_first_ = first_id;
    rec_stride_ = id_stride;
    comm_ = comm;
    world_ = comm ? world : 1;
    // the gather runs on its own stream: with the sub-batch streams that is 4 hardware queues,
    // the HIP default (GPU_MAX_HW_QUEUES), and the null stream stays idle in the steady state
    if (!gstream_) check(zr_stream_create(&gstream_));
    for (int k = 0; k < 2; k++) {
        if (!ev_gath_[k]) check(zr_event_create(&ev_gath_[k]));
        gath_used_[k] = false;
    }
}

// every active slot has enqueued step enq_steps_ (its records into set enq_steps_ & 1): the gather
// stream waits for their post-processing, all-gathers the set (with a communicator) and marks it
void DetectTrackPipeline::enqueue_gather() {
    if (!rec_rmax_) return;
    const int set = (int)(enq_steps_ & 1);
    for (size_t k = 0; k < active_slots_; k++) check(zr_stream_wait_event(gstream_, slots_[k]->ev_rec));
    if (comm_) {
        const size_t bytes = frames_.size() * record_width() * sizeof(float);
        d_gath_[set].resize((size_t)world_ * frames_.size() * record_width());
        check(zr_comm_all_gather_async(comm_, d_rec_[set].ptr, d_gath_[set].ptr, bytes, gstream_));
    }
    check(zr_event_record(ev_gath_[set], gstream_));
    gath_used_[set] = true;
    enq_steps_++;
}

std::vector<float> DetectTrackPipeline::records() {
    if (!rec_rmax_ || done_steps_ == 0) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "no finished step with records");
    const int set = (int)((done_steps_ - 1) & 1);
    check(zr_event_synchronize(ev_gath_[set]));
    std::vector<float> out(frames_.size() * record_width());
    check(zr_memcpy_async(out.data(), d_rec_[set].ptr, out.size() * 4, 1, nullptr));
    check(zr_stream_synchronize(nullptr));
    return out;
}

std::vector<float> DetectTrackPipeline::gathered() {
    if (!comm_ || done_steps_ == 0) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "no gathered step (no communicator)");
    const int set = (int)((done_steps_ - 1) & 1);
    check(zr_event_synchronize(ev_gath_[set]));
    std::vector<float> out((size_t)world_ * frames_.size() * record_width());
    check(zr_memcpy_async(out.data(), d_gath_[set].ptr, out.size() * 4, 1, nullptr));
    check(zr_stream_synchronize(nullptr));
    return out;
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

void DetectTrackPipeline::set_frames(std::vector<Image> frames, std::vector<std::vector<RotatedRect>> forced) {
    frames_ = std::move(frames);
    forced_ = std::move(forced);
    for (auto &s : slots_) s->inputs_ok = false;
}

namespace {
using clk = std::chrono::steady_clock;
double ms_since(clk::time_point t) {
    return std::chrono::duration<double, std::milli>(clk::now() - t).count();
}
}  // namespace

// stage 1 (enqueue only): letterbox views -> detector -> candidate compaction -> D2H
void DetectTrackPipeline::stage_detect(Slot &s, const std::vector<Image> &frames) {
    const Cnn &dc = *det_cnn_;
    const uint32_t A = (uint32_t)cfg_.detector.anchors().size(), D = (uint32_t)cfg_.detector.params;
    const uint32_t cap = cfg_.candidate_cap, rec_w = 2 + D;
    const size_t n = s.nf;
    s.zf.resize(n);
    s.letterbox.resize(n);
    std::vector<zr_view> zv(n);
    std::vector<uint32_t> vf(n);
    for (size_t i = 0; i < n; i++) {
        const Image &im = frames[s.f0 + i];
        if (!im.on_device) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "pipeline frames must be device-resident");
        s.zf[i] = zr_frame{im.rgba, im.width, im.height, im.row_stride};
        zv[i] = to_zr_view(letterbox_view(im.width, im.height, dc.aspect(), &s.letterbox[i]));
        vf[i] = (uint32_t)i;
    }
    s.d_boxes.resize(n * A * D);
    s.d_logits.resize(n * A);
    s.d_count.resize(n);
    s.d_rec.resize(n * cap * rec_w);
    float *douts[2] = {s.d_boxes.ptr, s.d_logits.ptr};
    if (cfg_.device_post) check(zr_event_record(s.ev_t[0], s.stream));
    dc.estimate_async(s.zf, zv, vf, douts, s.stream);
    if (cfg_.device_post) {  // stage_device_post continues on the stream
        check(zr_event_record(s.ev_t[1], s.stream));
        return;
    }
    check(zr_detection_candidates_async(s.d_logits.ptr, s.d_boxes.ptr, (uint32_t)n, A, D,
                                        candidate_logit_floor(cfg_.det_threshold), cap, s.d_count.ptr,
                                        s.d_rec.ptr, s.stream));
    s.h_count.resize(n);
    s.h_rec.resize(n * cap * rec_w);
    check(zr_memcpy_async(s.h_count.data(), s.d_count.ptr, n * sizeof(int32_t), 1, s.stream));
    check(zr_memcpy_async(s.h_rec.data(), s.d_rec.ptr, n * cap * rec_w * sizeof(float), 1, s.stream));
    check(zr_event_record(s.ev_det, s.stream));
}

zr_track_cfg DetectTrackPipeline::track_cfg() const {
    const Cnn &lc = *lm_cnn_;
    zr_track_cfg c{};
    c.kind = track_kind(cfg_.landmarker.kind);
    c.num_landmarks = cfg_.landmarker.num_landmarks;
    c.in_w = (int)lc.input_width();
    c.in_h = (int)lc.input_height();
    c.aspect_w = (int)lc.aspect().w;
    c.aspect_h = (int)lc.aspect().h;
    c.loss_thresh = cfg_.loss_threshold;
    c.padding = cfg_.roi_padding;
    c.rois_per_frame = (int)std::max(1u, cfg_.max_rois_per_frame);
    return c;
}

// device mode, enqueued right behind stage 1 on the slot's stream: decode + NMS + map
// (zr_detect_post_async), the ROI seeds and their views (zr_track_seed_detections_async), the
// landmark network on those views and the tracker update (zr_track_update_async), then one copy
// of the step's summary to the host.  ROI slot k of frame f is detection k (NMS order) or, when
// the frame has none, forced ROI k -- the host mode's seeds -- else idle.
void DetectTrackPipeline::stage_device_post(Slot &s, const std::vector<Image> &frames,
                                            const std::vector<std::vector<RotatedRect>> &forced) {
    const Cnn &dc = *det_cnn_, &lc = *lm_cnn_;
    const size_t n = s.nf, R = std::max(1u, cfg_.max_rois_per_frame), dcap = cfg_.det_cap;
    const size_t nv = n * R, nout = lc.nn().num_outputs();
    const int L = cfg_.landmarker.num_landmarks;
    const uint32_t A = (uint32_t)cfg_.detector.anchors().size(), D = (uint32_t)cfg_.detector.params;
    if (!s.inputs_ok) {  // letterbox rects, frame sizes, forced ROIs: fixed for a frame set
        s.h_lbox.resize(4 * n);
        s.h_fsize.resize(2 * n);
        s.h_forced.resize(5 * nv);
        s.h_nforced.resize(n);
        for (size_t i = 0; i < n; i++) {
            const size_t f = s.f0 + i;
            const Rect &r = s.letterbox[i];
            s.h_lbox[4 * i] = r.center().x;
            s.h_lbox[4 * i + 1] = r.center().y;
            s.h_lbox[4 * i + 2] = r.width();
            s.h_lbox[4 * i + 3] = r.height();
            s.h_fsize[2 * i] = frames[f].width;
            s.h_fsize[2 * i + 1] = frames[f].height;
            const size_t nf = f < forced.size() ? std::min(R, forced[f].size()) : 0;
            s.h_nforced[i] = (int32_t)nf;
            for (size_t k = 0; k < nf; k++) {
                const RotatedRect &q = forced[f][k];
                float *o = &s.h_forced[5 * (i * R + k)];
                o[0] = q.rect().center().x;
                o[1] = q.rect().center().y;
                o[2] = q.rect().width();
                o[3] = q.rect().height();
                o[4] = q.rotation_radians();
            }
        }
        s.d_lbox.resize(4 * n);
        s.d_fsize.resize(2 * n);
        s.d_forced.resize(5 * nv);
        s.d_nforced.resize(n);
        check(zr_memcpy_async(s.d_lbox.ptr, s.h_lbox.ptr, 4 * n * 4, 0, s.stream));
        check(zr_memcpy_async(s.d_fsize.ptr, s.h_fsize.ptr, 2 * n * 4, 0, s.stream));
        check(zr_memcpy_async(s.d_forced.ptr, s.h_forced.ptr, 5 * nv * 4, 0, s.stream));
        check(zr_memcpy_async(s.d_nforced.ptr, s.h_nforced.ptr, n * 4, 0, s.stream));
        s.inputs_ok = true;
    }
    Slot::Results &o = s.res[s.wr];
    const size_t sum_bytes = 2 * nv * sizeof(zr_track_state) + 3 * n * sizeof(int32_t);  // + count, ties
    o.sum.resize(sum_bytes);
    o.h_sum.resize(sum_bytes);
    o.dets.resize(n * dcap * 20);
    o.lmout.resize(nv * L * 3);
    zr_track_state *d_state = reinterpret_cast<zr_track_state *>(o.sum.ptr);
    zr_track_state *d_seed = d_state + nv;
    int32_t *d_count = reinterpret_cast<int32_t *>(d_seed + nv);
    int32_t *d_ties = d_count + n;
    s.d_views.resize(nv);
    zr_detpost_cfg pc{};
    pc.face = is_face_detector(cfg_.detector.kind) ? 1 : 0;
    pc.anchors = (int)A;
    pc.params = (int)D;
    pc.keypoints = cfg_.detector.keypoints;
    pc.in_w = (int)dc.input_width();
    pc.in_h = (int)dc.input_height();
    pc.thresh = cfg_.det_threshold;
    pc.iou = cfg_.nms_iou;
    pc.mode = cfg_.nms_mode == SuppressionMode::Remove ? 1 : 0;
    float *rec = nullptr;
    const bool records = rec_rmax_ && &frames == &frames_;  // (records cover the resident frame set)
    if (records) {  // this step's set of the all-gather records, frames f0 ..
        const int set = (int)(enq_steps_ & 1);
        d_rec_[set].resize(frames_.size() * record_width());
        // the set's previous gather (two steps ago) must have read it before it is rewritten
        if (gath_used_[set]) check(zr_stream_wait_event(s.stream, ev_gath_[set]));
        rec = d_rec_[set].ptr + s.f0 * record_width();
    }
    check(zr_detect_post_async(s.d_logits.ptr, s.d_boxes.ptr, d_anchors_.ptr, s.d_lbox.ptr, n, &pc, d_count,
                               o.dets.ptr, dcap, rec, rec_rmax_, rec_first_ + (uint32_t)s.f0 * rec_stride_,
                               rec_stride_, d_ties, s.stream));
    if (records) check(zr_event_record(s.ev_rec, s.stream));
    const zr_track_cfg tc = track_cfg();
    check(zr_track_seed_detections_async(d_count, o.dets.ptr, dcap, s.d_forced.ptr, s.d_nforced.ptr, s.d_fsize.ptr,
                                         n, &tc, cfg_.roi_grow, cfg_.roi_use_angle ? 1 : 0, d_state, d_seed,
                                         s.d_views.ptr, s.stream));
    check(zr_event_record(s.ev_t[2], s.stream));
    float *lptr[4] = {nullptr, nullptr, nullptr, nullptr};
    for (size_t k = 0; k < nout && k < 4; k++) {
        o.lm[k].resize((size_t)lc.nn().output_per_image(k) * nv);
        lptr[k] = o.lm[k].ptr;
    }
    const ColorMapper cm = lc.color_mapper();
    check(zr_cnn_estimate_device_views_async(lc.nn().handle(), s.zf.data(), n, s.d_views.ptr, nv, cm.lo, cm.hi, lptr,
                                             s.stream));
    check(zr_event_record(s.ev_t[3], s.stream));
    const bool flagged = tc.kind <= 2;
    check(zr_track_update_async(d_state, nv, &tc, lptr[0], (size_t)lc.nn().output_per_image(0),
                                flagged ? lptr[1] : nullptr, flagged ? (size_t)lc.nn().output_per_image(1) : 0,
                                o.lmout.ptr, s.d_views.ptr, s.stream));
    check(zr_event_record(s.ev_t[4], s.stream));
    check(zr_memcpy_async(o.h_sum.ptr, o.sum.ptr, sum_bytes, 1, s.stream));
    check(zr_event_record(s.ev_lm, s.stream));
    s.timed = true;
    s.wr ^= 1;  // the next step of this slot writes the other set
}

void DetectTrackPipeline::finish_device(Slot &s) {
    s.done = s.wr ^ 1;
    const Slot::Results &o = s.res[s.done];
    const size_t n = s.nf, R = std::max(1u, cfg_.max_rois_per_frame), nv = n * R;
    const zr_track_state *st = reinterpret_cast<const zr_track_state *>(o.h_sum.ptr);
    const int32_t *cnt = reinterpret_cast<const int32_t *>(st + 2 * nv), *tie = cnt + n;
    for (size_t i = 0; i < n; i++) {
        add_ties(NonMaxSuppression::TieCount{tie[2 * i], tie[2 * i + 1]});
        times_.detections += (size_t)cnt[i];
        if ((size_t)cnt[i] > cfg_.det_cap) times_.dropped_detections += (size_t)cnt[i] - cfg_.det_cap;
    }
    if (s.timed) {  // the stage spans of this step on the slot's stream
        float ms[4] = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < 4; k++) check(zr_event_elapsed(&ms[k], s.ev_t[k], s.ev_t[k + 1]));
        times_.detect_gpu_ms += ms[0];
        times_.decode_nms_ms += ms[1];
        times_.landmark_gpu_ms += ms[2];
        times_.map_ms += ms[3];
        s.timed = false;
    }
    for (size_t v = 0; v < nv; v++) {
        times_.rois += st[nv + v].active ? 1 : 0;
        times_.tracked += st[v].tracked ? 1 : 0;
    }
    stale_ = true;
}

void DetectTrackPipeline::materialize() const {
    if (!stale_) return;
    stale_ = false;
    rois_.clear();
    for (auto &d : dets_) d.clear();
    for (size_t k = 0; k < std::min(active_slots_, slots_.size()); k++) unpack_device(*slots_[k]);
}

// device mode, on demand: the last finished step's detections and ROI results as the host mode
// builds them (the set stays untouched until the slot's next step after this one is enqueued).
// The copies go on the null stream: the set is complete (its ev_lm was waited for), and one more
// stream would share a hardware queue with a slot's (GPU_MAX_HW_QUEUES = 4: null + 3 slots) and
// serialise two slots -- measured 12% slower on the face line (profiles/, r03i trace)
void DetectTrackPipeline::unpack_device(Slot &s) const {
    const Cnn &lc = *lm_cnn_;
    const size_t n = s.nf, R = std::max(1u, cfg_.max_rois_per_frame), dcap = cfg_.det_cap, nv = n * R;
    const int L = cfg_.landmarker.num_landmarks, nkp = cfg_.detector.keypoints;
    const size_t nout = lc.nn().num_outputs();
    const Slot::Results &o = s.res[s.done];
    const zr_track_state *state = reinterpret_cast<const zr_track_state *>(o.h_sum.ptr);
    const zr_track_state *seed = state + nv;
    const int32_t *count = reinterpret_cast<const int32_t *>(seed + nv);
    // only the rows that hold detections: dcap is the detector's whole output by default
    int maxc = 0;
    for (size_t i = 0; i < n; i++) maxc = std::max(maxc, std::min(count[i], (int32_t)dcap));
    const size_t dw = (size_t)maxc;  // detections per frame in the host copy
    std::vector<float> dets(std::max<size_t>(1, n * dw * 20)), lmout(nv * L * 3), extra[2];
    check(zr_memcpy2d_async(dets.data(), dw * 80, o.dets.ptr, dcap * 80, dw * 80, n, 1, nullptr));
    check(zr_memcpy_async(lmout.data(), o.lmout.ptr, lmout.size() * 4, 1, nullptr));
    for (size_t k = 2; k < nout && k < 4; k++) {  // handedness / world landmarks / tongue_out
        extra[k - 2].resize((size_t)lc.nn().output_per_image(k) * nv);
        check(zr_memcpy_async(extra[k - 2].data(), o.lm[k].ptr, extra[k - 2].size() * 4, 1, nullptr));
    }
    check(zr_stream_synchronize(nullptr));
    for (size_t i = 0; i < n; i++) {
        const size_t f = s.f0 + i;
        const int cnt = count[i];
        auto &fd = dets_[f];
        fd.clear();
        for (int k = 0; k < cnt && k < (int)dcap; k++) {
            const float *e = &dets[(i * dw + k) * 20];
            Detection d;
            d.confidence = e[0];
            d.angle = e[1];
            d.rect = Rect::from_center(e[2], e[3], e[4], e[5]);
            for (int p = 0; p < nkp; p++) d.keypoints.push_back(Vec2{e[6 + 2 * p], e[7 + 2 * p]});
            fd.push_back(std::move(d));
        }
        for (size_t k = 0; k < R; k++) {
            const size_t v = i * R + k;
            const zr_track_state &s0 = seed[v];
            if (!s0.active) continue;
            RoiResult r;
            r.frame = (uint32_t)f;
            r.from_detection = (int)k < cnt;
            r.roi = RotatedRect(Rect::from_center(s0.roi[0], s0.roi[1], s0.roi[2], s0.roi[3]), s0.roi[4]);
            r.result.view_rect = RotatedRect(
                Rect::from_center(s0.view_rect[0], s0.view_rect[1], s0.view_rect[2], s0.view_rect[3]), s0.view_rect[4]);
            const zr_track_state &st = state[v];
            r.confidence = st.confidence;
            r.tracked = st.tracked != 0;
            if (r.tracked) {
                r.result.updated_roi = RotatedRect(
                    Rect::from_center(st.updated[0], st.updated[1], st.updated[2], st.updated[3]), st.updated[4]);
                r.next_roi = RotatedRect(Rect::from_center(st.roi[0], st.roi[1], st.roi[2], st.roi[3]), st.roi[4]);
                Estimate &e = r.result.estimate;
                const float *lm = &lmout[v * L * 3];
                e.positions.assign(lm, lm + 3 * L);
                e.confidence = st.confidence;
                if (cfg_.landmarker.kind == NetworkKind::FaceMeshV2 && nout > 2) e.tongue_out = extra[0][v];
                if (cfg_.landmarker.kind == NetworkKind::HandLandmarkLite && nout > 3) {
                    e.raw_handedness = extra[0][v];
                    const float *w = &extra[1][v * 3 * L];
                    e.world.assign(w, w + 3 * L);
                }
            }
            rois_.push_back(std::move(r));
        }
    }
}

// stage 2 (after stage 1 completed): exact decode + NMS + map (detection.rs:231-267), the
// ROI views of every tracked object, then enqueue the landmark network over all of them
void DetectTrackPipeline::stage_decode_and_rois(Slot &s, const std::vector<Image> &frames,
                                                const std::vector<std::vector<RotatedRect>> &forced) {
    const Cnn &dc = *det_cnn_;
    const uint32_t din_w = dc.input_width(), din_h = dc.input_height();
    const uint32_t A = (uint32_t)cfg_.detector.anchors().size(), D = (uint32_t)cfg_.detector.params;
    const uint32_t cap = cfg_.candidate_cap, rec_w = 2 + D;
    const size_t n = s.nf;
    std::vector<std::vector<float>> full_boxes(n), full_logits(n);
    bool overflow = false;
    for (size_t i = 0; i < n; i++)
        if ((uint32_t)s.h_count[i] > cap) {  // rare: more candidates than slots -> whole frame
            overflow = true;
            full_boxes[i].resize((size_t)A * D);
            full_logits[i].resize(A);
            check(zr_memcpy_async(full_boxes[i].data(), s.d_boxes.ptr + i * A * D, (size_t)A * D * 4, 1, s.stream));
            check(zr_memcpy_async(full_logits[i].data(), s.d_logits.ptr + i * A, (size_t)A * 4, 1, s.stream));
        }
    if (overflow) check(zr_stream_synchronize(s.stream));
    const float thresh = cfg_.det_threshold;
    pool_.parallel_for(n, [&](size_t i) {
        std::vector<Detection> raw;
        if (!full_logits[i].empty()) {
            cfg_.detector.extract(full_boxes[i].data(), full_logits[i].data(), thresh, din_w, din_h, raw);
        } else {
            const int cnt = s.h_count[i];
            const float *rec = &s.h_rec[i * cap * rec_w];
            std::vector<std::pair<uint32_t, int>> order;  // restore anchor order (extract_outputs)
            for (int k = 0; k < cnt; k++) {
                uint32_t a;
                std::memcpy(&a, &rec[k * rec_w], 4);
                order.push_back({a, k});
            }
            std::sort(order.begin(), order.end());
            for (auto &o : order) {
                const float *r = &rec[o.second * rec_w];
                const float conf = sigmoid(r[1]);
                if (conf < thresh) continue;
                raw.push_back(cfg_.detector.decode(o.first, r + 2, conf, din_w, din_h));
            }
        }
        auto &dets = dets_[s.f0 + i];
        dets = nms_.process(raw, &ties_[s.f0 + i]);
        map_detections(dets, s.letterbox[i], din_w);
    });

    const Cnn &lc = *lm_cnn_;
    const AspectRatio la = lc.aspect();
    s.rv.clear();
    s.rf.clear();
    s.local_rect.clear();
    s.roi0 = rois_.size();
    for (size_t i = 0; i < n; i++) {
        const size_t f = s.f0 + i;
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
        for (const auto &sd : seeds) {
            RoiResult r;
            r.frame = (uint32_t)f;
            r.from_detection = sd.second;
            r.roi = sd.first;
            // LandmarkTracker::track_impl (landmark.rs:465-467) + Estimator (landmark.rs:320-323)
            r.result.view_rect = sd.first.grow_to_fit_aspect(la);
            const ViewData view = full.view(r.result.view_rect);
            const Rect rect = view.local_rect().grow_to_fit_aspect(la);
            s.rv.push_back(to_zr_view(view.view(RotatedRect(rect, 0.f))));
            s.rf.push_back((uint32_t)i);
            s.local_rect.push_back(rect);
            rois_.push_back(r);
        }
    }
    s.nroi = rois_.size() - s.roi0;
    if (s.nroi == 0) return;
    const size_t nout = lc.nn().num_outputs();
    std::vector<float *> lptr(nout);
    for (size_t k = 0; k < nout; k++) {
        s.d_lm[k].resize((size_t)lc.nn().output_per_image(k) * s.nroi);
        lptr[k] = s.d_lm[k].ptr;
    }
    lc.estimate_async(s.zf, s.rv, s.rf, lptr.data(), s.stream);
    for (size_t k = 0; k < nout; k++) {
        const size_t cnt = (size_t)lc.nn().output_per_image(k) * s.nroi;
        s.h_lm[k].resize(cnt);
        check(zr_memcpy_async(s.h_lm[k].data(), lptr[k], cnt * 4, 1, s.stream));
    }
    check(zr_event_record(s.ev_lm, s.stream));
}

// stage 4 (after the landmark outputs arrived): extract + Estimator map-out + tracker update
void DetectTrackPipeline::stage_map(Slot &s) {
    const Cnn &lc = *lm_cnn_;
    const uint32_t lin_w = lc.input_width();
    const size_t nout = lc.nn().num_outputs();
    pool_.parallel_for(s.nroi, [&](size_t i) {
        RoiResult &r = rois_[s.roi0 + i];
        const float *outs[4];
        for (size_t k = 0; k < nout; k++) outs[k] = &s.h_lm[k][i * lc.nn().output_per_image(k)];
        Estimate e;
        extract_landmarks(cfg_.landmarker, outs, e, lin_w, lc.input_height());
        map_estimate(e, s.local_rect[i], lin_w);
        r.confidence = e.confidence;
        r.tracked = tracker_update(cfg_.landmarker, r.roi, r.result.view_rect, cfg_.loss_threshold,
                                   cfg_.roi_padding, e, r.result, r.next_roi);
        // lost: LandmarkTracker::track returns None (landmark.rs:468-477) -- no landmarks are
        // published, in particular not the view-local ones of the discarded estimate
    });
}

void DetectTrackPipeline::run(const std::vector<Image> &frames,
                              const std::vector<std::vector<RotatedRect>> &forced) {
    const auto t0 = clk::now();
    const size_t B = frames.size();
    times_ = StageTimes{};
    times_.frames = B;
    dets_.assign(B, {});
    ties_.assign(B, {});
    rois_.clear();
    if (B == 0) return;
    // split into sub-batches (software pipeline): GPU det(k+1) overlaps host decode(k), GPU
    // landmarks(k) overlaps host decode(k+1), host map(k) overlaps GPU landmarks(k+1)
    const size_t S = std::min<size_t>(slots_.size(), B);
    size_t f0 = 0;
    for (size_t k = 0; k < S; k++) {
        Slot &s = *slots_[k];
        s.f0 = f0;
        s.nf = B / S + (k < B % S ? 1 : 0);
        f0 += s.nf;
        s.inputs_ok = false;  // new frames
        stage_detect(s, frames);
        if (cfg_.device_post) stage_device_post(s, frames, forced);
    }
    active_slots_ = S;
    if (cfg_.device_post && rec_rmax_ && &frames == &frames_) enqueue_gather();
    for (size_t k = 0; k < S && cfg_.device_post; k++) {
        Slot &s = *slots_[k];
        const auto t = clk::now();
        check(zr_event_synchronize(s.ev_lm));
        times_.host_wait_ms += ms_since(t);
        finish_device(s);
    }
    if (cfg_.device_post) done_steps_ = enq_steps_;
    if (cfg_.device_post) {
        times_.total_ms = ms_since(t0);
        return;
    }
    for (size_t k = 0; k < S && !cfg_.device_post; k++) {
        Slot &s = *slots_[k];
        const auto t = clk::now();
        check(zr_event_synchronize(s.ev_det));
        times_.detect_gpu_ms += ms_since(t);
        const auto t1 = clk::now();
        stage_decode_and_rois(s, frames, forced);
        times_.decode_nms_ms += ms_since(t1);
    }
    for (size_t k = 0; k < S && !cfg_.device_post; k++) {
        Slot &s = *slots_[k];
        const auto t = clk::now();
        if (s.nroi) check(zr_event_synchronize(s.ev_lm));
        times_.landmark_gpu_ms += ms_since(t);
        const auto t1 = clk::now();
        stage_map(s);
        times_.map_ms += ms_since(t1);
    }
    times_.rois = rois_.size();
    for (auto &d : dets_) times_.detections += d.size();
    for (const auto &t : ties_) add_ties(t);
    for (auto &r : rois_) times_.tracked += r.tracked ? 1 : 0;
    times_.total_ms = ms_since(t0);
}

void DetectTrackPipeline::begin_steps() {
    steps_t0_ = clk::now();
    times_ = StageTimes{};
    if (gstream_) check(zr_stream_synchronize(gstream_));
    enq_steps_ = done_steps_ = 0;
    gath_used_[0] = gath_used_[1] = false;
    const std::vector<Image> &frames = frames_;
    const size_t B = frames.size();
    active_slots_ = std::min<size_t>(slots_.size(), B);
    size_t f0 = 0;
    for (size_t k = 0; k < active_slots_; k++) {
        Slot &s = *slots_[k];
        s.f0 = f0;
        s.nf = B / active_slots_ + (k < B % active_slots_ ? 1 : 0);
        f0 += s.nf;
        s.inputs_ok = false;  // the slots' frame ranges may have changed
        stage_detect(s, frames);
        if (cfg_.device_post) stage_device_post(s, frames, forced_);
    }
    if (cfg_.device_post) enqueue_gather();
}

void DetectTrackPipeline::step(bool more) {
    const std::vector<Image> &frames = frames_;
    const size_t B = frames.size(), S = active_slots_;
    if (S == 0) return;
    dets_.assign(B, {});
    ties_.assign(B, {});
    rois_.clear();
    // device mode: a slot's whole step is on its stream; take its results and enqueue its next
    // step at once, while the other slots' steps run
    for (size_t k = 0; k < S && cfg_.device_post; k++) {
        Slot &s = *slots_[k];
        const auto t = clk::now();
        check(zr_event_synchronize(s.ev_lm));
        times_.host_wait_ms += ms_since(t);
        finish_device(s);
        if (more) {
            stage_detect(s, frames);
            stage_device_post(s, frames, forced_);
        }
    }
    if (cfg_.device_post) {
        done_steps_++;
        if (more) enqueue_gather();
        times_.frames += B;
        times_.total_ms = ms_since(steps_t0_);
        return;
    }
    for (size_t k = 0; k < S && !cfg_.device_post; k++) {
        Slot &s = *slots_[k];
        const auto t = clk::now();
        check(zr_event_synchronize(s.ev_det));
        times_.detect_gpu_ms += ms_since(t);
        const auto t1 = clk::now();
        stage_decode_and_rois(s, frames, forced_);
        times_.decode_nms_ms += ms_since(t1);
        // the next run's detections of this slot queue behind its landmarks at once, so the
        // GPU has them while the host decodes the later slots (the slot's detector outputs and
        // letterbox views are consumed; the landmark launch copied its view descriptors)
        if (more) stage_detect(s, frames);
    }
    for (size_t k = 0; k < S && !cfg_.device_post; k++) {
        Slot &s = *slots_[k];
        const auto t = clk::now();
        if (s.nroi) check(zr_event_synchronize(s.ev_lm));
        times_.landmark_gpu_ms += ms_since(t);
        const auto t1 = clk::now();
        stage_map(s);
        times_.map_ms += ms_since(t1);
    }
    times_.frames += B;
    times_.rois += rois_.size();
    for (auto &d : dets_) times_.detections += d.size();
    for (const auto &t : ties_) add_ties(t);
    for (auto &r : rois_) times_.tracked += r.tracked ? 1 : 0;
    times_.total_ms = ms_since(steps_t0_);
}

void DetectTrackPipeline::run_frames_repeated(int steps) {
    if (frames_.empty() || steps <= 0) {
        times_ = StageTimes{};
        return;
    }
    begin_steps();
    for (int it = 0; it < steps; it++) step(it + 1 < steps);
}

}  // namespace zh
