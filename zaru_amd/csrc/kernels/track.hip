// track.hip -- LandmarkTracker::track_impl (crates/zaru/src/landmark.rs:463-501) on the device,
// so a video loop runs estimate -> update -> next view without a host round trip per frame
// (SURVEY.md §8f-3).  One workgroup per tracked ROI:
//   1. Confidence::confidence of the estimate and the loss check (landmark.rs:468-477);
//   2. Estimator map-out of the landmarks (landmark.rs:336-345) and the estimate angle
//      (mediapipe.rs:146-160 / hand/landmark.rs:68-78);
//   3. transform_out into the frame (landmark.rs:481-486) and RotatedRect::bounding at the
//      tracked angle (rect.rs:287-325): a block min/max reduction;
//   4. next RoI = grow_rel(padding) (landmark.rs:493), and from it the next estimate's view
//      exactly as the host builds it (grow_to_fit_aspect, ViewData::view twice,
//      image/mod.rs:201-210, nn/mod.rs:118-126), written as the preprocessing's view table.
// f32 throughout, no contraction (HIPFLAGS -ffp-contract=off), Rust's operation order, and
// glibc's own sinf / cosf / atan2f / expf (glibc_math.h, verified over every f32 input), so the
// update and the view table it writes are bit-identical to the host restatement.
#include "../runtime/zr_track.h"
#include "geom_dev.h"

namespace zr {
namespace {

using namespace geo;

// The next estimate's sampling view of a RoI: track_impl's view_rect + Estimator's aspect-fit
// local rect (pipeline.cpp stage_decode_and_rois, landmark.rs:465-467 + 320-323).
__device__ void next_view(TrackState &st, ViewDesc &vd, int frame, int aw, int ah) {
    const RRect roi = {st.roi[0], st.roi[1], st.roi[2], st.roi[3], st.roi[4]};
    const RRect vr = grow_to_fit_aspect(roi, aw, ah);
    const RRect full = from_top_left(0.f, 0.f, (float)st.frame_w, (float)st.frame_h, 0.f);
    const RRect view = view_of(full, vr);
    const RRect local = grow_to_fit_aspect(from_top_left(0.f, 0.f, view.w, view.h, 0.f), aw, ah);
    const RRect net = view_of(view, local);
    st.view_rect[0] = vr.cx;
    st.view_rect[1] = vr.cy;
    st.view_rect[2] = vr.w;
    st.view_rect[3] = vr.h;
    st.view_rect[4] = vr.rad;
    const V2 ltl = top_left(local);
    st.local[0] = ltl.x;
    st.local[1] = ltl.y;
    st.local[2] = local.w;
    // make_view (session.cpp) on the zr_view {centre, size, rad} of `net`
    vd.half_w = net.w * 0.5f;
    vd.half_h = net.h * 0.5f;
    vd.tl_x = net.cx - net.w * 0.5f;
    vd.tl_y = net.cy - net.h * 0.5f;
    vd.view_w = net.w;
    vd.view_h = net.h;
    vd.cos_r = glibc::cosf(net.rad);
    vd.sin_r = glibc::sinf(net.rad);
    vd.frame = (uint32_t)frame;
    vd.pad_ = 0;
}

__device__ __forceinline__ float wave_min(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// Landmark rows of a ROI that is not tracked this step (lost now or earlier) hold NaN, so a
// reader that ignores states()[i].tracked cannot mistake a stale estimate for a result.
__device__ void invalidate_rows(const TrackParams &P, int i, int tid) {
    if (!P.lm_out) return;
    float *q = P.lm_out + (int64_t)i * P.L * 3;
    for (int j = tid; j < 3 * P.L; j += 256) q[j] = __builtin_nanf("");
}

__global__ __launch_bounds__(256) void track_kernel(const TrackParams P) {
    const int i = blockIdx.x, tid = threadIdx.x;
    if (i >= P.n) return;  // whole workgroup
    __shared__ float red[4][4];
    TrackState st = P.state[i];
    if (!P.seed) {
        if (!st.active) {  // lost earlier: stays lost (roi = None)
            invalidate_rows(P, i, tid);
            if (tid == 0) P.state[i].tracked = 0;
            return;
        }
        float conf = 1.f;
        if (P.kind == 0) conf = sigmoid(P.flag[(int64_t)i * P.flag_stride]);  // num.rs:6-8
        else if (P.kind == 1) conf = P.flag[(int64_t)i * P.flag_stride];
        if (conf < P.loss_thresh) {
            invalidate_rows(P, i, tid);
            if (tid == 0) {
                P.state[i].active = 0;
                P.state[i].tracked = 0;
                P.state[i].confidence = conf;
            }
            return;
        }
        const int L = P.L;
        // per-image landmark output 0 (lm_stride floats per image, checked on the host to hold
        // L x 3, 2L for kind 3, or the 71-point eye contour for kind 2, whose 5 iris points come
        // first from output 1, eye.rs:47-64)
        const float *lm = P.lm + (int64_t)i * P.lm_stride;
        const float *iris = P.kind == 2 ? P.flag + (int64_t)i * P.flag_stride : nullptr;
        const float scale = st.local[2] / (float)P.in_w;
        // map-out of landmark j (Estimator, landmark.rs:336-345): p * scale, then + rect.x / .y
        auto mapped = [&](int j, float &x, float &y, float &z) {
            if (P.kind == 3) {  // multipie68.rs:71-80: relative (x, y) * input resolution, z = 0
                x = lm[2 * j] * (float)P.in_w;
                y = lm[2 * j + 1] * (float)P.in_h;
                z = 0.f;
            } else if (P.kind == 2) {
                const float *src = j < 5 ? iris + 3 * j : lm + 3 * (j - 5);
                x = src[0];
                y = src[1];
                z = src[2];
            } else {
                x = lm[3 * j];
                y = lm[3 * j + 1];
                z = lm[3 * j + 2];
            }
            x = x * scale;
            y = y * scale;
            z = z * scale;
            x += st.local[0];
            y += st.local[1];
        };
        float est = 0.f;  // Estimate::angle_radians; None -> unwrap_or(0.0) (landmark.rs:479)
        if (P.kind == 0 || P.kind == 1) {
            const int a = P.kind == 0 ? 263 : 0, b = P.kind == 0 ? 33 : 9;
            float ax, ay, az, bx, by, bz;
            mapped(a, ax, ay, az);
            mapped(b, bx, by, bz);
            est = P.kind == 0 ? signed_angle_to({ax - bx, ay - by}, {1.f, 0.f})
                              : signed_angle_to({ax - bx, ay - by}, {0.f, 1.f});
        }
        const float angle = st.roi[4] + est;
        const RRect vr = {st.view_rect[0], st.view_rect[1], st.view_rect[2], st.view_rect[3], st.view_rect[4]};
        const float c = glibc::cosf(-angle), s = glibc::sinf(-angle), ns = -s;  // rect.rs:287-325
        float mnx = 3.40282347e38f, mny = 3.40282347e38f, mxx = -3.40282347e38f, mxy = -3.40282347e38f;
        for (int j = tid; j < L; j += 256) {
            float x, y, z;
            mapped(j, x, y, z);
            const V2 o = transform_out(vr, {x, y});
            if (P.lm_out) {
                float *q = P.lm_out + ((int64_t)i * L + j) * 3;
                q[0] = o.x;
                q[1] = o.y;
                q[2] = z;
            }
            const float rx = (0.f + c * o.x) + ns * o.y, ry = (0.f + s * o.x) + c * o.y;
            mnx = fminf(mnx, rx);
            mny = fminf(mny, ry);
            mxx = fmaxf(mxx, rx);
            mxy = fmaxf(mxy, ry);
        }
        mnx = wave_min(mnx);
        mny = wave_min(mny);
        mxx = wave_max(mxx);
        mxy = wave_max(mxy);
        const int w = tid >> 6;
        if ((tid & 63) == 0) {
            red[w][0] = mnx;
            red[w][1] = mny;
            red[w][2] = mxx;
            red[w][3] = mxy;
        }
        __syncthreads();
        if (tid != 0) return;
        for (int k = 1; k < 4; ++k) {
            red[0][0] = fminf(red[0][0], red[k][0]);
            red[0][1] = fminf(red[0][1], red[k][1]);
            red[0][2] = fmaxf(red[0][2], red[k][2]);
            red[0][3] = fmaxf(red[0][3], red[k][3]);
        }
        const V2 ctr = rot_ccw({(red[0][0] + red[0][2]) * 0.5f, (red[0][1] + red[0][3]) * 0.5f}, angle);
        const float uw = red[0][2] - red[0][0], uh = red[0][3] - red[0][1];
        st.updated[0] = ctr.x;
        st.updated[1] = ctr.y;
        st.updated[2] = uw;
        st.updated[3] = uh;
        st.updated[4] = angle;
        // grow_rel(padding) adds padding * size to each side (rect.rs:84-93)
        const float l = uw * P.padding, t = uh * P.padding;
        st.roi[0] = ctr.x;
        st.roi[1] = ctr.y;
        st.roi[2] = uw + l + l;
        st.roi[3] = uh + t + t;
        st.roi[4] = angle;
        st.tracked = 1;
        st.confidence = conf;
    } else if (tid != 0) {
        return;
    }
    next_view(st, P.views[i], i / P.rpf, P.asp_w, P.asp_h);
    P.state[i] = st;
}

// One thread per ROI slot (frame f = i / R, slot k = i % R): the seed ROI the host pipeline
// builds (pipeline.cpp stage_decode_and_rois: RotatedRect(det.rect[.grow_rel(g)], angle or 0)
// per detection in NMS order, up to R, or the frame's forced ROIs when it has no detection) and
// its first view, as LandmarkTracker::set_roi + track_impl would sample it.
__global__ __launch_bounds__(256) void seed_kernel(const SeedParams P) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P.N * P.R) return;
    const int f = i / P.R, k = i - f * P.R;
    const int cnt = P.count[f];
    TrackState st{};
    st.frame_w = P.fsize[2 * f];
    st.frame_h = P.fsize[2 * f + 1];
    if (k < cnt && k < P.dcap) {
        const float *d = P.dets + ((int64_t)f * P.dcap + k) * 20;
        RRect r = {d[2], d[3], d[4], d[5], P.roi_use_angle ? d[1] : 0.f};
        if (P.roi_grow > 0.f) r = grow_rel(r, P.roi_grow);
        st.roi[0] = r.cx;
        st.roi[1] = r.cy;
        st.roi[2] = r.w;
        st.roi[3] = r.h;
        st.roi[4] = r.rad;
        st.active = 1;
    } else if (cnt == 0 && P.nforced && k < P.nforced[f]) {
        const float *r = P.forced + ((int64_t)f * P.R + k) * 5;
        for (int c = 0; c < 5; ++c) st.roi[c] = r[c];
        st.active = 1;
    } else {  // idle slot: a valid (empty-frame) view so the batched network stays in bounds
        st.roi[2] = st.roi[3] = 1.f;
        st.active = 0;
    }
    next_view(st, P.views[i], f, P.asp_w, P.asp_h);
    P.state[i] = st;
    if (P.seed_copy) P.seed_copy[i] = st;
}

// One thread per video stream: HandTracker::track's bookkeeping (tracking.rs:115-219) over the
// stream's hand slots, in the reference's order.  Rect::iou and grow_rel as the host restates
// them (geom_dev.h), so filter and de-duplication decide exactly as the host HandTracker does.
__device__ void move_hand(const HandManageParams &P, int to, int from) {
    P.state[to] = P.state[from];
    P.ids[to] = P.ids[from];
    P.src[to] = P.src[from];
    for (int c = 0; c < 5; ++c) P.hroi[to * 5 + c] = P.hroi[from * 5 + c];
}

__global__ __launch_bounds__(64) void hand_manage_kernel(const HandManageParams P) {
    const int s = blockIdx.x * 64 + threadIdx.x;
    if (s >= P.S) return;
    const int base = s * P.H;
    if (P.init_clock) P.next_det[s] = P.now;
    // 1. retain_mut: hands whose tracking was lost leave; the others' ROI is their updated_roi
    int k = 0;
    const int n = P.nhands[s];
    for (int h = 0; h < n; ++h) {
        const int i = base + h;
        if (!P.state[i].active) continue;
        const TrackState st = P.state[i];
        const int j = base + k;
        float r[5];
        for (int c = 0; c < 5; ++c) r[c] = st.tracked ? st.updated[c] : P.hroi[i * 5 + c];
        const uint64_t id = P.ids[i];
        P.state[j] = st;
        P.ids[j] = id;
        P.src[j] = h;
        for (int c = 0; c < 5; ++c) P.hroi[j * 5 + c] = r[c];
        ++k;
    }
    // 2./3. the previous step's palm detections: keep those whose grown box overlaps no hand
    // that existed before this step's new ones (Vec::retain over self.hands, tracking.rs:140-156),
    // then start a hand for each kept one (RotatedRect(grow_rel(1.5), angle), LandmarkTracker::
    // set_roi, 158-194).  Every detection is visited (dcap is the detector's whole output); a
    // kept detection with no free slot left is counted in `dropped` (the reference's Vec grows)
    int dropped = 0;
    if (P.det_pending[s]) {
        const int cnt = min(P.count[s], P.dcap);
        const int k0 = k;
        for (int d = 0; d < cnt; ++d) {
            const float *dd = P.dets + ((int64_t)s * P.dcap + d) * 20;
            const RRect g = grow_rel({dd[2], dd[3], dd[4], dd[5], 0.f}, P.grow);
            bool ok = true;
            for (int j = 0; j < k0 && ok; ++j) {
                const float *r = P.hroi + (base + j) * 5;
                ok = iou(r[0], r[1], r[2], r[3], g.cx, g.cy, g.w, g.h) < P.iou;
            }
            if (!ok) continue;
            if (k >= P.H) {  // capacity: reported, never silent
                ++dropped;
                continue;
            }
            const int j = base + k;
            TrackState st{};
            st.roi[0] = g.cx;
            st.roi[1] = g.cy;
            st.roi[2] = g.w;
            st.roi[3] = g.h;
            st.roi[4] = dd[1];
            st.active = 1;
            st.frame_w = P.fsize[2 * s];
            st.frame_h = P.fsize[2 * s + 1];
            for (int c = 0; c < 5; ++c) P.hroi[j * 5 + c] = st.roi[c];
            P.state[j] = st;
            P.ids[j] = P.next_id[s]++;
            P.src[j] = -1;
            ++k;
        }
    }
    if (P.dropped) P.dropped[s] = dropped;
    // 4. for i in (0..len).rev(): the first earlier hand it overlaps removes it by swap_remove
    for (int i = k - 1; i >= 0; --i) {
        const float *a = P.hroi + (base + i) * 5;
        for (int j = 0; j < i; ++j) {
            const float *b = P.hroi + (base + j) * 5;
            if (iou(a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]) >= P.iou) {
                if (i != k - 1) move_hand(P, base + i, base + k - 1);
                --k;
                break;
            }
        }
    }
    // 5. start a detection when no hand is tracked or the redetect interval elapsed (none is
    // running here: the previous one's result was consumed above)
    const bool req = k == 0 || P.now >= P.next_det[s];
    if (req) P.next_det[s] += P.interval;
    P.det_pending[s] = req ? 1 : 0;
    P.nhands[s] = k;
    // this step's views; idle slots get a valid empty-frame view (the batched network stays in bounds)
    for (int h = 0; h < P.H; ++h) {
        const int i = base + h;
        TrackState st = P.state[i];
        if (h >= k) {
            st = TrackState{};
            st.roi[2] = st.roi[3] = 1.f;
            st.frame_w = P.fsize[2 * s];
            st.frame_h = P.fsize[2 * s + 1];
            P.src[i] = -1;
        }
        next_view(st, P.views[i], s, P.asp_w, P.asp_h);
        P.state[i] = st;
    }
}

}  // namespace

// one workgroup: a block-wide exclusive scan of the request flags per 1024-stream chunk; the
// flags are pending[s] != 0, or (lost_of != null) the streams whose tracker holds no RoI
__global__ __launch_bounds__(1024) void due_compact_kernel(const int32_t *pending, const TrackState *lost_of, int S,
                                                           const ViewDesc tmpl, int32_t *due, int32_t *ndue,
                                                           ViewDesc *due_views, uint64_t *total) {
    __shared__ int wsum[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int base = 0;
    for (int c0 = 0; c0 < S; c0 += 1024) {
        const int s = c0 + t;
        const bool req = s < S && (lost_of ? lost_of[s].active == 0 : pending[s] != 0);
        const uint64_t m = __ballot(req);
        const int in_wave = (int)__popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = (int)__popcll(m);
        __syncthreads();
        int before = 0, total = 0;
        for (int i = 0; i < 16; ++i) {
            before += i < w ? wsum[i] : 0;
            total += wsum[i];
        }
        if (req) {
            const int k = base + before + in_wave;
            due[k] = s;
            ViewDesc v = tmpl;
            v.frame = (uint32_t)s;
            due_views[k] = v;
        }
        base += total;
        __syncthreads();  // wsum is rewritten by the next chunk
    }
    if (t == 0) {
        *ndue = base;
        if (total) *total += (uint64_t)base;
    }
}

const char *launch_due_compact(const int32_t *det_pending, const TrackState *lost_of, int S, const ViewDesc &tmpl,
                               int32_t *due, int32_t *ndue, ViewDesc *due_views, uint64_t *total, hipStream_t s) {
    hipLaunchKernelGGL(due_compact_kernel, dim3(1), dim3(1024), 0, s, det_pending, lost_of, S, tmpl, due, ndue,
                       due_views, total);
    return "due_compact_kernel";
}

// Rust's f32::total_cmp key (TotalF32, num.rs): the bits with the magnitude flipped for negatives,
// compared as signed integers
__device__ __forceinline__ int32_t total_key(float v) {
    const int32_t b = __float_as_int(v);
    return b ^ (int32_t)((uint32_t)(b >> 31) >> 1);
}

// One thread per stream: examples/facemesh.rs:45-54 after `tracker.track` returned None.  A
// stream whose tracker holds no RoI ran this frame's detection (its slot of count / dets); if it
// found any face, the RoI becomes the bounding rect of the most confident detection --
// `max_by_key(TotalF32(confidence))`, which keeps the LAST of equal maxima -- unrotated and
// unpadded (LandmarkTracker::set_roi), and the next frame's view is derived from it.
__global__ __launch_bounds__(256) void reseed_kernel(const ReseedParams P) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= P.N) return;
    TrackState st = P.state[s];
    if (st.active) return;  // tracked this frame: no detection ran for it
    const int cnt = min(P.count[s], P.dcap);
    if (cnt <= 0) return;   // nothing detected: still lost, the next frame detects again
    const float *d = P.dets + (int64_t)s * P.dcap * 20;
    int best = 0;
    int32_t bk = total_key(d[0]);
    for (int k = 1; k < cnt; ++k) {
        const int32_t key = total_key(d[k * 20]);
        if (key >= bk) {  // >=: the last maximum
            bk = key;
            best = k;
        }
    }
    const float *b = d + best * 20;
    st.roi[0] = b[2];
    st.roi[1] = b[3];
    st.roi[2] = b[4];
    st.roi[3] = b[5];
    st.roi[4] = 0.f;
    st.active = 1;
    st.frame_w = P.fsize[2 * s];
    st.frame_h = P.fsize[2 * s + 1];
    next_view(st, P.views[s], s, P.asp_w, P.asp_h);
    P.state[s] = st;
    if (P.reseeded) atomicAdd((unsigned long long *)P.reseeded, 1ull);
}

const char *launch_reseed(const ReseedParams &p, hipStream_t s) {
    hipLaunchKernelGGL(reseed_kernel, dim3((p.N + 255) / 256), dim3(256), 0, s, p);
    return "reseed_kernel";
}

const char *launch_hand_manage(const HandManageParams &p, hipStream_t s) {
    hipLaunchKernelGGL(hand_manage_kernel, dim3((p.S + 63) / 64), dim3(64), 0, s, p);
    return "hand_manage_kernel";
}

const char *launch_track(const TrackParams &p, hipStream_t s) {
    hipLaunchKernelGGL(track_kernel, dim3(p.n), dim3(256), 0, s, p);
    return "track_kernel";
}

const char *launch_seed(const SeedParams &p, hipStream_t s) {
    hipLaunchKernelGGL(seed_kernel, dim3((p.N * p.R + 255) / 256), dim3(256), 0, s, p);
    return "seed_kernel";
}

// Test hook (zr_debug_glibc_math): the device evaluation of glibc_math.h, one thread per input.
__global__ __launch_bounds__(256) void glibc_math_kernel(int fn, const float *a, const float *b, float *out,
                                                         int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = a[i];
    float r;
    switch (fn) {
        case 0: r = glibc::sinf(x); break;
        case 1: r = glibc::cosf(x); break;
        case 2: r = glibc::expf(x); break;
        case 3: r = glibc::atanf(x); break;
        default: r = glibc::atan2f(x, b[i]); break;
    }
    out[i] = r;
}

const char *launch_glibc_math(int fn, const float *a, const float *b, float *out, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(glibc_math_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, fn, a, b, out, n);
    return "glibc_math_kernel";
}

}  // namespace zr
