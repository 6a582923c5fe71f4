// detection.cpp -- see detection.h.
#include "detection.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>

namespace zh {

std::vector<Vec2> calculate_anchors(const std::vector<LayerInfo> &layers) {
    std::vector<Vec2> a;
    for (const auto &l : layers)
        for (uint32_t y = 0; y < l.height; y++)
            for (uint32_t x = 0; x < l.width; x++)
                for (uint32_t b = 0; b < l.boxes_per_cell; b++)
                    a.push_back({((float)x + 0.5f) / (float)l.width, ((float)y + 0.5f) / (float)l.height});
    return a;
}

namespace {
// f32::total_cmp key (zaru-image/src/num.rs:7-27)
int32_t total_key(float f) {
    int32_t i;
    std::memcpy(&i, &f, 4);
    return i ^ (int32_t)(((uint32_t)(i >> 31)) >> 1);
}
}  // namespace

// nms.rs:59-145
std::vector<Detection> NonMaxSuppression::process(std::vector<Detection> &dets, TieCount *ties) const {
    std::stable_sort(dets.begin(), dets.end(), [](const Detection &a, const Detection &b) {
        return total_key(a.confidence) < total_key(b.confidence);
    });
    if (ties) {  // members of runs of equal keys in the sorted list
        ties->candidates = (int)dets.size();
        ties->tied = 0;
        for (size_t i = 0; i < dets.size(); i++) {
            const int32_t k = total_key(dets[i].confidence);
            const bool eq = (i > 0 && total_key(dets[i - 1].confidence) == k) ||
                            (i + 1 < dets.size() && total_key(dets[i + 1].confidence) == k);
            ties->tied += eq ? 1 : 0;
        }
    }
    std::vector<Detection> out, group;
    while (!dets.empty()) {
        Detection seed = std::move(dets.back());
        dets.pop_back();
        if (mode_ == SuppressionMode::Remove) {
            dets.erase(std::remove_if(dets.begin(), dets.end(),
                                      [&](const Detection &o) { return !(seed.rect.iou(o.rect) < iou_); }),
                       dets.end());
            out.push_back(std::move(seed));
            continue;
        }
        group.clear();
        group.push_back(seed);
        std::vector<Detection> keep;
        keep.reserve(dets.size());
        for (auto &o : dets) {  // Vec::retain: visits in order, keeps order
            if (seed.rect.iou(o.rect) >= iou_) group.push_back(o);
            else keep.push_back(std::move(o));
        }
        dets.swap(keep);
        float ax = 0.f, ay = 0.f, aw = 0.f, ah = 0.f, aa = 0.f, divisor = 0.f;
        Detection acc;
        acc.confidence = seed.confidence;
        acc.anchor = seed.anchor;
        for (const auto &d : group) {
            if (acc.keypoints.empty() && !d.keypoints.empty()) acc.keypoints.assign(d.keypoints.size(), Vec2{});
            if (acc.keypoints.size() != d.keypoints.size())
                throw ZaruError(ZR_ERR_SHAPE, "landmark count must be constant");
            const float f = d.confidence;
            divisor += f;
            for (size_t k = 0; k < acc.keypoints.size(); k++) {
                acc.keypoints[k].x += d.keypoints[k].x * f;
                acc.keypoints[k].y += d.keypoints[k].y * f;
            }
            ax += d.rect.center().x * f;
            ay += d.rect.center().y * f;
            aw += d.rect.width() * f;
            ah += d.rect.height() * f;
            aa += d.angle * f;
        }
        for (auto &k : acc.keypoints) {
            k.x /= divisor;
            k.y /= divisor;
        }
        ax /= divisor;
        ay /= divisor;
        aw /= divisor;
        ah /= divisor;
        aa /= divisor;
        acc.rect = Rect::from_center(ax, ay, aw, ah);
        acc.angle = aa;
        out.push_back(std::move(acc));
    }
    return out;
}

DetectorNetwork DetectorNetwork::short_range_face() {
    DetectorNetwork n;
    n.kind = NetworkKind::FaceDetectionShortRange;
    n.layers = {{2, 16, 16}, {6, 8, 8}};
    n.params = 16;
    n.keypoints = 6;
    return n;
}

DetectorNetwork DetectorNetwork::full_range_face() {
    DetectorNetwork n;
    n.kind = NetworkKind::FaceDetectionFullRange;
    n.layers = {{1, 48, 48}};  // 2304 anchors (face/detection.rs:86-88)
    n.params = 16;
    n.keypoints = 6;
    return n;
}

DetectorNetwork DetectorNetwork::palm_lite() {
    DetectorNetwork n;
    n.kind = NetworkKind::PalmDetectionLite;
    n.layers = {{2, 24, 24}, {6, 12, 12}};
    n.params = 18;
    n.keypoints = 7;
    return n;
}

const std::vector<Vec2> &DetectorNetwork::anchors() const {
    static std::mutex mu;
    std::lock_guard<std::mutex> g(mu);
    if (!anchors_) anchors_ = std::make_shared<std::vector<Vec2>>(calculate_anchors(layers));
    return *anchors_;
}

Detection DetectorNetwork::decode(uint32_t anchor, const float *b, float confidence, uint32_t in_w,
                                  uint32_t in_h) const {
    const Vec2 input_size{(float)in_w, (float)in_h};
    const Vec2 center = Vec2{b[0], b[1]} + anchors()[anchor] * input_size;
    Detection d;
    d.confidence = confidence;
    d.anchor = (int32_t)anchor;
    d.rect = Rect::from_center(center.x, center.y, b[2], b[3]);
    for (int k = 0; k < keypoints; k++)  // quirk kept: offset by centre * input size
        d.keypoints.push_back(Vec2{b[4 + 2 * k], b[5 + 2 * k]} + center * input_size);
    if (is_face_detector(kind)) {
        // left eye -> right eye against +X (face/detection.rs:151-154)
        d.angle = signed_angle_to(d.keypoints[1] - d.keypoints[0], Vec2{1.f, 0.f});
    } else {
        // wrist - middle finger MCP against +Y (hand/detection.rs:172-176)
        d.angle = signed_angle_to(d.keypoints[0] - d.keypoints[2], Vec2{0.f, 1.f});
    }
    return d;
}

void DetectorNetwork::extract(const float *boxes, const float *logits, float thresh, uint32_t in_w,
                              uint32_t in_h, std::vector<Detection> &out) const {
    const auto &a = anchors();
    for (uint32_t i = 0; i < a.size(); i++) {
        const float conf = sigmoid(logits[i]);
        if (conf < thresh) continue;
        out.push_back(decode(i, boxes + (size_t)i * params, conf, in_w, in_h));
    }
}

void map_detections(std::vector<Detection> &dets, const Rect &rect, uint32_t in_w) {
    const float scale = rect.width() / (float)in_w;
    const Vec2 tl = rect.top_left();
    for (auto &d : dets) {
        const Vec2 c = d.rect.center(), s = d.rect.size();
        d.rect = Rect::from_center(c.x * scale, c.y * scale, s.x * scale, s.y * scale);
        for (auto &k : d.keypoints) k = k * scale;
        d.rect = d.rect.move_by(tl);
        for (auto &k : d.keypoints) k = k + tl;
    }
}

void pack_detection_records(const std::vector<std::vector<Detection>> &dets,
                            const std::vector<uint32_t> &frame_ids, uint32_t rmax, float *out) {
    const uint32_t w = det_record_width(rmax);
    for (size_t f = 0; f < dets.size(); f++) {
        float *r = out + f * w;
        std::fill(r, r + w, 0.f);
        const uint32_t id = f < frame_ids.size() ? frame_ids[f] : (uint32_t)f;
        const uint32_t cnt = (uint32_t)dets[f].size();
        std::memcpy(&r[0], &id, 4);
        std::memcpy(&r[1], &cnt, 4);
        for (uint32_t k = 0; k < std::min<uint32_t>(cnt, rmax); k++) {
            const Detection &d = dets[f][k];
            float *e = r + 2 + DET_RECORD_FIELDS * k;
            e[0] = d.confidence;
            e[1] = d.angle;
            e[2] = d.rect.center().x;
            e[3] = d.rect.center().y;
            e[4] = d.rect.width();
            e[5] = d.rect.height();
            for (size_t p = 0; p < d.keypoints.size() && p < 7; p++) {
                e[6 + 2 * p] = d.keypoints[p].x;
                e[7 + 2 * p] = d.keypoints[p].y;
            }
        }
    }
}

ViewData letterbox_view(uint32_t w, uint32_t h, AspectRatio in_aspect, Rect *rect_out) {
    const ViewData full = ViewData::full(w, h);
    const Rect rect = full.local_rect().grow_to_fit_aspect(in_aspect);
    if (rect_out) *rect_out = rect;
    return full.view(RotatedRect(rect, 0.f));
}

float candidate_logit_floor(float thresh) {
    if (!(thresh > 0.f)) return -INFINITY;
    if (thresh >= 1.f) return INFINITY;
    const double l = std::log((double)thresh / (1.0 - (double)thresh));
    return (float)(l - 1e-3 * (1.0 + std::fabs(l)));
}

Detector::Detector(DetectorNetwork net, int device)
    : net_(std::move(net)), cnn_(network_cnn(net_.kind, device)) {}

const std::vector<Detection> &Detector::detect(const Image &img) {
    dets_.clear();
    Rect rect;
    const ViewData view = letterbox_view(img.width, img.height, cnn_->aspect(), &rect);
    auto outs = cnn_->estimate(img, {view});
    std::vector<Detection> raw;
    net_.extract(outs[0].data(), outs[1].data(), thresh_, cnn_->input_width(), cnn_->input_height(), raw);
    dets_ = nms_.process(raw);
    map_detections(dets_, rect, cnn_->input_width());
    return dets_;
}

}  // namespace zh
