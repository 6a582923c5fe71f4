// networks.cpp -- NeuralNetwork / Cnn over the C ABI, and the per-network singletons.
#include "networks.h"

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>

namespace zh {

std::vector<uint8_t> read_file(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "cannot open " + path);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

NeuralNetwork::NeuralNetwork(const std::vector<uint8_t> &onnx, const std::vector<uint32_t> &out_sel,
                             int device) {
    check(zr_session_create(onnx.data(), onnx.size(), out_sel.empty() ? nullptr : out_sel.data(),
                            out_sel.size(), device, &s_));
    int64_t shape[8];
    size_t rank = 0;
    const char *name = nullptr;
    check(zr_session_io(s_, 0, 0, &name, shape, &rank));
    in_shape_.assign(shape, shape + rank);
    size_t n = 0;
    check(zr_session_num_io(s_, 1, &n));
    for (size_t i = 0; i < n; i++) {
        check(zr_session_io(s_, 1, i, &name, shape, &rank));
        out_shapes_.emplace_back(shape, shape + rank);
        out_names_.emplace_back(name);
    }
}

NeuralNetwork::~NeuralNetwork() { zr_session_destroy(s_); }

int64_t NeuralNetwork::output_per_image(size_t i) const {
    int64_t n = 1;
    for (size_t d = 1; d < out_shapes_[i].size(); d++) n *= out_shapes_[i][d];
    return n;
}

// Cnn::new / get_input_res (nn/mod.rs:46-106): exactly one [1,3,h,w] input
Cnn::Cnn(std::shared_ptr<NeuralNetwork> nn, ColorMapper cm) : nn_(std::move(nn)), cm_(cm) {
    const auto &s = nn_->input_shape();
    if (s.size() != 4 || s[1] != 3)
        throw ZaruError(ZR_ERR_SHAPE, "invalid model input shape for NCHW CNN");
    if (!(cm.hi > cm.lo)) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "ColorMapper needs end > start");
    in_h_ = (uint32_t)s[2];
    in_w_ = (uint32_t)s[3];
}

zr_view to_zr_view(const ViewData &v) {
    const Rect &r = v.rect.rect();
    return zr_view{r.center().x, r.center().y, r.width(), r.height(), v.rect.rotation_radians()};
}

std::vector<std::vector<float>> Cnn::estimate(const Image &img, const std::vector<ViewData> &views) const {
    if (img.on_device) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "estimate() takes a host image");
    std::vector<zr_view> zv;
    for (auto &v : views) zv.push_back(to_zr_view(v));
    std::vector<std::vector<float>> outs(nn_->num_outputs());
    std::vector<float *> ptrs;
    for (size_t i = 0; i < outs.size(); i++) {
        outs[i].resize((size_t)nn_->output_per_image(i) * views.size());
        ptrs.push_back(outs[i].data());
    }
    check(zr_cnn_estimate_views(nn_->handle(), img.rgba, img.width, img.height, img.row_stride,
                                zv.data(), zv.size(), cm_.lo, cm_.hi, ptrs.data()));
    return outs;
}

void Cnn::estimate_async(const std::vector<zr_frame> &frames, const std::vector<zr_view> &views,
                         const std::vector<uint32_t> &view_frame, float *const *d_outputs,
                         void *stream) const {
    if (views.empty()) return;
    check(zr_cnn_estimate_views_async(nn_->handle(), frames.data(), frames.size(), views.data(),
                                      view_frame.data(), views.size(), cm_.lo, cm_.hi, d_outputs,
                                      stream));
}

namespace {
std::mutex g_mu;
std::string g_models_dir;
std::map<std::pair<int, int>, std::shared_ptr<const Cnn>> g_cnns;
}  // namespace

void set_models_dir(const std::string &dir) {
    std::lock_guard<std::mutex> g(g_mu);
    g_models_dir = dir;
}

std::string models_dir() {
    std::lock_guard<std::mutex> g(g_mu);
    if (!g_models_dir.empty()) return g_models_dir;
    const char *e = std::getenv("ZARU_MODELS_DIR");
    return e ? e : "zaru_amd/models";
}

std::shared_ptr<const Cnn> network_cnn(NetworkKind k, int device) {
    const std::string dir = models_dir();
    std::lock_guard<std::mutex> g(g_mu);
    auto key = std::make_pair((int)k, device);
    auto it = g_cnns.find(key);
    if (it != g_cnns.end()) return it->second;
    const char *file = nullptr;
    ColorMapper cm;
    switch (k) {
    case NetworkKind::FaceDetectionShortRange:  // face/detection.rs:35-46
        file = "face_detection_short_range.onnx";
        cm = {-1.f, 1.f};
        break;
    case NetworkKind::FaceMeshV1:  // face/landmark/mediapipe.rs:46-57
        file = "face_landmark.onnx";
        cm = {-1.f, 1.f};
        break;
    case NetworkKind::PalmDetectionLite:  // hand/detection.rs:54-65
        file = "palm_detection_lite.onnx";
        cm = {0.f, 1.f};
        break;
    case NetworkKind::HandLandmarkLite:  // hand/landmark.rs:254-265
        file = "hand_landmark_lite.onnx";
        cm = {0.f, 1.f};
        break;
    case NetworkKind::FaceDetectionFullRange:  // face/detection.rs:67-79
        file = "face_detection_full_range.onnx";
        cm = {-1.f, 1.f};
        break;
    case NetworkKind::FaceMeshV2:  // face/landmark/mediapipe.rs:86-97 (fp16 weights, upcast at load)
        file = "face_landmarks_detector.onnx";
        cm = {-1.f, 1.f};
        break;
    case NetworkKind::IrisLandmark:  // face/eye.rs:33-46
        file = "iris_landmark.onnx";
        cm = {-1.f, 1.f};
        break;
    case NetworkKind::FaceOnnx68:  // face/landmark/multipie68.rs:93-106
        file = "landmarks_68_pfld.onnx";
        cm = {0.f, 1.f};
        break;
    case NetworkKind::PeppaFacialLandmark68:  // face/landmark/multipie68.rs:56-69
        file = "slim_160_latest.onnx";
        cm = {-1.f, 1.f};
        break;
    }
    auto nn = std::make_shared<NeuralNetwork>(read_file(dir + "/" + file), std::vector<uint32_t>{}, device);
    auto cnn = std::make_shared<const Cnn>(nn, cm);
    g_cnns[key] = cnn;
    return cnn;
}

}  // namespace zh
