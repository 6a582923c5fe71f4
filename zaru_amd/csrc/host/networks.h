// networks.h -- Cnn / ColorMapper (crates/zaru/src/nn/mod.rs:30-168) and the four hot-path
// network wrappers: face::detection::{ShortRangeNetwork, FullRangeNetwork},
// face::landmark::mediapipe::{FaceMeshV1, FaceMeshV2}, hand::detection::LiteNetwork,
// hand::landmark::LiteNetwork.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "geometry.h"
#include "runtime.h"

namespace zh {

struct ColorMapper {  // ColorMapper::linear (nn/mod.rs:146-154)
    float lo = 0.f, hi = 1.f;
};

class Cnn {
  public:
    Cnn(std::shared_ptr<NeuralNetwork> nn, ColorMapper cm);
    uint32_t input_width() const { return in_w_; }
    uint32_t input_height() const { return in_h_; }
    AspectRatio aspect() const { return AspectRatio::of(in_w_, in_h_); }
    const NeuralNetwork &nn() const { return *nn_; }
    ColorMapper color_mapper() const { return cm_; }

    // Cnn::estimate (nn/mod.rs:118-126) on views of one host image, batched: returns one host
    // vector per output holding views.size() * per-image floats.
    std::vector<std::vector<float>> estimate(const Image &img, const std::vector<ViewData> &views) const;

    // Device-resident variant over frames already in HBM (enqueue only).
    void estimate_async(const std::vector<zr_frame> &frames, const std::vector<zr_view> &views,
                        const std::vector<uint32_t> &view_frame, float *const *d_outputs,
                        void *stream) const;

  private:
    std::shared_ptr<NeuralNetwork> nn_;
    ColorMapper cm_;
    uint32_t in_w_ = 0, in_h_ = 0;
};

zr_view to_zr_view(const ViewData &v);

enum class NetworkKind {
    FaceDetectionShortRange,
    FaceMeshV1,
    PalmDetectionLite,
    HandLandmarkLite,
    FaceDetectionFullRange,
    FaceMeshV2,
    IrisLandmark,            // face::eye::EyeNetwork
    FaceOnnx68,              // face::landmark::multipie68::FaceOnnx (landmarks_68_pfld)
    PeppaFacialLandmark68,   // face::landmark::multipie68::PeppaFacialLandmark (slim_160)
};

inline bool is_face_mesh(NetworkKind k) { return k == NetworkKind::FaceMeshV1 || k == NetworkKind::FaceMeshV2; }
inline bool is_face_detector(NetworkKind k) {
    return k == NetworkKind::FaceDetectionShortRange || k == NetworkKind::FaceDetectionFullRange;
}

// Lazily loaded, process-wide CNN per (network, device) -- the reference's
// `static MODEL: OnceLock<Cnn>` (e.g. face/detection.rs:36-45).
std::shared_ptr<const Cnn> network_cnn(NetworkKind k, int device = 0);
void set_models_dir(const std::string &dir);
std::string models_dir();

}  // namespace zh
