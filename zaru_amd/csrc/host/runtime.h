// runtime.h -- thin C++ handles over the C ABI (include/zaru_hip.h).  Host code above the
// boundary uses only these; it never includes HIP headers (the layering a Rust shim would
// have: crates/zaru/src/nn/mod.rs calling `Session::Hip`).
#pragma once
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/zaru_hip.h"

namespace zh {

struct ZaruError : std::runtime_error {
    int code;
    ZaruError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

inline void check(int rc) {
    if (rc != ZR_OK) throw ZaruError(rc, zr_last_error());
}

// An RGBA8 image (crates/zaru/src/image/mod.rs:47-51): host or device resident.
struct Image {
    const uint8_t *rgba = nullptr;
    uint32_t width = 0, height = 0;
    uint64_t row_stride = 0;
    bool on_device = false;
};

template <typename T>
struct DeviceArray {
    T *ptr = nullptr;
    size_t n = 0;
    DeviceArray() = default;
    explicit DeviceArray(size_t count) { resize(count); }
    DeviceArray(const DeviceArray &) = delete;
    DeviceArray &operator=(const DeviceArray &) = delete;
    ~DeviceArray() {
        if (ptr) zr_free(ptr);
    }
    void resize(size_t count) {
        if (count <= n) return;
        if (ptr) zr_free(ptr);
        ptr = nullptr;
        void *p = nullptr;
        check(zr_malloc(&p, count * sizeof(T)));
        ptr = static_cast<T *>(p);
        n = count;
    }
};

// Page-locked host array: device<->host copies into it stay asynchronous.
template <typename T>
struct PinnedArray {
    T *ptr = nullptr;
    size_t n = 0;
    PinnedArray() = default;
    PinnedArray(const PinnedArray &) = delete;
    PinnedArray &operator=(const PinnedArray &) = delete;
    ~PinnedArray() {
        if (ptr) zr_host_free(ptr);
    }
    void resize(size_t count) {
        if (count <= n) return;
        if (ptr) zr_host_free(ptr);
        ptr = nullptr;
        void *p = nullptr;
        check(zr_host_alloc(&p, count * sizeof(T)));
        ptr = static_cast<T *>(p);
        n = count;
    }
    T &operator[](size_t i) { return ptr[i]; }
    const T &operator[](size_t i) const { return ptr[i]; }
    T *data() { return ptr; }
};

// NeuralNetwork (crates/zaru/src/nn/mod.rs:365-539) = one HIP session.
class NeuralNetwork {
  public:
    NeuralNetwork(const std::vector<uint8_t> &onnx, const std::vector<uint32_t> &out_sel = {},
                  int device = 0);
    ~NeuralNetwork();
    NeuralNetwork(const NeuralNetwork &) = delete;
    NeuralNetwork &operator=(const NeuralNetwork &) = delete;

    zr_session *handle() const { return s_; }
    size_t num_outputs() const { return out_shapes_.size(); }
    const std::vector<int64_t> &input_shape() const { return in_shape_; }
    const std::vector<std::vector<int64_t>> &output_shapes() const { return out_shapes_; }
    const std::vector<std::string> &output_names() const { return out_names_; }
    int64_t output_per_image(size_t i) const;

  private:
    zr_session *s_ = nullptr;
    std::vector<int64_t> in_shape_;
    std::vector<std::vector<int64_t>> out_shapes_;
    std::vector<std::string> out_names_;
};

std::vector<uint8_t> read_file(const std::string &path);

}  // namespace zh
