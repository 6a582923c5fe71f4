// onnx_model.h -- in-memory ONNX graph (only what the CNN runner needs), parsed straight
// from the protobuf wire format (no libprotobuf/onnx dependency).  Replaces the graph
// loading that tract_onnx::onnx().model_for_read does for the reference
// (crates/zaru/src/nn/mod.rs:259-290).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace zr {

struct OnnxAttr {
    std::string name;
    float f = 0.f;
    int64_t i = 0;
    std::string s;
    std::vector<int64_t> ints;
    std::vector<float> floats;
};

struct OnnxNode {
    std::string op, name;
    std::vector<std::string> in, out;
    std::vector<OnnxAttr> attrs;
    const OnnxAttr *attr(const char *n) const {
        for (auto &a : attrs)
            if (a.name == n) return &a;
        return nullptr;
    }
    int64_t geti(const char *n, int64_t d) const {
        auto a = attr(n);
        return a ? a->i : d;
    }
    float getf(const char *n, float d) const {
        auto a = attr(n);
        return a ? a->f : d;
    }
    std::vector<int64_t> getints(const char *n, std::vector<int64_t> d = {}) const {
        auto a = attr(n);
        return a ? a->ints : d;
    }
    std::string gets(const char *n, const char *d = "") const {
        auto a = attr(n);
        return a ? a->s : std::string(d);
    }
};

struct OnnxTensor {
    std::vector<int64_t> dims;
    int dtype = 0;             // TensorProto.DataType: 1 float, 7 int64, 10 float16
    std::vector<float> f;      // float / float16 data (converted to f32)
    std::vector<int64_t> i64;  // int64 data
    // element count; only meaningful after parse_tensor validated the dims (each >= 0, product
    // <= kMaxTensorElems), so it cannot overflow
    int64_t numel() const {
        int64_t n = 1;
        for (auto d : dims) n *= d;
        return n;
    }
    static constexpr int64_t kMaxTensorElems = int64_t(1) << 30;  // 4 GiB of f32
};

struct OnnxValueInfo {
    std::string name;
    std::vector<int64_t> dims;
    int elem = 0;
};

struct OnnxModel {
    int64_t opset = 0;
    std::vector<OnnxNode> nodes;
    std::map<std::string, OnnxTensor> inits;
    std::vector<OnnxValueInfo> inputs, outputs;  // inputs exclude initializers
};

// Returns false and fills err on malformed input.
bool parse_onnx(const uint8_t *data, size_t len, OnnxModel &m, std::string &err);

}  // namespace zr
