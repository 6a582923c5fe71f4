// onnx_model.cpp -- protobuf wire-format reader for ModelProto (onnx/onnx.proto field
// numbers).  Malformed input is reported as an error string, never a crash: the reference
// surfaces loader failures as anyhow::Error (crates/zaru/src/nn/mod.rs:255-262).
#include "onnx_model.h"

#include <cstring>

namespace zr {
namespace {

struct Reader {
    const uint8_t *p, *end;
    bool ok = true;
    bool done() const { return p >= end || !ok; }
    uint64_t varint() {
        uint64_t r = 0;
        for (int s = 0; s < 64; s += 7) {
            if (p >= end) {
                ok = false;
                return 0;
            }
            uint8_t c = *p++;
            r |= (uint64_t)(c & 0x7F) << s;
            if (!(c & 0x80)) return r;
        }
        ok = false;
        return 0;
    }
};

struct Field {
    uint32_t num = 0, wire = 0;
    uint64_t v = 0;
    const uint8_t *data = nullptr;
    size_t len = 0;
};

bool next(Reader &r, Field &f) {
    if (r.done()) return false;
    uint64_t key = r.varint();
    if (!r.ok) return false;
    f.num = (uint32_t)(key >> 3);
    f.wire = (uint32_t)(key & 7);
    f.data = nullptr;
    f.len = 0;
    switch (f.wire) {
    case 0: f.v = r.varint(); break;
    case 1:
        if (r.end - r.p < 8) return r.ok = false;
        memcpy(&f.v, r.p, 8);
        r.p += 8;
        break;
    case 5: {
        if (r.end - r.p < 4) return r.ok = false;
        uint32_t t;
        memcpy(&t, r.p, 4);
        f.v = t;
        r.p += 4;
        break;
    }
    case 2: {
        uint64_t l = r.varint();
        if (!r.ok || (uint64_t)(r.end - r.p) < l) return r.ok = false;
        f.data = r.p;
        f.len = (size_t)l;
        r.p += l;
        break;
    }
    default: return r.ok = false;
    }
    return r.ok;
}

Reader sub(const Field &f) { return Reader{f.data, f.data + f.len}; }
std::string str(const Field &f) { return std::string((const char *)f.data, f.len); }

void packed_varints(const Field &f, std::vector<int64_t> &out) {
    if (f.wire == 0) {
        out.push_back((int64_t)f.v);
        return;
    }
    Reader r = sub(f);
    while (!r.done()) out.push_back((int64_t)r.varint());
}

float half_to_float(uint16_t h) {
    uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1F, m = h & 0x3FF, bits;
    if (e == 0) {
        if (m == 0) bits = s;
        else {  // subnormal
            e = 127 - 15 + 1;
            while (!(m & 0x400)) {
                m <<= 1;
                e--;
            }
            bits = s | (e << 23) | ((m & 0x3FF) << 13);
        }
    } else if (e == 31) bits = s | 0x7F800000u | (m << 13);
    else bits = s | ((e + 127 - 15) << 23) | (m << 13);
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

bool parse_tensor(Reader r, std::string &name, OnnxTensor &t, std::string &err) {
    Field f;
    const uint8_t *raw = nullptr;
    size_t raw_len = 0;
    std::vector<float> fdata;
    std::vector<int64_t> idata;
    std::vector<int64_t> i32data;
    while (next(r, f)) {
        switch (f.num) {
        case 1: packed_varints(f, t.dims); break;
        case 2: t.dtype = (int)f.v; break;
        case 4:
            if (f.wire == 5) {
                float v;
                memcpy(&v, &f.v, 4);
                fdata.push_back(v);
            } else {
                size_t n = f.len / 4;
                size_t o = fdata.size();
                fdata.resize(o + n);
                memcpy(fdata.data() + o, f.data, n * 4);
            }
            break;
        case 5: packed_varints(f, i32data); break;  // int32_data (also carries float16 bits)
        case 7: packed_varints(f, idata); break;
        case 8: name = str(f); break;
        case 9:
            raw = f.data;
            raw_len = f.len;
            break;
        default: break;
        }
    }
    if (!r.ok) {
        err = "malformed TensorProto";
        return false;
    }
    // untrusted dims: each >= 0 and the product bounded before anything is sized from it
    int64_t n = 1;
    for (int64_t d : t.dims) {
        if (d < 0 || (d > 0 && n > OnnxTensor::kMaxTensorElems / d))
            return err = "tensor " + name + ": negative or oversized dims", false;
        n *= d;
    }
    auto need = [&](size_t have, int64_t elem, const char *what) {
        if ((uint64_t)have != (uint64_t)n * (uint64_t)elem) {
            err = std::string(what) + " size mismatch for " + name;
            return false;
        }
        return true;
    };
    if (t.dtype == 1) {
        if (raw) {
            if (!need(raw_len, 4, "float raw_data")) return false;
            t.f.resize((size_t)n);
            memcpy(t.f.data(), raw, raw_len);
        } else {
            if (!need(fdata.size(), 1, "float_data")) return false;
            t.f = std::move(fdata);
        }
    } else if (t.dtype == 10) {
        if (raw ? !need(raw_len, 2, "float16 raw_data") : !need(i32data.size(), 1, "float16 int32_data"))
            return false;
        t.f.resize((size_t)n);
        for (int64_t i = 0; i < n; i++) {
            uint16_t h;
            if (raw) memcpy(&h, raw + 2 * i, 2);
            else h = (uint16_t)i32data[i];
            t.f[i] = half_to_float(h);
        }
        t.dtype = 1;
    } else if (t.dtype == 7) {
        if (raw) {
            if (!need(raw_len, 8, "int64 raw_data")) return false;
            t.i64.resize((size_t)n);
            memcpy(t.i64.data(), raw, raw_len);
        } else {
            if (!need(idata.size(), 1, "int64_data")) return false;
            t.i64 = std::move(idata);
        }
    } else if (t.dtype == 6) {  // int32 -> int64
        if (raw) {
            if (!need(raw_len, 4, "int32 raw_data")) return false;
            t.i64.resize((size_t)n);
            for (int64_t i = 0; i < n; i++) {
                int32_t v;
                memcpy(&v, raw + 4 * i, 4);
                t.i64[i] = v;
            }
        } else {
            if (!need(i32data.size(), 1, "int32_data")) return false;
            t.i64 = std::move(i32data);
        }
        t.dtype = 7;
    }
    return true;
}

bool parse_attr(Reader r, OnnxAttr &a) {
    Field f;
    while (next(r, f)) {
        switch (f.num) {
        case 1: a.name = str(f); break;
        case 2: memcpy(&a.f, &f.v, 4); break;
        case 3: a.i = (int64_t)f.v; break;
        case 4: a.s = str(f); break;
        case 7:
            if (f.wire == 5) {
                float v;
                memcpy(&v, &f.v, 4);
                a.floats.push_back(v);
            } else {
                size_t n = f.len / 4, o = a.floats.size();
                a.floats.resize(o + n);
                memcpy(a.floats.data() + o, f.data, n * 4);
            }
            break;
        case 8: packed_varints(f, a.ints); break;
        default: break;
        }
    }
    return r.ok;
}

bool parse_value_info(Reader r, OnnxValueInfo &vi) {
    Field f;
    while (next(r, f)) {
        if (f.num == 1) vi.name = str(f);
        else if (f.num == 2) {  // TypeProto
            Reader tr = sub(f);
            Field g;
            while (next(tr, g)) {
                if (g.num != 1) continue;  // tensor_type
                Reader tt = sub(g);
                Field h;
                while (next(tt, h)) {
                    if (h.num == 1) vi.elem = (int)h.v;
                    else if (h.num == 2) {  // shape
                        Reader sr = sub(h);
                        Field d;
                        while (next(sr, d)) {
                            if (d.num != 1) continue;
                            Reader dr = sub(d);
                            Field e;
                            int64_t v = -1;
                            while (next(dr, e))
                                if (e.num == 1) v = (int64_t)e.v;
                            vi.dims.push_back(v);
                        }
                    }
                }
            }
        }
    }
    return r.ok;
}

}  // namespace

bool parse_onnx(const uint8_t *data, size_t len, OnnxModel &m, std::string &err) {
    if (!data || len == 0) {
        err = "empty model";
        return false;
    }
    Reader r{data, data + len};
    Field f;
    Reader graph{nullptr, nullptr};
    bool have_graph = false;
    while (next(r, f)) {
        if (f.num == 7 && f.wire == 2) {
            graph = sub(f);
            have_graph = true;
        } else if (f.num == 8 && f.wire == 2) {  // OperatorSetIdProto
            Reader o = sub(f);
            Field g;
            std::string domain;
            int64_t ver = 0;
            while (next(o, g)) {
                if (g.num == 1) domain = str(g);
                else if (g.num == 2) ver = (int64_t)g.v;
            }
            if (domain.empty() || domain == "ai.onnx") m.opset = ver;
        }
    }
    if (!r.ok || !have_graph) {
        err = "not an ONNX ModelProto (no graph)";
        return false;
    }
    std::vector<OnnxValueInfo> all_inputs;
    while (next(graph, f)) {
        if (f.num == 1 && f.wire == 2) {
            OnnxNode nd;
            Reader nr = sub(f);
            Field g;
            while (next(nr, g)) {
                if (g.num == 1) nd.in.push_back(str(g));
                else if (g.num == 2) nd.out.push_back(str(g));
                else if (g.num == 3) nd.name = str(g);
                else if (g.num == 4) nd.op = str(g);
                else if (g.num == 5) {
                    OnnxAttr a;
                    if (!parse_attr(sub(g), a)) {
                        err = "malformed attribute";
                        return false;
                    }
                    nd.attrs.push_back(std::move(a));
                }
            }
            if (!nr.ok) {
                err = "malformed NodeProto";
                return false;
            }
            m.nodes.push_back(std::move(nd));
        } else if (f.num == 5 && f.wire == 2) {
            std::string name;
            OnnxTensor t;
            if (!parse_tensor(sub(f), name, t, err)) return false;
            m.inits[name] = std::move(t);
        } else if (f.num == 11 && f.wire == 2) {
            OnnxValueInfo vi;
            if (!parse_value_info(sub(f), vi)) {
                err = "malformed graph input";
                return false;
            }
            all_inputs.push_back(vi);
        } else if (f.num == 12 && f.wire == 2) {
            OnnxValueInfo vi;
            if (!parse_value_info(sub(f), vi)) {
                err = "malformed graph output";
                return false;
            }
            m.outputs.push_back(vi);
        }
    }
    if (!graph.ok) {
        err = "malformed GraphProto";
        return false;
    }
    for (auto &vi : all_inputs)
        if (!m.inits.count(vi.name)) m.inputs.push_back(vi);
    return true;
}

}  // namespace zr
