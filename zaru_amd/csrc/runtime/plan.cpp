// plan.cpp -- ONNX graph -> fused HIP launch plan (see plan.h), and the plan executor.
#include "plan.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>

namespace zr {
namespace {

struct Val {
    std::vector<int64_t> shape;
    int tensor = -1;        // internal storage id when materialised
    int lazy = 0;           // 1: MaxPool 2x2/2 of lazy_src, 2: channel Pad of lazy_src,
                            // 3: ReduceMean over W of lazy_src (completed by the one over H)
    std::string lazy_src;
    int step = -1;          // producing step (after fusion aliasing)
    int consumers = 0;
    bool is_input = false;
    // graph-output placement
    int out_idx = -1;
    int64_t out_off = 0;
    bool nhwc = false;
};

int64_t per_image(const std::vector<int64_t> &s) {
    int64_t n = 1;
    for (size_t i = 1; i < s.size(); i++) n *= s[i];
    return n;
}

int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

class Compiler {
  public:
    Compiler(const OnnxModel &m, Plan &p, std::string &e) : M(m), P(p), err(e) {}

    bool run(const std::vector<uint32_t> &sel);

  private:
    const OnnxModel &M;
    Plan &P;
    std::string &err;
    std::map<std::string, Val> vals;
    std::map<std::string, int> producer;  // value -> node index
    std::set<int> layout_nodes;           // folded into store addressing
    std::vector<bool> needed;

    bool fail(const std::string &s) {
        err = s;
        return false;
    }
    const OnnxTensor *init(const std::string &n) const {
        auto it = M.inits.find(n);
        return it == M.inits.end() ? nullptr : &it->second;
    }
    Val &val(const std::string &n) { return vals[n]; }

    bool infer_shapes();
    bool trace_output(const std::string &name, int oi, int64_t off, bool nhwc);
    bool lower();
    bool lower_conv(const OnnxNode &nd);
    bool lower_gemm_node(const OnnxNode &nd);
    bool lower_act(const OnnxNode &nd);
    bool lower_add(const OnnxNode &nd);
    bool ensure_tensor(const std::string &name);
    TRef ref_of(const std::string &name);
    TRef out_ref(const std::string &name, int C, int H, int W);
    int new_storage(int64_t per_img) {
        P.storage_size.push_back(per_img);
        return (int)P.storage_size.size() - 1;
    }
    int64_t push_weights(const std::vector<float> &w) {
        int64_t off = (int64_t)P.weights.size();
        P.weights.insert(P.weights.end(), w.begin(), w.end());
        // keep every block 16-B aligned
        while (P.weights.size() % 4) P.weights.push_back(0.f);
        return off;
    }
    bool act_from_node(const OnnxNode &nd, int C, int Cpad, ActDesc &a);
    void finalize_outputs();
    void fuse_dw_gap();
    void group_siblings();
    void mark_inverted_residuals();
    void allocate();
};

// ---------------------------------------------------------------- shape inference
bool Compiler::infer_shapes() {
    for (auto &vi : M.inputs) {
        Val &v = val(vi.name);
        v.shape = vi.dims;
        if (!v.shape.empty() && v.shape[0] <= 0) v.shape[0] = 1;
        v.is_input = true;
    }
    for (auto &kv : M.inits) {
        // a float initializer must carry exactly numel values (the parser checked the raw
        // sizes; this also rejects dtypes that carry no f32 data, e.g. double weights)
        const OnnxTensor &t = kv.second;
        if (t.dtype == 1 && (int64_t)t.f.size() != t.numel()) return fail("initializer " + kv.first + ": no f32 data");
        val(kv.first).shape = t.dims;
    }
    for (auto &vi : M.inputs)
        for (size_t i = 1; i < vi.dims.size(); i++)
            if (vi.dims[i] <= 0 || vi.dims[i] > (1 << 16)) return fail("graph input " + vi.name + ": bad dims");
    // f32 weight operand with exactly the expected rank
    auto weight = [&](const std::string &n, size_t rank) -> const OnnxTensor * {
        const OnnxTensor *t = init(n);
        if (!t || t->dtype != 1 || t->dims.size() != rank) return nullptr;
        for (auto d : t->dims)
            if (d <= 0) return nullptr;
        return t;
    };
    for (size_t ni = 0; ni < M.nodes.size(); ni++) {
        const OnnxNode &nd = M.nodes[ni];
        const std::string &op = nd.op;
        // operand arity, and every operand must be a known value (graph input, initializer or
        // an earlier node's output: ONNX graphs are topologically sorted)
        const size_t arity = (op == "Conv" || op == "Add" || op == "PRelu" || op == "Gemm" ||
                              op == "Reshape") ? 2 : 1;
        if (nd.in.size() < arity || nd.out.empty() || nd.in[0].empty())
            return fail(op + " " + nd.name + ": missing operands");
        for (auto &i : nd.in)
            if (!i.empty() && !init(i) && (!vals.count(i) || vals[i].shape.empty()))
                return fail(op + " " + nd.name + ": operand " + i + " is not defined before use");
        for (auto &o : nd.out) producer[o] = (int)ni;
        for (auto &i : nd.in)
            if (!i.empty()) vals[i].consumers++;
        auto in = [&](int k) -> std::vector<int64_t> & { return val(nd.in[k]).shape; };
        std::vector<int64_t> s;
        if (op == "Conv") {
            auto &x = in(0);
            const OnnxTensor *w = weight(nd.in[1], 4);
            if (!w || x.size() != 4) return fail("Conv " + nd.name + ": unsupported operands");
            auto st = nd.getints("strides", {1, 1});
            auto pads = nd.getints("pads", {0, 0, 0, 0});
            const int64_t g = nd.geti("group", 1);
            if (st.size() != 2 || st[0] <= 0 || st[1] <= 0 || pads.size() != 4 ||
                *std::min_element(pads.begin(), pads.end()) < 0 || g <= 0 || x[1] != w->dims[1] * g ||
                w->dims[0] % g)
                return fail("Conv " + nd.name + ": bad strides/pads/group");
            if (nd.in.size() > 2 && !nd.in[2].empty()) {
                const OnnxTensor *b = weight(nd.in[2], 1);
                if (!b || b->dims[0] != w->dims[0]) return fail("Conv " + nd.name + ": bias shape");
            }
            if (nd.gets("auto_pad", "NOTSET") != "NOTSET") return fail("Conv auto_pad unsupported");
            int64_t oh = (x[2] + pads[0] + pads[2] - w->dims[2]) / st[0] + 1;
            int64_t ow = (x[3] + pads[1] + pads[3] - w->dims[3]) / st[1] + 1;
            s = {x[0], w->dims[0], oh, ow};
        } else if (op == "Relu" || op == "PRelu" || op == "Clip" || op == "Sigmoid" || op == "Add") {
            s = in(0);
            if (op == "Add" && in(1) != s) return fail("Add " + nd.name + ": broadcasting unsupported");
        } else if (op == "MaxPool") {
            auto &x = in(0);
            auto k = nd.getints("kernel_shape");
            auto st = nd.getints("strides", {1, 1});
            auto pads = nd.getints("pads", {0, 0, 0, 0});
            if (k.size() != 2 || st.size() != 2 || st[0] <= 0 || st[1] <= 0 || pads.size() != 4 || x.size() != 4)
                return fail("MaxPool kernel_shape/strides/pads");
            s = {x[0], x[1], (x[2] + pads[0] + pads[2] - k[0]) / st[0] + 1,
                 (x[3] + pads[1] + pads[3] - k[1]) / st[1] + 1};
        } else if (op == "Pad") {
            auto &x = in(0);
            std::vector<int64_t> pads;
            if (nd.in.size() > 1 && !nd.in[1].empty()) {
                const OnnxTensor *pt = init(nd.in[1]);
                if (!pt) return fail("Pad with dynamic pads unsupported");
                pads = pt->i64;
            } else
                pads = nd.getints("pads");
            if (pads.size() != 2 * x.size()) return fail("Pad rank");
            s = x;
            for (size_t i = 0; i < x.size(); i++) s[i] += pads[i] + pads[i + x.size()];
        } else if (op == "Resize") {
            auto &x = in(0);
            const OnnxTensor *sz = nd.in.size() > 3 && !nd.in[3].empty() ? init(nd.in[3]) : nullptr;
            const OnnxTensor *sc = nd.in.size() > 2 && !nd.in[2].empty() ? init(nd.in[2]) : nullptr;
            if (x.size() != 4) return fail("Resize of a non-4D tensor");
            if (sz && sz->i64.size() == 4) s = sz->i64;
            else if (sc && sc->f.size() == 4 && sc->f[2] > 0.f && sc->f[3] > 0.f && sc->f[2] <= 64.f &&
                     sc->f[3] <= 64.f)
                s = {x[0], x[1], (int64_t)std::floor(x[2] * sc->f[2]), (int64_t)std::floor(x[3] * sc->f[3])};
            else return fail("Resize needs constant sizes or scales");
        } else if (op == "GlobalAveragePool") {
            auto &x = in(0);
            s = {x[0], x[1], 1, 1};
        } else if (op == "AveragePool") {
            auto &x = in(0);
            auto k = nd.getints("kernel_shape");
            auto st = nd.getints("strides", {1, 1});
            auto pads = nd.getints("pads", {0, 0, 0, 0});
            if (k.size() != 2 || st.size() != 2 || st[0] <= 0 || st[1] <= 0 || pads.size() != 4 || x.size() != 4 ||
                k[0] <= 0 || k[1] <= 0 || nd.geti("ceil_mode", 0))
                return fail("AveragePool kernel_shape/strides/pads");
            s = {x[0], x[1], (x[2] + pads[0] + pads[2] - k[0]) / st[0] + 1,
                 (x[3] + pads[1] + pads[3] - k[1]) / st[1] + 1};
        } else if (op == "ReduceMean") {
            auto &x = in(0);
            auto axes = nd.getints("axes");
            if (axes.empty() && nd.in.size() > 1 && init(nd.in[1])) axes = init(nd.in[1])->i64;
            const bool keep = nd.geti("keepdims", 1) != 0;
            if (axes.empty()) return fail("ReduceMean over all axes unsupported");
            for (size_t i = 0; i < x.size(); i++) {
                bool red = false;
                for (auto a : axes)
                    if (a == (int64_t)i || a + (int64_t)x.size() == (int64_t)i) red = true;
                if (red && i < 2) return fail("ReduceMean over batch/channels unsupported");
                if (!red) s.push_back(x[i]);
                else if (keep) s.push_back(1);
            }
        } else if (op == "Squeeze") {
            auto &x = in(0);
            auto axes = nd.getints("axes");
            if (axes.empty() && nd.in.size() > 1 && init(nd.in[1])) axes = init(nd.in[1])->i64;
            for (size_t i = 0; i < x.size(); i++) {
                bool drop = false;
                for (auto a : axes)
                    if (a == (int64_t)i || a + (int64_t)x.size() == (int64_t)i) drop = true;
                if (axes.empty() && x[i] == 1 && i > 0) drop = true;
                if (!drop) s.push_back(x[i]);
            }
        } else if (op == "Flatten") {
            auto &x = in(0);
            s = {x[0], per_image(x)};
        } else if (op == "Reshape") {
            auto &x = in(0);
            const OnnxTensor *t = init(nd.in[1]);
            if (!t) return fail("Reshape with dynamic shape unsupported");
            int64_t known = 1;
            int neg = -1;
            for (size_t i = 0; i < t->i64.size(); i++) {
                if (t->i64[i] == 0 && i >= x.size()) return fail("Reshape copies a missing dim");
                int64_t d = t->i64[i] == 0 ? x[i] : t->i64[i];
                if (d == -1 && neg < 0) neg = (int)i;
                else if (d <= 0) return fail("Reshape dims");
                else known *= d;
                s.push_back(d);
            }
            int64_t total = 1;
            for (auto d : x) total *= d;
            if (neg >= 0) s[neg] = total / known;
            int64_t got = 1;
            for (auto d : s) got *= d;
            if (got != total) return fail("Reshape changes the element count");
        } else if (op == "Transpose") {
            auto &x = in(0);
            auto perm = nd.getints("perm");
            if (perm.size() != x.size()) return fail("Transpose perm");
            for (auto p : perm) {
                if (p < 0 || p >= (int64_t)x.size()) return fail("Transpose perm");
                s.push_back(x[p]);
            }
        } else if (op == "Concat") {
            s = in(0);
            int64_t ax = nd.geti("axis", 0);
            if (ax < 0) ax += (int64_t)s.size();
            if (ax < 0 || ax >= (int64_t)s.size()) return fail("Concat axis");
            for (size_t k = 1; k < nd.in.size(); k++) {
                if (nd.in[k].empty() || in((int)k).size() != s.size()) return fail("Concat operands");
                s[ax] += in((int)k)[ax];
            }
        } else if (op == "Gemm") {
            auto &a = in(0);
            const OnnxTensor *b = weight(nd.in[1], 2);
            if (!b || a.size() != 2) return fail("Gemm operands");
            const bool tb = nd.geti("transB", 0) != 0;
            if (a[1] != (tb ? b->dims[1] : b->dims[0])) return fail("Gemm K mismatch");
            int64_t m = tb ? b->dims[0] : b->dims[1];
            if (nd.in.size() > 2 && !nd.in[2].empty()) {
                const OnnxTensor *c = init(nd.in[2]);
                if (!c || c->dtype != 1 || (c->f.size() != 1 && (int64_t)c->f.size() != m))
                    return fail("Gemm bias shape");
            }
            s = {a[0], m};
        } else {
            return fail("unsupported operator " + op + " (" + nd.name + ")");
        }
        // every produced shape: positive dims, bounded per-image size (kernels address with
        // 32-bit element offsets)
        if (s.empty()) return fail(op + " " + nd.name + ": empty shape");
        int64_t pi = 1;
        for (size_t i = 0; i < s.size(); i++) {
            if (s[i] <= 0 || s[i] > (1 << 24)) return fail(op + " " + nd.name + ": bad output shape");
            if (i > 0) {
                pi *= s[i];
                if (pi > (int64_t(1) << 28)) return fail(op + " " + nd.name + ": tensor too large");
            }
        }
        for (auto &o : nd.out) val(o).shape = s;
    }
    return true;
}

// ---------------------------------------------------------------- output placement
bool Compiler::trace_output(const std::string &name, int oi, int64_t off, bool nhwc) {
    auto it = producer.find(name);
    if (it == producer.end()) return fail("graph output " + name + " is not computed");
    const OnnxNode &nd = M.nodes[it->second];
    if (nd.op == "Concat") {
        int64_t ax = nd.geti("axis", 0);
        if (ax < 0) ax += (int64_t)val(name).shape.size();
        if (ax != 1) return fail("Concat on axis != 1 cannot be folded");
        layout_nodes.insert(it->second);
        int64_t o = off;
        for (auto &i : nd.in) {
            if (!trace_output(i, oi, o, nhwc)) return false;
            o += per_image(val(i).shape);
        }
        return true;
    }
    if (nd.op == "Reshape" || nd.op == "Squeeze" || nd.op == "Flatten") {
        if (val(nd.in[0]).consumers != 1) return fail("layout node input has other consumers");
        layout_nodes.insert(it->second);
        return trace_output(nd.in[0], oi, off, nhwc);
    }
    if (nd.op == "Transpose") {
        auto perm = nd.getints("perm");
        if (perm != std::vector<int64_t>{0, 2, 3, 1} || nhwc)
            return fail("only NCHW->NHWC output transposes can be folded");
        if (val(nd.in[0]).consumers != 1) return fail("transposed tensor has other consumers");
        layout_nodes.insert(it->second);
        return trace_output(nd.in[0], oi, off, true);
    }
    Val &v = val(name);
    if (v.out_idx >= 0) return fail("value feeds two graph outputs");
    v.out_idx = oi;
    v.out_off = off;
    v.nhwc = nhwc;
    return true;
}

// ---------------------------------------------------------------- helpers
TRef Compiler::ref_of(const std::string &name) {
    Val &v = val(name);
    TRef r;
    auto &s = v.shape;
    r.C = (int)s[1];
    r.H = s.size() > 2 ? (int)s[2] : 1;
    r.W = s.size() > 3 ? (int)s[3] : 1;
    if (v.is_input) {
        r.kind = 1;
        r.id = 0;
    } else {
        r.kind = 0;
        r.id = v.tensor;
    }
    return r;
}

// destination of a step producing `name` (graph output buffer or a fresh arena slot)
TRef Compiler::out_ref(const std::string &name, int C, int H, int W) {
    Val &v = val(name);
    TRef r;
    r.C = C;
    r.H = H;
    r.W = W;
    if (v.out_idx >= 0) {
        r.kind = 2;
        r.id = v.out_idx;
        r.off = v.out_off;
        r.o_sN = P.outputs[v.out_idx].per_image;
        if (v.nhwc) {
            r.o_sC = 1;
            r.o_sP = C;
        } else {
            r.o_sC = (int64_t)H * W;
            r.o_sP = 1;
        }
    } else {
        r.kind = 0;
        r.id = new_storage((int64_t)C * H * W);
        v.tensor = r.id;
    }
    return r;
}

bool Compiler::ensure_tensor(const std::string &name) {
    Val &v = val(name);
    if (v.is_input || v.tensor >= 0) return true;
    if (v.out_idx >= 0) return fail("graph output " + name + " is also consumed internally");
    if (!v.lazy) return fail("value " + name + " was never materialised");
    if (v.lazy == 3) return fail("partial ReduceMean " + name + " is consumed by other than its H mean");
    if (!ensure_tensor(v.lazy_src)) return false;
    Step s;
    s.kind = S_ELT;
    s.name = name;
    s.elt_op = v.lazy == 1 ? 2 : 3;
    s.in = ref_of(v.lazy_src);
    auto &sh = val(name).shape;
    s.out = out_ref(name, (int)sh[1], (int)sh[2], (int)sh[3]);
    s.bytes = 4.0 * (per_image(val(v.lazy_src).shape) + per_image(sh));
    P.steps.push_back(s);
    val(name).step = (int)P.steps.size() - 1;
    return true;
}

bool Compiler::act_from_node(const OnnxNode &nd, int C, int Cpad, ActDesc &a) {
    if (nd.op == "Relu") a.kind = ACT_RELU;
    else if (nd.op == "Sigmoid") a.kind = ACT_SIGMOID;
    else if (nd.op == "Clip") {
        a.kind = ACT_CLIP;
        a.lo = nd.getf("min", -3.402823466e38f);
        a.hi = nd.getf("max", 3.402823466e38f);
        if (nd.in.size() > 1 && !nd.in[1].empty()) {
            const OnnxTensor *t = init(nd.in[1]);
            if (!t || t->f.empty()) return fail("Clip min must be constant");
            a.lo = t->f[0];
        }
        if (nd.in.size() > 2 && !nd.in[2].empty()) {
            const OnnxTensor *t = init(nd.in[2]);
            if (!t || t->f.empty()) return fail("Clip max must be constant");
            a.hi = t->f[0];
        }
    } else if (nd.op == "PRelu") {
        const OnnxTensor *t = init(nd.in[1]);
        if (!t || (t->f.size() != (size_t)C && t->f.size() != 1)) return fail("PRelu slope shape");
        std::vector<float> sl(std::max(C, Cpad), 0.f);
        for (int c = 0; c < C; c++) sl[c] = t->f.size() == 1 ? t->f[0] : t->f[c];
        a.kind = ACT_PRELU;
        a.slope_off = push_weights(sl);
    } else
        return false;
    return true;
}

// ---------------------------------------------------------------- lowering
bool Compiler::lower_conv(const OnnxNode &nd) {
    const std::string &xn = nd.in[0];
    if (!ensure_tensor(xn)) return false;
    const OnnxTensor *w = init(nd.in[1]);
    const OnnxTensor *b = nd.in.size() > 2 && !nd.in[2].empty() ? init(nd.in[2]) : nullptr;
    if (!w || (nd.in.size() > 2 && !nd.in[2].empty() && !b)) return fail("Conv weights must be constant");
    auto &xs = val(xn).shape;
    auto &ys = val(nd.out[0]).shape;
    const int Cin = (int)xs[1], H = (int)xs[2], W = (int)xs[3];
    const int Mo = (int)w->dims[0], Cg = (int)w->dims[1], kh = (int)w->dims[2], kw = (int)w->dims[3];
    const int OH = (int)ys[2], OW = (int)ys[3];
    const int64_t g = nd.geti("group", 1);
    auto st = nd.getints("strides", {1, 1});
    auto pads = nd.getints("pads", {0, 0, 0, 0});
    auto dil = nd.getints("dilations", {1, 1});
    if (dil[0] != 1 || dil[1] != 1) return fail("dilated Conv unsupported");
    std::vector<float> bias(Mo, 0.f);
    if (b) bias = b->f;

    Step s;
    s.name = nd.name.empty() ? nd.out[0] : nd.name;
    s.in = ref_of(xn);
    s.kh = kh;
    s.kw = kw;
    s.stride = (int)st[0];
    s.pad_t = (int)pads[0];
    s.pad_l = (int)pads[1];
    s.flops = 2.0 * Mo * (double)Cg * kh * kw * OH * OW;
    s.bytes = 4.0 * ((double)Cin * H * W + (double)Mo * OH * OW);

    const bool depthwise = g == Cin && Mo == Cin && Cg == 1 && kh == kw && (kh == 3 || kh == 5) &&
                           st[0] == st[1] && (st[0] == 1 || st[0] == 2);
    const bool pointwise = g == 1 && kh == 1 && kw == 1 && st[0] == 1 && st[1] == 1 &&
                           pads[0] == 0 && pads[1] == 0 && pads[2] == 0 && pads[3] == 0;
    const bool fullplane = g == 1 && kh == H && kw == W && OH == 1 && OW == 1 && pads[0] == 0 &&
                           pads[1] == 0 && pads[2] == 0 && pads[3] == 0 && (kw >= 2 || kh == 1);
    // non-overlapping patches (kernel == stride, no padding: FaceMesh V2's 2x2/2 downsampling
    // convs) are a GEMM over k = (ci, ky, kx) whose B operand gathers each output's patch
    const bool patch = g == 1 && kh == kw && st[0] == kh && st[1] == kw && kh >= 2 && kh <= 4 &&
                       pads[0] == 0 && pads[1] == 0 && pads[2] == 0 && pads[3] == 0 &&
                       H % kh == 0 && W % kw == 0 && !fullplane;
    if (depthwise) {
        s.kind = S_DW;
        s.w_off = push_weights(w->f);
        s.b_off = push_weights(bias);
    } else if (pointwise || fullplane || patch) {
        s.kind = S_GEMM;
        s.in2 = TRef{};
        s.KK = kh * kw;
        s.M = Mo;
        s.K = Cin * s.KK;
        s.Mpad = (int)round_up(Mo, 32);
        s.Kpad = (int)round_up(s.K, 2);
        std::vector<float> wt((size_t)s.Kpad * s.Mpad, 0.f);
        for (int m = 0; m < Mo; m++)
            for (int k = 0; k < s.K; k++) wt[(size_t)k * s.Mpad + m] = w->f[(size_t)m * s.K + k];
        s.w_off = push_weights(wt);
        bias.resize(s.Mpad, 0.f);
        s.b_off = push_weights(bias);
    } else if (g == 1 && st[0] == st[1]) {
        s.kind = S_DIRECT;
        s.M = Mo;
        s.stem = kh == kw && stem_supported(Cin, kh, (int)st[0], Mo);
        std::vector<float> wf = w->f;
        if (s.stem) {  // stem_kernel: [Cin][kh][kw][32], output channel innermost, zero-padded
            wf.assign((size_t)32 * Cin * kh * kw, 0.f);
            for (int m = 0; m < Mo; m++)
                for (int t = 0; t < Cin * kh * kw; t++) wf[(size_t)t * 32 + m] = w->f[(size_t)m * Cin * kh * kw + t];
            bias.resize(32, 0.f);
        }
        s.w_off = push_weights(wf);
        s.b_off = push_weights(bias);
        s.bytes_pre = 4.0 * ((double)H * W + (double)Mo * OH * OW);
    } else {
        return fail("Conv " + s.name + ": unsupported configuration");
    }
    // A 1x1 conv whose input is a depthwise conv's private output (the step just lowered)
    // absorbs it: the depthwise result then never leaves the CU (fused.hip dwpw_kernel).
    if (pointwise && !P.steps.empty()) {
        Val &xv = val(xn);
        const Step &d = P.steps.back();
        if (xv.step == (int)P.steps.size() - 1 && xv.consumers == 1 && xv.out_idx < 0 &&
            d.kind == S_DW && d.out.kind == 0 && dwpw_supported(d.kh, d.stride)) {
            Step f = s;
            f.kind = S_DWPW;
            f.in = d.in;
            f.kh = d.kh;
            f.kw = d.kw;
            f.stride = d.stride;
            f.pad_t = d.pad_t;
            f.pad_l = d.pad_l;
            f.dw_w_off = d.w_off;
            f.dw_b_off = d.b_off;
            f.dw_act = d.pre;
            f.flops = d.flops + s.flops;
            // depthwise input read + 1x1 output write; the intermediate is on chip
            f.bytes = 4.0 * ((double)d.in.C * d.in.H * d.in.W + (double)Mo * OH * OW);
            P.steps.pop_back();
            s = f;
        }
    }
    s.out = out_ref(nd.out[0], Mo, OH, OW);
    P.steps.push_back(s);
    val(nd.out[0]).step = (int)P.steps.size() - 1;
    return true;
}

bool Compiler::lower_gemm_node(const OnnxNode &nd) {
    const std::string &an = nd.in[0];
    if (!ensure_tensor(an)) return false;
    const OnnxTensor *bm = init(nd.in[1]);
    const OnnxTensor *cb = nd.in.size() > 2 && !nd.in[2].empty() ? init(nd.in[2]) : nullptr;
    if (!bm || (nd.in.size() > 2 && !nd.in[2].empty() && !cb)) return fail("Gemm weights must be constant");
    if (nd.geti("transA", 0)) return fail("Gemm transA unsupported");
    const float alpha = nd.getf("alpha", 1.f), beta = nd.getf("beta", 1.f);
    const bool tb = nd.geti("transB", 0) != 0;
    const int K = (int)(tb ? bm->dims[1] : bm->dims[0]), Mo = (int)(tb ? bm->dims[0] : bm->dims[1]);
    TRef in = ref_of(an);
    if (in.C * in.H * in.W != K) return fail("Gemm K mismatch");
    Step s;
    s.kind = S_GEMM;
    s.name = nd.name.empty() ? nd.out[0] : nd.name;
    s.in = in;
    s.KK = 1;
    s.M = Mo;
    s.K = K;
    s.Mpad = (int)round_up(Mo, 32);
    s.Kpad = (int)round_up(K, 2);
    std::vector<float> wt((size_t)s.Kpad * s.Mpad, 0.f);
    for (int k = 0; k < K; k++)
        for (int m = 0; m < Mo; m++)
            wt[(size_t)k * s.Mpad + m] = alpha * (tb ? bm->f[(size_t)m * K + k] : bm->f[(size_t)k * Mo + m]);
    s.w_off = push_weights(wt);
    std::vector<float> bias(s.Mpad, 0.f);
    if (cb)
        for (int m = 0; m < Mo; m++) bias[m] = beta * (cb->f.size() == 1 ? cb->f[0] : cb->f[m]);
    s.b_off = push_weights(bias);
    s.flops = 2.0 * K * Mo;
    s.bytes = 4.0 * (K + Mo);
    s.out = out_ref(nd.out[0], Mo, 1, 1);
    P.steps.push_back(s);
    val(nd.out[0]).step = (int)P.steps.size() - 1;
    return true;
}

bool Compiler::lower_act(const OnnxNode &nd) {
    const std::string &xn = nd.in[0];
    Val &x = val(xn);
    auto &sh = val(nd.out[0]).shape;
    const int C = (int)sh[1];
    // fold into the producing step when this activation is its only consumer
    if (x.step >= 0 && x.consumers == 1 && x.out_idx < 0) {
        Step &s = P.steps[x.step];
        ActDesc a;
        const bool gemm = s.kind == S_GEMM || s.kind == S_DWPW;
        const int Cpad = gemm ? s.Mpad : (s.stem ? std::max(C, 32) : C);
        ActDesc *slot = nullptr;
        if (gemm) slot = s.res_mode ? &s.post : (s.pre.kind ? nullptr : &s.pre);
        else if (s.kind == S_DW || s.kind == S_DIRECT || s.kind == S_ELT) slot = s.pre.kind ? nullptr : &s.pre;
        if (gemm && s.res_mode && s.post.kind) slot = nullptr;
        if (slot) {
            if (!act_from_node(nd, C, Cpad, a)) return false;
            *slot = a;
            Val &y = val(nd.out[0]);
            y.step = x.step;
            // re-target the step output to the activation's value
            if (y.out_idx >= 0) {
                if (s.out.kind != 0) return fail("double output placement");
                TRef r = out_ref(nd.out[0], s.out.C, s.out.H, s.out.W);
                s.out = r;
            } else {
                y.tensor = x.tensor;
            }
            x.tensor = -1;
            return true;
        }
    }
    if (!ensure_tensor(xn)) return false;
    Step s;
    s.kind = S_ELT;
    s.name = nd.name.empty() ? nd.out[0] : nd.name;
    s.elt_op = 0;
    s.in = ref_of(xn);
    if (!act_from_node(nd, C, C, s.pre)) return false;
    s.out = out_ref(nd.out[0], C, (int)(sh.size() > 2 ? sh[2] : 1), (int)(sh.size() > 3 ? sh[3] : 1));
    s.bytes = 8.0 * per_image(sh);
    P.steps.push_back(s);
    val(nd.out[0]).step = (int)P.steps.size() - 1;
    return true;
}

bool Compiler::lower_add(const OnnxNode &nd) {
    auto &sh = val(nd.out[0]).shape;
    if (sh.size() != 4) return fail("Add on non-4D tensors unsupported");
    for (int side = 0; side < 2; side++) {
        const std::string &pn = nd.in[side], &rn = nd.in[1 - side];
        Val &p = val(pn);
        if (p.step < 0 || p.consumers != 1 || p.out_idx >= 0) continue;
        const int si = p.step;
        if ((P.steps[si].kind != S_GEMM && P.steps[si].kind != S_DWPW) || P.steps[si].res_mode ||
            P.steps[si].post.kind)
            continue;
        // resolve the shortcut through lazily kept Pad / MaxPool nodes
        std::string r = rn;
        int rc = (int)val(r).shape[1];
        bool pool = false;
        if (val(r).lazy == 2) {
            r = val(r).lazy_src;
            rc = (int)val(r).shape[1];
        }
        if (val(r).lazy == 1) {
            pool = true;
            r = val(r).lazy_src;
        }
        if (!ensure_tensor(r)) return false;  // may append steps: index P.steps afresh below
        Step &s = P.steps[si];
        auto &rs = val(r).shape;
        if (pool ? (rs[2] / 2 != sh[2] || rs[3] / 2 != sh[3]) : (rs[2] != sh[2] || rs[3] != sh[3]))
            continue;
        if (rc > s.M) continue;
        s.res_mode = pool ? 2 : 1;
        s.r_C = rc;
        s.in2 = ref_of(r);
        s.bytes += 4.0 * rc * (double)sh[2] * sh[3] * (pool ? 4 : 1);
        Val &y = val(nd.out[0]);
        y.step = p.step;
        if (y.out_idx >= 0) {
            s.out = out_ref(nd.out[0], s.out.C, s.out.H, s.out.W);
        } else {
            y.tensor = p.tensor;
        }
        p.tensor = -1;
        // The shortcut may come from a step emitted after the conv this Add fuses into (BlazeFace
        // full range's FPN: conv(12^2 features) + Resize(6^2 branch), the conv first in ONNX
        // order).  The fused step then runs after the shortcut's producer: nothing between reads
        // the conv's output (its one consumer is this Add), so moving it to the end is safe.
        if (val(r).step > si) {
            Step moved = P.steps[si];
            P.steps.erase(P.steps.begin() + si);
            P.steps.push_back(std::move(moved));
            const int last = (int)P.steps.size() - 1;
            for (auto &kv : vals) {
                if (kv.second.step == si) kv.second.step = last;
                else if (kv.second.step > si) kv.second.step--;
            }
        }
        return true;
    }
    if (!ensure_tensor(nd.in[0]) || !ensure_tensor(nd.in[1])) return false;
    Step s;
    s.kind = S_ELT;
    s.name = nd.name.empty() ? nd.out[0] : nd.name;
    s.elt_op = 1;
    s.in = ref_of(nd.in[0]);
    s.in2 = ref_of(nd.in[1]);
    s.out = out_ref(nd.out[0], (int)sh[1], (int)sh[2], (int)sh[3]);
    s.bytes = 12.0 * per_image(sh);
    P.steps.push_back(s);
    val(nd.out[0]).step = (int)P.steps.size() - 1;
    return true;
}

bool Compiler::lower() {
    for (size_t ni = 0; ni < M.nodes.size(); ni++) {
        if (!needed[ni] || layout_nodes.count((int)ni)) continue;
        const OnnxNode &nd = M.nodes[ni];
        const std::string &op = nd.op;
        if (op == "Conv") {
            if (!lower_conv(nd)) return false;
        } else if (op == "Gemm") {
            if (!lower_gemm_node(nd)) return false;
        } else if (op == "Relu" || op == "PRelu" || op == "Clip" || op == "Sigmoid") {
            if (!lower_act(nd)) return false;
        } else if (op == "Add") {
            if (!lower_add(nd)) return false;
        } else if (op == "MaxPool") {
            auto k = nd.getints("kernel_shape");
            auto st = nd.getints("strides", {1, 1});
            auto pads = nd.getints("pads", {0, 0, 0, 0});
            if (k != std::vector<int64_t>{2, 2} || st != std::vector<int64_t>{2, 2} ||
                pads != std::vector<int64_t>{0, 0, 0, 0} || nd.geti("ceil_mode", 0))
                return fail("only MaxPool 2x2/2 without padding is supported");
            Val &y = val(nd.out[0]);
            y.lazy = 1;
            y.lazy_src = nd.in[0];
            if (y.out_idx >= 0 && !ensure_tensor(nd.out[0])) return false;
        } else if (op == "Pad") {
            auto &xs = val(nd.in[0]).shape, &ys = val(nd.out[0]).shape;
            std::vector<int64_t> pads = nd.in.size() > 1 && !nd.in[1].empty() ? init(nd.in[1])->i64
                                                                              : nd.getints("pads");
            if (pads.size() != 8) return fail("Pad rank");
            const std::string mode = nd.gets("mode", "constant");
            float cval = 0.f;
            if (nd.in.size() > 2 && !nd.in[2].empty()) {
                const OnnxTensor *t = init(nd.in[2]);
                if (!t || t->f.empty()) return fail("Pad value must be constant");
                cval = t->f[0];
            } else
                cval = nd.getf("value", 0.f);
            bool chan_only = xs.size() == 4 && mode == "constant" && cval == 0.f;
            for (size_t i = 0; i < pads.size() && chan_only; i++)
                if (i != 5 && pads[i] != 0) chan_only = false;
            if (!chan_only || ys[1] < xs[1]) return fail("only trailing channel zero-padding is supported");
            Val &y = val(nd.out[0]);
            y.lazy = 2;
            y.lazy_src = nd.in[0];
            if (y.out_idx >= 0 && !ensure_tensor(nd.out[0])) return false;
        } else if (op == "Resize") {
            if (nd.gets("mode", "nearest") != "linear" ||
                nd.gets("coordinate_transformation_mode", "half_pixel") != "half_pixel")
                return fail("only linear/half_pixel Resize is supported");
            if (!ensure_tensor(nd.in[0])) return false;
            auto &xs = val(nd.in[0]).shape, &ys = val(nd.out[0]).shape;
            Step s;
            s.kind = S_RESIZE;
            s.name = nd.name;
            s.in = ref_of(nd.in[0]);
            s.scale_y = (float)xs[2] / (float)ys[2];
            s.scale_x = (float)xs[3] / (float)ys[3];
            s.out = out_ref(nd.out[0], (int)ys[1], (int)ys[2], (int)ys[3]);
            s.bytes = 4.0 * (per_image(xs) + per_image(ys));
            P.steps.push_back(s);
            val(nd.out[0]).step = (int)P.steps.size() - 1;
        } else if (op == "GlobalAveragePool") {
            if (!ensure_tensor(nd.in[0])) return false;
            auto &xs = val(nd.in[0]).shape;
            Step s;
            s.kind = S_GAP;
            s.name = nd.name;
            s.in = ref_of(nd.in[0]);
            s.out = out_ref(nd.out[0], (int)xs[1], 1, 1);
            s.bytes = 4.0 * (per_image(xs) + xs[1]);
            P.steps.push_back(s);
            val(nd.out[0]).step = (int)P.steps.size() - 1;
        } else if (op == "AveragePool" || op == "ReduceMean") {
            // global average pooling in its two spellings: an AveragePool whose window is the
            // whole plane (landmarks_68_pfld), and ReduceMean over W then over H (slim_160) or
            // over both at once.  ReduceMean over W alone stays lazy until the H mean follows.
            auto &xs = val(nd.in[0]).shape;
            std::string src = nd.in[0];
            bool gap = false;
            if (op == "AveragePool") {
                auto k = nd.getints("kernel_shape");
                auto pads = nd.getints("pads", {0, 0, 0, 0});
                gap = xs.size() == 4 && k.size() == 2 && k[0] == xs[2] && k[1] == xs[3] &&
                      pads == std::vector<int64_t>{0, 0, 0, 0};
                if (!gap) return fail("only whole-plane AveragePool is supported");
            } else {
                auto axes = nd.getints("axes");
                if (axes.empty() && nd.in.size() > 1 && init(nd.in[1])) axes = init(nd.in[1])->i64;
                std::set<int64_t> ax;
                for (auto a : axes) ax.insert(a < 0 ? a + (int64_t)xs.size() : a);
                if (xs.size() == 4 && ax == std::set<int64_t>{2, 3}) {
                    gap = true;
                } else if (xs.size() == 4 && ax == std::set<int64_t>{3} && nd.geti("keepdims", 1) == 0) {
                    Val &y = val(nd.out[0]);
                    y.lazy = 3;
                    y.lazy_src = nd.in[0];
                    continue;
                } else if (xs.size() == 3 && ax == std::set<int64_t>{2} && val(nd.in[0]).lazy == 3) {
                    src = val(nd.in[0]).lazy_src;  // mean over H of the mean over W
                    gap = true;
                } else {
                    return fail("ReduceMean pattern unsupported (only the spatial mean)");
                }
            }
            if (!gap || !ensure_tensor(src)) return false;
            auto &ss = val(src).shape;
            Step s;
            s.kind = S_GAP;
            s.name = nd.name.empty() ? nd.out[0] : nd.name;
            s.in = ref_of(src);
            s.out = out_ref(nd.out[0], (int)ss[1], 1, 1);
            s.bytes = 4.0 * (per_image(ss) + ss[1]);
            P.steps.push_back(s);
            val(nd.out[0]).step = (int)P.steps.size() - 1;
        } else if (op == "Concat") {
            // channel Concat of per-image vectors feeding an internal consumer (the pooled
            // multi-scale features of the 68-point nets): each member's producing step writes
            // straight into its channel range of one storage, so no copy runs
            if (nd.geti("axis", 0) != 1 && nd.geti("axis", 0) != -(int64_t)val(nd.out[0]).shape.size() + 1)
                return fail("internal Concat on axis != 1 unsupported");
            auto &ys = val(nd.out[0]).shape;
            if (per_image(ys) != ys[1]) return fail("internal Concat of non-vector tensors unsupported");
            if (val(nd.out[0]).out_idx >= 0) return fail("unexpected output placement on Concat");
            const int id = new_storage(ys[1]);
            int c0 = 0;
            for (auto &in_name : nd.in) {
                if (!ensure_tensor(in_name)) return false;
                Val &x = val(in_name);
                const int C = (int)per_image(x.shape);
                if (x.consumers != 1 || x.is_input || x.tensor < 0) return fail("Concat member " + in_name + " is shared");
                Step *prod = nullptr;
                for (auto &st : P.steps)
                    if (st.out.kind == 0 && st.out.id == x.tensor) prod = &st;
                if (!prod || prod->out.C * prod->out.H * prod->out.W != C)
                    return fail("Concat member " + in_name + " has no retargetable producer");
                for (auto &st : P.steps)
                    if ((st.in.kind == 0 && st.in.id == x.tensor) || (st.in2.kind == 0 && st.in2.id == x.tensor))
                        return fail("Concat member " + in_name + " is read internally");
                prod->out.id = id;
                prod->out.c_off = c0;
                c0 += C;
            }
            Val &y = val(nd.out[0]);
            y.tensor = id;
            y.step = -1;
        } else if (op == "Squeeze" || op == "Reshape" || op == "Flatten") {
            // internal alias: same storage, reinterpreted as (C = per-image size, 1, 1) or kept
            if (!ensure_tensor(nd.in[0])) return false;
            Val &x = val(nd.in[0]);
            Val &y = val(nd.out[0]);
            const int64_t hw_in = per_image(x.shape) / x.shape[1];
            if (!(hw_in == 1 || (y.shape.size() == 4 && y.shape[1] == x.shape[1])))
                return fail("reshape that mixes channels and positions is not supported internally");
            if (x.is_input) return fail("reshape of the graph input is not supported");
            if (y.out_idx >= 0) return fail("unexpected output placement on reshape");
            y.tensor = x.tensor;
            y.step = -1;
        } else {
            return fail("unsupported operator " + op);
        }
    }
    return true;
}

// Launch grouping: sibling steps that do not depend on each other and would run the same kernel
// instance (the FaceMesh flag and mesh branches after the 6^2 trunk, the four hand-landmark
// heads over the pooled features) are scheduled next to each other and launched as one grid
// (kernels/group.h).  A list schedule in plan order: a step with no ready partner but one later
// in the plan waits while ready steps without any prospective partner run first, so the two
// FaceMesh branches line up layer by layer.  Runs before allocate(), which gives the members of
// a group one shared time step (they run concurrently).
static bool groupable(const Step &a, const Step &b) {
    if (a.kind != b.kind || a.in.kind == 1 || b.in.kind == 1) return false;
    if (a.kind == S_DWPW)
        return a.kh == b.kh && a.stride == b.stride && a.pad_t == b.pad_t && a.pad_l == b.pad_l &&
               a.in.H == b.in.H && a.in.W == b.in.W && a.out.H == b.out.H && a.out.W == b.out.W &&
               a.K == b.K && a.Mpad == b.Mpad;
    if (a.kind == S_GEMM)
        return a.KK == b.KK && a.K == b.K && a.kh == b.kh && a.kw == b.kw && a.stride == b.stride &&
               a.in.C == b.in.C && a.in.H == b.in.H && a.in.W == b.in.W && a.out.H == b.out.H &&
               a.out.W == b.out.W;  // (M may differ: the launch checks the parts' kernel instance)
    return false;
}

// A global average pool over a depthwise conv's output, which nothing else reads, folds into
// the depthwise launch (dwgap_kernel): the hand landmark network's 672 x 7^2 tail.
void Compiler::fuse_dw_gap() {
    for (size_t gi = 0; gi < P.steps.size(); ++gi) {
        Step &g = P.steps[gi];
        if (g.kind != S_GAP || g.in.kind != 0 || g.in.c_off != 0) continue;
        int prod = -1, readers = 0;
        for (size_t i = 0; i < P.steps.size(); ++i) {
            const Step &s = P.steps[i];
            if (s.out.kind == 0 && s.out.id == g.in.id) prod = prod < 0 ? (int)i : -2;
            for (const TRef *r : {&s.in, &s.in2})
                if (r->kind == 0 && r->id == g.in.id) ++readers;
        }
        if (prod < 0 || readers != 1) continue;
        Step &d = P.steps[prod];
        if (d.kind != S_DW || (d.kh != 3 && d.kh != 5) || d.kh != d.kw || (int64_t)d.in.H * d.in.W > 512) continue;
        d.kind = S_DWGAP;
        d.dw_oh = d.out.H;
        d.dw_ow = d.out.W;
        d.name += "+" + g.name;
        d.out = g.out;
        d.bytes = 4.0 * ((double)d.in.C * d.in.H * d.in.W + d.in.C);
        P.steps.erase(P.steps.begin() + gi);
        --gi;
    }
}

// Expand 1x1 -> (depthwise -> 1x1) pairs whose expanded tensor nothing else reads: the executor
// may launch them as one inverted-residual kernel (ir.hip), the expanded tensor never stored.
void Compiler::mark_inverted_residuals() {
    std::vector<int> reads(P.storage_size.size(), 0);
    for (const Step &s : P.steps)
        for (const TRef *r : {&s.in, &s.in2})
            if (r->kind == 0 && r->id >= 0) reads[r->id]++;
    for (size_t i = 0; i + 1 < P.steps.size(); i++) {
        Step &e = P.steps[i];
        const Step &d = P.steps[i + 1];
        e.ir = e.kind == S_GEMM && e.group == 1 && d.group == 1 && e.KK == 1 && e.res_mode == 0 && e.out.kind == 0 &&
               e.out.c_off == 0 && e.in.kind == 0 && e.in.c_off == 0 && d.kind == S_DWPW && d.in.kind == 0 &&
               d.in.id == e.out.id && d.in.c_off == 0 && reads[e.out.id] == 1 && e.M == d.K;
    }
}

void Compiler::group_siblings() {
    const int n = (int)P.steps.size();
    if (n < 2) return;
    auto touches = [](const TRef &r, const TRef &w) {  // same storage (internal) or same graph output
        return r.kind == w.kind && r.kind != 1 && r.id >= 0 && r.id == w.id;
    };
    // dep[j][i]: j must run after i (reads what i writes, writes what i reads or writes)
    std::vector<std::vector<char>> dep(n, std::vector<char>(n, 0));
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < j; ++i) {
            const Step &a = P.steps[i], &b = P.steps[j];
            bool d = touches(b.in, a.out) || touches(b.out, a.out) || touches(b.out, a.in);
            if (b.res_mode || b.kind == S_ELT) d = d || touches(b.in2, a.out);
            if (a.res_mode || a.kind == S_ELT) d = d || touches(b.out, a.in2);
            dep[j][i] = d;
        }
    // transitive closure: related[i][j] = one of them (transitively) depends on the other
    std::vector<std::vector<char>> anc = dep;
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < j; ++i)
            if (anc[j][i])
                for (int k = 0; k < i; ++k) anc[j][k] |= anc[i][k];
    auto related = [&](int a, int b) { return a < b ? anc[b][a] : anc[a][b]; };
    std::vector<char> done(n, 0);
    auto ready = [&](int j) {
        if (done[j]) return false;
        for (int i = 0; i < j; ++i)
            if (dep[j][i] && !done[i]) return false;
        return true;
    };
    auto future_partner = [&](int s) {
        for (int t = 0; t < n; ++t)
            if (t != s && !done[t] && !ready(t) && !related(s, t) && groupable(P.steps[s], P.steps[t])) return true;
        return false;
    };
    std::vector<Step> out;
    out.reserve(n);
    for (int left = n; left > 0;) {
        std::vector<int> rd;
        for (int j = 0; j < n; ++j)
            if (ready(j)) rd.push_back(j);
        auto partners_of = [&](int s) {
            std::vector<int> g{s};
            for (int t : rd)
                if (t != s && (int)g.size() < ZR_GROUP_MAX && groupable(P.steps[s], P.steps[t])) g.push_back(t);
            return g;
        };
        std::vector<int> g = partners_of(rd[0]);
        if (g.size() == 1 && future_partner(rd[0]))
            for (int r : rd)
                if (r != rd[0] && !future_partner(r)) {
                    g = partners_of(r);
                    break;
                }
        for (size_t k = 0; k < g.size(); ++k) {
            Step st = P.steps[g[k]];
            st.group = k == 0 ? (int)g.size() : 0;
            out.push_back(std::move(st));
            done[g[k]] = 1;
        }
        left -= (int)g.size();
    }
    P.steps = std::move(out);
}

void Compiler::allocate() {
    // liveness over launch times (the members of a launch group share one)
    const size_t ns = P.storage_size.size();
    std::vector<int> first(ns, 1 << 30), last(ns, -1);
    int time = -1;
    std::vector<int> tof(P.steps.size());
    for (size_t i = 0; i < P.steps.size(); i++) {
        const Step &s = P.steps[i];
        if (s.group != 0) ++time;
        tof[i] = time;
        for (const TRef *r : {&s.in, &s.in2, &s.out})
            if (r->kind == 0 && r->id >= 0) {
                first[r->id] = std::min(first[r->id], time);
                last[r->id] = std::max(last[r->id], time);
            }
    }
    // a fused inverted residual (Step::ir) reads the expand's input and writes the projection's
    // output in ONE launch: the two must not share memory, so each is live across both steps
    for (size_t i = 0; i + 1 < P.steps.size(); i++) {
        if (!P.steps[i].ir) continue;
        const TRef &x = P.steps[i].in, &o = P.steps[i + 1].out;
        if (x.kind == 0 && x.id >= 0) last[x.id] = std::max(last[x.id], tof[i + 1]);
        if (o.kind == 0 && o.id >= 0) first[o.id] = std::min(first[o.id], tof[i]);
    }
    std::vector<int> order(ns);
    for (size_t i = 0; i < ns; i++) order[i] = (int)i;
    std::sort(order.begin(), order.end(),
              [&](int a, int b) { return P.storage_size[a] > P.storage_size[b]; });
    P.storage_off.assign(ns, 0);
    std::vector<int> placed;
    int64_t arena = 0;
    for (int id : order) {
        if (last[id] < 0) continue;
        // candidate offsets: 0 and the end of every time-overlapping placed slot
        std::vector<std::pair<int64_t, int64_t>> busy;
        for (int o : placed)
            if (!(last[o] < first[id] || last[id] < first[o]))
                busy.push_back({P.storage_off[o], P.storage_off[o] + P.storage_size[o]});
        std::sort(busy.begin(), busy.end());
        int64_t off = 0;
        for (auto &b : busy) {
            if (off + P.storage_size[id] <= b.first) break;
            off = std::max(off, b.second);
        }
        off = round_up(off, 64);  // 256-B aligned slots per image
        P.storage_off[id] = off;
        arena = std::max(arena, off + P.storage_size[id]);
        placed.push_back(id);
    }
    P.arena_per_image = round_up(arena, 64);
}

bool Compiler::run(const std::vector<uint32_t> &sel) {
    if (M.inputs.size() != 1) return fail("CNN plans take exactly one input");
    if (!infer_shapes()) return false;
    auto &is = val(M.inputs[0].name).shape;
    if (is.size() != 4) return fail("input must be NCHW");
    P.input_name = M.inputs[0].name;
    P.in_C = (int)is[1];
    P.in_H = (int)is[2];
    P.in_W = (int)is[3];
    std::vector<uint32_t> outs = sel;
    if (outs.empty())
        for (uint32_t i = 0; i < M.outputs.size(); i++) outs.push_back(i);
    for (size_t oi = 0; oi < outs.size(); oi++) {
        if (outs[oi] >= M.outputs.size()) return fail("output selection index out of range");
        const std::string &name = M.outputs[outs[oi]].name;
        PlanOutput po;
        po.name = name;
        po.shape = val(name).shape;
        po.per_image = per_image(po.shape);
        P.outputs.push_back(po);
    }
    for (size_t oi = 0; oi < outs.size(); oi++)
        if (!trace_output(P.outputs[oi].name, (int)oi, 0, false)) return false;
    // dead-node elimination from the selected outputs
    needed.assign(M.nodes.size(), false);
    std::vector<std::string> work;
    for (auto &o : P.outputs) work.push_back(o.name);
    std::set<std::string> seen;
    while (!work.empty()) {
        std::string n = work.back();
        work.pop_back();
        if (!seen.insert(n).second) continue;
        auto it = producer.find(n);
        if (it == producer.end()) continue;
        needed[it->second] = true;
        for (auto &i : M.nodes[it->second].in)
            if (!i.empty() && !init(i)) work.push_back(i);
    }
    // consumer counts restricted to needed nodes
    for (auto &kv : vals) kv.second.consumers = 0;
    for (size_t ni = 0; ni < M.nodes.size(); ni++)
        if (needed[ni])
            for (auto &i : M.nodes[ni].in)
                if (!i.empty()) vals[i].consumers++;
    if (!lower()) return false;
    for (size_t oi = 0; oi < P.outputs.size(); oi++) {
        bool written = false;
        for (auto &s : P.steps)
            if (s.out.kind == 2 && s.out.id == (int)oi) written = true;
        if (!written) return fail("output " + P.outputs[oi].name + " is never written");
    }
    for (auto &s : P.steps) {
        P.bytes_per_image += s.bytes;
        P.flops_per_image += s.flops;
    }
    P.bytes_per_image += 0;  // input read is counted by the stem
    int readers = 0, reader = -1;
    for (size_t i = 0; i < P.steps.size(); i++)
        for (const TRef *r : {&P.steps[i].in, &P.steps[i].in2})
            if (r->kind == 1) {
                readers++;
                reader = (int)i;
            }
    P.input_fusable = readers == 1 && P.steps[reader].kind == S_DIRECT && P.steps[reader].stem;
    if (form_on(FORM_DWGAP)) fuse_dw_gap();
    if (form_on(FORM_GROUPS)) group_siblings();
    if (form_on(FORM_IR)) mark_inverted_residuals();
    allocate();
    return true;
}

}  // namespace

bool compile_plan(const OnnxModel &m, const std::vector<uint32_t> &out_sel, Plan &plan,
                  std::string &err) {
    Compiler c(m, plan, err);
    return c.run(out_sel);
}

// ---------------------------------------------------------------- executor
namespace {

struct Resolved {
    const float *p;
    int64_t sN, sC, sP;
};

Resolved resolve(const TRef &r, const Plan &plan, const Binding &b) {
    Resolved o{};
    const int64_t P = (int64_t)r.H * r.W;
    if (r.kind == 0) {
        o.p = b.arena + plan.storage_off[r.id] * b.Ns + (int64_t)r.c_off * P * b.Ns;
        o.sN = P;
        o.sC = P * b.Ns;
        o.sP = 1;
    } else if (r.kind == 1) {
        o.p = b.input;
        o.sN = b.in_sN;
        o.sC = b.in_sC;
        o.sP = 1;
    } else {
        o.p = b.outputs[r.id] + r.off;
        o.sN = r.o_sN;
        o.sC = r.o_sC;
        o.sP = r.o_sP;
    }
    return o;
}

Act act_of(const ActDesc &a, const float *w) {
    Act o;
    o.kind = a.kind;
    o.lo = a.lo;
    o.hi = a.hi;
    o.slope = a.slope_off >= 0 ? w + a.slope_off : nullptr;
    return o;
}

Plane plane_of(const TRef &r, const Plan &plan, const Binding &b) {
    Resolved x = resolve(r, plan, b);
    Plane p;
    p.p = x.p;
    p.sN = x.sN;
    p.sC = x.sC;
    p.C = r.C;
    p.H = r.H;
    p.W = r.W;
    return p;
}

}  // namespace

void run_plan(const Plan &plan, const Binding &b, hipStream_t stream, LaunchHook *hook) {
    const float *W = b.weights;
    auto gemm_of = [&](const Step &s) {
        Resolved out = resolve(s.out, plan, b);
        Resolved x = resolve(s.in, plan, b);
        GemmParams g{};
        g.x = x.p;
        g.x_sN = x.sN;
        g.x_sC = x.sC;
        g.KK = s.KK;
        g.x_sK = 1;
        g.pk = s.kw;
        g.ph = s.kh;
        g.x_W = s.in.W;
        g.P = s.out.H * s.out.W;
        g.ncols = b.N * g.P;
        g.M = s.M;
        g.K = s.K;
        g.Mpad = s.Mpad;
        g.Kpad = s.Kpad;
        g.wt = W + s.w_off;
        g.bias = W + s.b_off;
        g.pre = act_of(s.pre, W);
        g.post = act_of(s.post, W);
        g.res_mode = s.res_mode;
        if (s.res_mode) {
            Resolved r = resolve(s.in2, plan, b);
            g.r = r.p;
            g.r_sN = r.sN;
            g.r_sC = r.sC;
            g.r_C = s.r_C;
            g.r_W = s.in2.W;
        }
        g.out_W = s.out.W;
        g.out = const_cast<float *>(out.p);
        g.o_sN = out.sN;
        g.o_sC = out.sC;
        g.o_sP = out.sP;
        g.nact = b.nact;
        return g;
    };
    auto dwpw_of = [&](const Step &s) {
        Resolved out = resolve(s.out, plan, b);
        DwPwParams d{};
        GemmParams &g = d.g;
        g.P = s.out.H * s.out.W;
        g.ncols = b.N * g.P;
        g.M = s.M;
        g.K = s.K;
        g.KK = 1;
        g.Mpad = s.Mpad;
        g.Kpad = s.Kpad;
        g.wt = W + s.w_off;
        g.bias = W + s.b_off;
        g.pre = act_of(s.pre, W);
        g.post = act_of(s.post, W);
        g.res_mode = s.res_mode;
        if (s.res_mode) {
            Resolved r = resolve(s.in2, plan, b);
            g.r = r.p;
            g.r_sN = r.sN;
            g.r_sC = r.sC;
            g.r_C = s.r_C;
            g.r_W = s.in2.W;
        }
        g.out_W = s.out.W;
        g.out = const_cast<float *>(out.p);
        g.o_sN = out.sN;
        g.o_sC = out.sC;
        g.o_sP = out.sP;
        d.in = plane_of(s.in, plan, b);
        d.OW = s.out.W;
        d.k = s.kh;
        d.stride = s.stride;
        d.pad_t = s.pad_t;
        d.pad_l = s.pad_l;
        d.dw_w = W + s.dw_w_off;
        d.dw_b = W + s.dw_b_off;
        d.dw_act = act_of(s.dw_act, W);
        g.nact = b.nact;
        return d;
    };
    for (size_t si = 0; si < plan.steps.size(); ++si) {
        const Step &s = plan.steps[si];
        if (s.ir && si + 1 < plan.steps.size()) {
            // expand + depthwise + projection in one launch (mark_inverted_residuals); nullptr: the
            // shapes do not fit the fused kernel, so both run on their own below
            const Step &s2 = plan.steps[si + 1];
            const GemmParams ge = gemm_of(s);
            const DwPwParams dp = dwpw_of(s2);
            if (hook) hook->before(stream);
            const char *kname = launch_ir(ge, dp, stream);
            if (!kname) kname = launch_irl(ge, dp, stream);
            if (!kname) kname = launch_bneck(ge, dp, stream);
            if (kname) {
                // fused-boundary bytes: the block input (+ residual) and the output
                const double bytes = s.bytes + s2.bytes - 8.0 * (double)s.out.C * s.out.H * s.out.W;
                if (hook) hook->after(stream, kname, bytes * b.N, (s.flops + s2.flops) * b.N);
                ++si;
                continue;
            }
            if (hook) hook->cancel();
        }
        if (s.group >= 2 && (s.kind == S_GEMM || s.kind == S_DWPW)) {
            // a launch group (group_siblings): one grid if the parts run the same grouped kernel
            // instance at this batch, else the members one by one below
            const int ng = std::min(s.group, ZR_GROUP_MAX);
            GemmParams gp[ZR_GROUP_MAX];
            DwPwParams dp[ZR_GROUP_MAX];
            double bytes = 0, flops = 0;
            for (int k = 0; k < ng; ++k) {
                const Step &m = plan.steps[si + k];
                if (s.kind == S_GEMM) gp[k] = gemm_of(m);
                else dp[k] = dwpw_of(m);
                bytes += m.bytes * b.N;
                flops += m.flops * b.N;
            }
            if (hook) hook->before(stream);
            const char *kname = s.kind == S_GEMM ? launch_gemm_group(gp, ng, stream) : launch_dwpw_group(dp, ng, stream);
            if (kname) {
                if (hook) hook->after(stream, kname, bytes, flops);
                si += ng - 1;
                continue;
            }
            if (hook) hook->cancel();
        }
        Resolved out = resolve(s.out, plan, b);
        const char *kname = nullptr;
        if (hook) hook->before(stream);
        switch (s.kind) {
        case S_GEMM: {
            kname = launch_gemm(gemm_of(s), stream);
            break;
        }
        case S_DWPW: {
            kname = launch_dwpw(dwpw_of(s), stream);
            break;
        }
        case S_DW: {
            DwParams d{};
            d.in = plane_of(s.in, plan, b);
            d.out = const_cast<float *>(out.p);
            d.o_sN = out.sN;
            d.o_sC = out.sC;
            d.OH = s.out.H;
            d.OW = s.out.W;
            d.N = b.N;
            d.k = s.kh;
            d.stride = s.stride;
            d.pad_t = s.pad_t;
            d.pad_l = s.pad_l;
            d.w = W + s.w_off;
            d.bias = W + s.b_off;
            d.act = act_of(s.pre, W);
            kname = launch_dw(d, stream);
            break;
        }
        case S_DIRECT: {
            if (s.stem) {
                StemParams sp{};
                const bool pre = s.in.kind == 1 && b.pre;
                if (pre) sp.pre = *b.pre;
                else sp.in = plane_of(s.in, plan, b);
                sp.out = const_cast<float *>(out.p);
                sp.o_sN = out.sN;
                sp.o_sC = out.sC;
                sp.IH = s.in.H;
                sp.IW = s.in.W;
                sp.OH = s.out.H;
                sp.OW = s.out.W;
                sp.N = b.N;
                sp.Cout = s.M;
                sp.k = s.kh;
                sp.stride = s.stride;
                sp.pad_t = s.pad_t;
                sp.pad_l = s.pad_l;
                sp.w = W + s.w_off;
                sp.bias = W + s.b_off;
                sp.act = act_of(s.pre, W);
                sp.nact = b.nact;
                kname = launch_stem(sp, pre, stream);
                if (hook) hook->after(stream, kname, (pre ? s.bytes_pre : s.bytes) * b.N, s.flops * b.N);
                continue;
            }
            DirectParams d{};
            d.in = plane_of(s.in, plan, b);
            d.out = const_cast<float *>(out.p);
            d.o_sN = out.sN;
            d.o_sC = out.sC;
            d.OH = s.out.H;
            d.OW = s.out.W;
            d.N = b.N;
            d.Cout = s.M;
            d.kh = s.kh;
            d.kw = s.kw;
            d.stride = s.stride;
            d.pad_t = s.pad_t;
            d.pad_l = s.pad_l;
            d.w = W + s.w_off;
            d.bias = W + s.b_off;
            d.act = act_of(s.pre, W);
            kname = launch_direct(d, stream);
            break;
        }
        case S_ELT: {
            EltParams e{};
            e.op = s.elt_op;
            e.a = plane_of(s.in, plan, b);
            if (s.elt_op == 1) e.b = plane_of(s.in2, plan, b);
            e.out = const_cast<float *>(out.p);
            e.o_sN = out.sN;
            e.o_sC = out.sC;
            e.N = b.N;
            e.C = s.out.C;
            e.H = s.out.H;
            e.W = s.out.W;
            e.act = act_of(s.pre, W);
            kname = launch_elt(e, stream);
            break;
        }
        case S_RESIZE: {
            ResizeParams r{};
            r.in = plane_of(s.in, plan, b);
            r.out = const_cast<float *>(out.p);
            r.o_sN = out.sN;
            r.o_sC = out.sC;
            r.N = b.N;
            r.OH = s.out.H;
            r.OW = s.out.W;
            r.scale_y = s.scale_y;
            r.scale_x = s.scale_x;
            r.nact = b.nact;
            kname = launch_resize(r, stream);
            break;
        }
        case S_DWGAP: {
            DwParams d{};
            d.in = plane_of(s.in, plan, b);
            d.out = const_cast<float *>(out.p);
            d.o_sN = out.sN;
            d.o_sC = out.sC;
            d.OH = s.dw_oh;
            d.OW = s.dw_ow;
            d.N = b.N;
            d.k = s.kh;
            d.stride = s.stride;
            d.pad_t = s.pad_t;
            d.pad_l = s.pad_l;
            d.w = W + s.w_off;
            d.bias = W + s.b_off;
            d.act = act_of(s.pre, W);
            kname = launch_dwgap(d, stream);
            break;
        }
        case S_GAP: {
            GapParams g{};
            g.in = plane_of(s.in, plan, b);
            g.out = const_cast<float *>(out.p);
            g.o_sN = out.sN;
            g.o_sC = out.sC;
            g.N = b.N;
            kname = launch_gap(g, stream);
            break;
        }
        }
        if (hook) hook->after(stream, kname, s.bytes * b.N, s.flops * b.N);
    }
}

}  // namespace zr
