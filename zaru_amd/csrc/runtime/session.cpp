// session.cpp -- the C ABI of include/zaru_hip.h: sessions, execution contexts and the
// view-sampling entry points.  This is the HIP `Session` variant that sits where
// `Session::Ort` / `Session::Tract` sit in the reference (crates/zaru/src/nn/mod.rs:377-381).
#include <hip/hip_runtime.h>

#include <cmath>
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/zaru_hip.h"
#include "onnx_model.h"
#include "plan.h"
#include "zr_track.h"

namespace {

thread_local std::string g_err;

int set_err(int code, const std::string &msg) noexcept {
    try {
        g_err = msg;
    } catch (...) {  // out of memory for the message: keep the code, drop the text
    }
    return code;
}

}  // namespace

// the thread-local error of the C ABI, for entry points defined in other translation units
// (runtime/jpeg.cpp)
namespace zr_internal {
int set_error(int code, const std::string &msg) { return set_err(code, msg); }
}  // namespace zr_internal

namespace {

// Every extern "C" entry point runs its body through this: no C++ exception crosses the C
// boundary (zaru_hip.h; a throw into the Rust caller's FFI frame is undefined behaviour).
// std::bad_alloc (host allocations: pools, staging vectors, strings) maps to ZR_ERR_DEVICE's
// "out of memory" class, anything else to ZR_ERR_INTERNAL.
template <class F>
int guarded(F &&body) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc &) {
        return set_err(ZR_ERR_DEVICE, "out of host memory");
    } catch (const std::exception &e) {
        return set_err(ZR_ERR_INTERNAL, std::string("internal error: ") + e.what());
    } catch (...) {
        return set_err(ZR_ERR_INTERNAL, "internal error: unknown exception");
    }
}

// A failed HIP call is returned to the caller once: the thread's last-error slot, which the
// failing call also set, is consumed here, so the next entry point (zr_comm_*'s pending-error
// check, the kernel-launch checks below) does not report the same, already returned failure again.
#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            (void)hipGetLastError();                                                     \
            return set_err(ZR_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
        }                                                                                \
    } while (0)

// One set of scratch buffers + a private stream.  Sessions keep a small pool so concurrent
// callers never share a workspace; reuse across streams is ordered by `done`.
struct Ctx {
    std::mutex mu;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    float *arena = nullptr;
    size_t arena_floats = 0;
    float *input = nullptr;  // network input staging
    size_t input_floats = 0;
    uint8_t *image = nullptr;  // host-image upload (zr_cnn_estimate_views)
    size_t image_bytes = 0;
    // the view and frame descriptors of a launch: one device block [views | frames] and its pinned
    // host staging, so an upload is one copy (one blit on the stream, not two)
    uint8_t *desc = nullptr, *h_desc = nullptr;
    size_t desc_bytes = 0;
    zr::ViewDesc *views = nullptr;    // (into desc)
    zr::FrameDesc *frames = nullptr;  // (into desc)
    std::vector<float *> outs;  // device outputs for the synchronous entry points
    std::vector<size_t> outs_floats;

    ~Ctx() {
        if (stream) (void)hipStreamSynchronize(stream);
        (void)hipFree(arena);
        (void)hipFree(input);
        (void)hipFree(image);
        (void)hipFree(desc);
        (void)hipHostFree(h_desc);
        for (auto p : outs) (void)hipFree(p);
        if (done) (void)hipEventDestroy(done);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

template <typename T>
int grow(T *&p, size_t &cap, size_t need) {
    if (cap >= need) return ZR_OK;
    if (p) {
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipFree(p));
        p = nullptr;
    }
    size_t n = need + need / 4 + 64;
    HIP_TRY(hipMalloc((void **)&p, n * sizeof(T)));
    cap = n;
    return ZR_OK;
}

// f32 quantities of a view exactly as the reference derives them (rect.rs:135-137,417-423;
// matrix.rs:571-579 with glibc cosf/sinf evaluated here on the host).
zr::ViewDesc make_view(const zr_view &v, uint32_t frame) {
#pragma clang fp contract(off)
    zr::ViewDesc d{};
    d.half_w = v.w * 0.5f;
    d.half_h = v.h * 0.5f;
    d.tl_x = v.cx - v.w * 0.5f;
    d.tl_y = v.cy - v.h * 0.5f;
    d.view_w = v.w;
    d.view_h = v.h;
    d.cos_r = cosf(v.rad);
    d.sin_r = sinf(v.rad);
    d.frame = frame;
    return d;
}

// Per-launch HIP-event timing (zr_profile_*): events are recorded on the launching stream
// around every kernel, so the measured durations come from the timed work itself.
struct Profiler final : zr::LaunchHook {
    struct Rec {
        const char *kernel;
        double bytes, flops;
        hipEvent_t a, b;
    };
    std::mutex mu;
    std::atomic<bool> on{false};  // read without the lock on the launch path
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    hipEvent_t pending = nullptr;

    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
    void before(hipStream_t s) override {
        pending = get();
        (void)hipEventRecord(pending, s);
    }
    void cancel() override {
        if (pending) pool.push_back(pending);
        pending = nullptr;
    }
    void after(hipStream_t s, const char *k, double bytes, double flops) override {
        hipEvent_t e = get();
        (void)hipEventRecord(e, s);
        recs.push_back({k, bytes, flops, pending, e});
    }
    ~Profiler() {
        for (auto &r : recs) {
            (void)hipEventDestroy(r.a);
            (void)hipEventDestroy(r.b);
        }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

}  // namespace

struct zr_session {
    Profiler prof;
    int device = 0;
    zr::Plan plan;
    float *weights = nullptr;
    std::vector<std::unique_ptr<Ctx>> pool;
    std::mutex pool_mu;
    size_t next = 0;

    Ctx *acquire() {
        std::lock_guard<std::mutex> g(pool_mu);
        // prefer a context whose previous work has completed on the GPU (its workspace and
        // pinned staging may then be rewritten without any wait); grow the pool up to 8
        for (size_t i = 0; i < pool.size(); i++) {
            Ctx *c = pool[(next + i) % pool.size()].get();
            if (c->mu.try_lock()) {
                if (hipEventQuery(c->done) == hipSuccess) {
                    next = (next + i + 1) % pool.size();
                    return c;
                }
                c->mu.unlock();
            }
        }
        if (pool.size() < 8) {
            auto c = std::make_unique<Ctx>();
            (void)hipSetDevice(device);
            // (the private stream is created on first use by a synchronous entry point: the async
            // ones run on the caller's stream, and an idle stream still takes a hardware queue)
            if (hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) return nullptr;
            c->mu.lock();
            pool.push_back(std::move(c));
            return pool.back().get();
        }
        Ctx *c = pool[next].get();
        next = (next + 1) % pool.size();
        c->mu.lock();
        (void)hipEventSynchronize(c->done);  // all 8 busy: reuse the oldest once it is done
        return c;
    }

    ~zr_session() {
        pool.clear();
        (void)hipFree(weights);
    }
};

namespace {

struct CtxLock {
    Ctx *c;
    explicit CtxLock(Ctx *x) : c(x) {}
    ~CtxLock() {
        if (c) c->mu.unlock();
    }
};

// enqueue the plan on `stream` with a context's workspace
int enqueue(zr_session *s, Ctx *c, int N, const float *input, int64_t in_sN, int64_t in_sC,
            float *const *outs, hipStream_t stream, const zr::PreprocParams *pre = nullptr,
            const int *d_nact = nullptr) {
    const int Ns = (N + 3) / 4 * 4;  // zr::Binding::Ns
    const size_t need = (size_t)s->plan.arena_per_image * (size_t)Ns;
    // kernels address every tensor with 32-bit element offsets (kernels/epilogue.h)
    size_t largest = std::max(need, (size_t)(input ? in_sN : 0) * (size_t)N);
    for (const auto &o : s->plan.outputs) largest = std::max(largest, (size_t)o.per_image * (size_t)N);
    if (largest >= ((size_t)1 << 31))
        return set_err(ZR_ERR_INVALID_ARGUMENT, "batch too large: a tensor would exceed 2^31 elements; split it");
    if (int rc = grow(c->arena, c->arena_floats, need ? need : 1)) return rc;
    HIP_TRY(hipStreamWaitEvent(stream, c->done, 0));
    zr::Binding b;
    b.N = N;
    b.Ns = Ns;
    b.input = input;
    b.in_sN = in_sN;
    b.in_sC = in_sC;
    b.outputs = outs;
    b.arena = c->arena;
    b.weights = s->weights;
    b.pre = pre;
    b.nact = d_nact;
    {
        const bool prof = s->prof.on.load();  // one read: the hook and its lock agree
        std::unique_lock<std::mutex> pl(s->prof.mu, std::defer_lock);
        if (prof) pl.lock();
        zr::run_plan(s->plan, b, stream, prof ? &s->prof : nullptr);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->done, stream));
    return ZR_OK;
}

// the context's private stream (synchronous entry points only)
int ctx_stream(Ctx *c) {
    if (!c->stream) HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    return ZR_OK;
}

int check_session(const zr_session *s) {
    if (!s) return set_err(ZR_ERR_INVALID_ARGUMENT, "null session");
    return ZR_OK;
}

int sync_outputs(zr_session *s, Ctx *c, size_t batch) {
    const auto &po = s->plan.outputs;
    c->outs.resize(po.size(), nullptr);
    c->outs_floats.resize(po.size(), 0);
    for (size_t i = 0; i < po.size(); i++)
        if (int rc = grow(c->outs[i], c->outs_floats[i], (size_t)po[i].per_image * batch)) return rc;
    return ZR_OK;
}

int upload_views(Ctx *c, const zr_frame *frames, size_t nf, const zr_view *views,
                 const uint32_t *view_frame, size_t nv, hipStream_t stream) {
    // [views | frames], the frames 256-byte aligned.  Pinned staging: the context was acquired idle
    // (or waited for), so it is free to rewrite, and the copy stays asynchronous (a pageable
    // source would block the host on the stream)
    const size_t foff = (nv * sizeof(zr::ViewDesc) + 255) & ~(size_t)255;
    const size_t bytes = foff + (nf ? nf : 1) * sizeof(zr::FrameDesc);
    if (c->desc_bytes < bytes) {
        (void)hipFree(c->desc);
        (void)hipHostFree(c->h_desc);
        c->desc = c->h_desc = nullptr;
        c->desc_bytes = 0;
        const size_t cap = bytes + bytes / 2 + 4096;
        HIP_TRY(hipMalloc((void **)&c->desc, cap));
        HIP_TRY(hipHostMalloc((void **)&c->h_desc, cap));
        c->desc_bytes = cap;
    }
    zr::ViewDesc *hv = reinterpret_cast<zr::ViewDesc *>(c->h_desc);
    zr::FrameDesc *hf = reinterpret_cast<zr::FrameDesc *>(c->h_desc + foff);
    c->views = reinterpret_cast<zr::ViewDesc *>(c->desc);
    c->frames = reinterpret_cast<zr::FrameDesc *>(c->desc + foff);
    for (size_t i = 0; i < nv; i++) {
        const uint32_t f = view_frame ? view_frame[i] : 0;
        if (f >= nf) return set_err(ZR_ERR_INVALID_ARGUMENT, "view_frame index out of range");
        hv[i] = make_view(views[i], f);
    }
    for (size_t i = 0; i < nf; i++) {
        if (!frames[i].rgba || frames[i].width == 0 || frames[i].height == 0)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "empty frame");
        hf[i].rgba = frames[i].rgba;
        hf[i].w = frames[i].width;
        hf[i].h = frames[i].height;
        hf[i].stride = frames[i].row_stride;
    }
    HIP_TRY(hipMemcpyAsync(c->desc, c->h_desc, foff + nf * sizeof(zr::FrameDesc), hipMemcpyHostToDevice, stream));
    return ZR_OK;
}

}  // namespace

extern "C" {

const char *zr_last_error(void) { return g_err.c_str(); }

int zr_session_create(const uint8_t *onnx, size_t len, const uint32_t *out_sel, size_t n_sel,
                      int device, zr_session **out) {
    return guarded([&]() -> int {
        if (!onnx || !out) return set_err(ZR_ERR_INVALID_ARGUMENT, "null model or out pointer");
        *out = nullptr;
        zr::OnnxModel m;
        std::string err;
        if (!zr::parse_onnx(onnx, len, m, err)) return set_err(ZR_ERR_MODEL, "ONNX parse error: " + err);
        auto s = std::make_unique<zr_session>();
        s->device = device;
        std::vector<uint32_t> sel(out_sel, out_sel + n_sel);
        if (!zr::compile_plan(m, sel, s->plan, err)) return set_err(ZR_ERR_MODEL, err);
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
            (void)hipGetLastError();  // returned here, as HIP_TRY does
            return set_err(ZR_ERR_DEVICE, "no HIP device " + std::to_string(device));
        }
        HIP_TRY(hipSetDevice(device));
        const size_t wb = s->plan.weights.size() * sizeof(float);
        HIP_TRY(hipMalloc((void **)&s->weights, wb ? wb : 4));
        HIP_TRY(hipMemcpy(s->weights, s->plan.weights.data(), wb, hipMemcpyHostToDevice));
        *out = s.release();
        return ZR_OK;
    });
}

void zr_session_destroy(zr_session *s) { delete s; }  // destructors are noexcept

int zr_session_num_io(const zr_session *s, int is_output, size_t *n) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        if (!n) return set_err(ZR_ERR_INVALID_ARGUMENT, "null n");
        *n = is_output ? s->plan.outputs.size() : 1;
        return ZR_OK;
    });
}

int zr_session_io(const zr_session *s, int is_output, size_t idx, const char **name,
                  int64_t *shape, size_t *rank) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        if (!is_output) {
            if (idx != 0) return set_err(ZR_ERR_INVALID_ARGUMENT, "input index out of range");
            if (name) *name = s->plan.input_name.c_str();
            if (shape) {
                shape[0] = 1;
                shape[1] = s->plan.in_C;
                shape[2] = s->plan.in_H;
                shape[3] = s->plan.in_W;
            }
            if (rank) *rank = 4;
            return ZR_OK;
        }
        if (idx >= s->plan.outputs.size()) return set_err(ZR_ERR_INVALID_ARGUMENT, "output index out of range");
        const auto &o = s->plan.outputs[idx];
        if (name) *name = o.name.c_str();
        if (shape)
            for (size_t i = 0; i < o.shape.size() && i < 8; i++) shape[i] = i == 0 ? 1 : o.shape[i];
        if (rank) *rank = o.shape.size();
        return ZR_OK;
    });
}

int zr_plan_describe(const uint8_t *onnx, size_t len, const uint32_t *out_sel, size_t n_sel,
                     char *buf, size_t cap, size_t *needed) {
    return guarded([&]() -> int {
        if (!onnx) return set_err(ZR_ERR_INVALID_ARGUMENT, "null model");
        zr::OnnxModel m;
        std::string err;
        if (!zr::parse_onnx(onnx, len, m, err)) return set_err(ZR_ERR_MODEL, "ONNX parse error: " + err);
        zr::Plan plan;
        std::vector<uint32_t> sel(out_sel, out_sel + n_sel);
        if (!zr::compile_plan(m, sel, plan, err)) return set_err(ZR_ERR_MODEL, err);
        static const char *kinds[] = {"gemm", "dw", "direct", "elt", "resize", "gap", "dwpw", "dwgap"};
        static const char *acts[] = {"none", "relu", "clip", "prelu", "sigmoid"};
        std::string t;
        char line[512];
        auto ref = [](const zr::TRef &r) {
            char b[96];
            snprintf(b, sizeof b, "%s%d[%dx%dx%d]", r.kind == 0 ? "t" : r.kind == 1 ? "in" : "out",
                     r.id, r.C, r.H, r.W);
            return std::string(b);
        };
        snprintf(line, sizeof line, "input %s %dx%dx%d arena_per_image=%lld weights=%zu bytes/img=%.0f flops/img=%.0f fusable=%d\n",
                 plan.input_name.c_str(), plan.in_C, plan.in_H, plan.in_W,
                 (long long)plan.arena_per_image, plan.weights.size(), plan.bytes_per_image,
                 plan.flops_per_image, plan.input_fusable ? 1 : 0);
        t += line;
        for (auto &o : plan.outputs) {
            snprintf(line, sizeof line, "output %s per_image=%lld\n", o.name.c_str(), (long long)o.per_image);
            t += line;
        }
        for (auto &st : plan.steps) {
            snprintf(line, sizeof line,
                     "%s%s in=%s out=%s k=%dx%d s=%d M=%d K=%d KK=%d pre=%s post=%s res=%d rC=%d elt=%d off=%lld oN=%lld oC=%lld oP=%lld in2=%s grp=%d ir=%d\n",
                     kinds[st.kind], st.stem ? " stem" : "", ref(st.in).c_str(), ref(st.out).c_str(), st.kh, st.kw, st.stride,
                     st.M, st.K, st.KK, acts[st.pre.kind], acts[st.post.kind], st.res_mode, st.r_C,
                     st.elt_op, (long long)st.out.off, (long long)st.out.o_sN, (long long)st.out.o_sC,
                     (long long)st.out.o_sP, (st.res_mode || st.kind == zr::S_ELT) ? ref(st.in2).c_str() : "-", st.group,
                     st.ir);
            t += line;
        }
        if (needed) *needed = t.size() + 1;
        if (buf && cap) {
            size_t n = std::min(cap - 1, t.size());
            memcpy(buf, t.data(), n);
            buf[n] = 0;
        }
        return ZR_OK;
    });
}

int zr_profile_enable(zr_session *s, int enable) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        std::lock_guard<std::mutex> g(s->prof.mu);
        s->prof.on = enable != 0;
        return ZR_OK;
    });
}

int zr_profile_read(zr_session *s, char *buf, size_t cap, size_t *needed) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        std::lock_guard<std::mutex> g(s->prof.mu);
        struct Agg {
            size_t n = 0;
            double ms = 0, bytes = 0, flops = 0;
        };
        std::vector<std::pair<std::string, Agg>> aggs;
        for (auto &r : s->prof.recs) {
            HIP_TRY(hipEventSynchronize(r.b));
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
            auto it = std::find_if(aggs.begin(), aggs.end(), [&](auto &p) { return p.first == r.kernel; });
            if (it == aggs.end()) {
                aggs.push_back({r.kernel, Agg{}});
                it = aggs.end() - 1;
            }
            it->second.n++;
            it->second.ms += ms;
            it->second.bytes += r.bytes;
            it->second.flops += r.flops;
            s->prof.pool.push_back(r.a);
            s->prof.pool.push_back(r.b);
        }
        s->prof.recs.clear();
        std::string t;
        char line[256];
        for (auto &a : aggs) {
            snprintf(line, sizeof line, "%s %zu %.6f %.0f %.0f\n", a.first.c_str(), a.second.n, a.second.ms,
                     a.second.bytes, a.second.flops);
            t += line;
        }
        if (needed) *needed = t.size() + 1;
        if (buf && cap) {
            size_t n = std::min(cap - 1, t.size());
            memcpy(buf, t.data(), n);
            buf[n] = 0;
        }
        return ZR_OK;
    });
}

int zr_session_stats(const zr_session *s, double *bytes, double *flops, size_t *launches) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        if (bytes) *bytes = s->plan.bytes_per_image;
        if (flops) *flops = s->plan.flops_per_image;
        if (launches) *launches = s->plan.steps.size();
        return ZR_OK;
    });
}

int zr_session_run_async(zr_session *s, size_t batch, const float *d_input, float *const *d_outputs,
                         size_t n_out, void *hip_stream) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        if (!d_input || !d_outputs || batch == 0) return set_err(ZR_ERR_INVALID_ARGUMENT, "null tensor or empty batch");
        if (n_out != s->plan.outputs.size()) return set_err(ZR_ERR_SHAPE, "output count mismatch");
        Ctx *c = s->acquire();
        if (!c) return set_err(ZR_ERR_DEVICE, "cannot create execution context");
        CtxLock lk(c);
        HIP_TRY(hipSetDevice(s->device));
        const int64_t hw = (int64_t)s->plan.in_H * s->plan.in_W;
        return enqueue(s, c, (int)batch, d_input, hw * s->plan.in_C, hw, d_outputs,
                       (hipStream_t)hip_stream);
    });
}

int zr_session_run(zr_session *s, size_t batch, const float *const *inputs, size_t n_in,
                   float *const *outputs, size_t n_out) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        if (!inputs || !outputs || batch == 0) return set_err(ZR_ERR_INVALID_ARGUMENT, "null tensor or empty batch");
        if (n_in != 1) return set_err(ZR_ERR_SHAPE, "CNN sessions take exactly 1 input");
        if (n_out != s->plan.outputs.size()) return set_err(ZR_ERR_SHAPE, "output count mismatch");
        Ctx *c = s->acquire();
        if (!c) return set_err(ZR_ERR_DEVICE, "cannot create execution context");
        CtxLock lk(c);
        HIP_TRY(hipSetDevice(s->device));
        const int64_t hw = (int64_t)s->plan.in_H * s->plan.in_W;
        const size_t in_floats = (size_t)hw * s->plan.in_C * batch;
        if (int rc = ctx_stream(c)) return rc;
        if (int rc = grow(c->input, c->input_floats, in_floats)) return rc;
        if (int rc = sync_outputs(s, c, batch)) return rc;
        HIP_TRY(hipMemcpyAsync(c->input, inputs[0], in_floats * 4, hipMemcpyHostToDevice, c->stream));
        if (int rc = enqueue(s, c, (int)batch, c->input, hw * s->plan.in_C, hw, c->outs.data(), c->stream))
            return rc;
        for (size_t i = 0; i < n_out; i++)
            HIP_TRY(hipMemcpyAsync(outputs[i], c->outs[i], s->plan.outputs[i].per_image * batch * 4,
                                   hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return ZR_OK;
    });
}

static int views_common(zr_session *s, Ctx *c, const zr_frame *frames, size_t nf, const zr_view *views,
                        const uint32_t *view_frame, size_t nv, float lo, float hi, float *const *outs,
                        hipStream_t stream, const zr::ViewDesc *d_views = nullptr, const int *d_nact = nullptr) {
    const int64_t hw = (int64_t)s->plan.in_H * s->plan.in_W;
    if (s->plan.in_C != 3) return set_err(ZR_ERR_SHAPE, "view sampling needs a 3-channel input");
    if (!(hi > lo)) return set_err(ZR_ERR_INVALID_ARGUMENT, "ColorMapper range must satisfy end > start");
    HIP_TRY(hipStreamWaitEvent(stream, c->done, 0));
    // a device view table (the tracker's) needs only the frame table uploaded
    if (int rc = upload_views(c, frames, nf, views, view_frame, d_views ? 0 : nv, stream)) return rc;
    zr::PreprocParams p{};
    p.frames = c->frames;
    p.nframes = (int)nf;
    p.views = d_views ? d_views : c->views;
    p.nviews = (int)nv;
    p.OW = s->plan.in_W;
    p.OH = s->plan.in_H;
    p.lo = lo;
    p.adjust = (hi - lo) / 255.0f;  // nn/mod.rs:162
    if (s->plan.input_fusable)  // the stem samples the frames itself: no input tensor at all
        return enqueue(s, c, (int)nv, nullptr, 0, 0, outs, stream, &p, d_nact);
    if (int rc = grow(c->input, c->input_floats, (size_t)hw * 3 * nv)) return rc;
    p.out = c->input;
    p.o_sN = hw;                    // CNHW straight into the plan's input layout
    p.o_sC = hw * (int64_t)nv;
    {
        const bool prof = s->prof.on.load();
        std::unique_lock<std::mutex> pl(s->prof.mu, std::defer_lock);
        if (prof) pl.lock();
        if (prof) s->prof.before(stream);
        const char *k = zr::launch_preproc(p, stream);
        // algorithmic bytes: RGBA gather 4 B + 3 f32 writes per output position
        if (prof) s->prof.after(stream, k, 16.0 * (double)hw * nv, 0.0);
    }
    HIP_TRY(hipGetLastError());
    return enqueue(s, c, (int)nv, c->input, hw, hw * (int64_t)nv, outs, stream, nullptr, d_nact);
}

int zr_cnn_estimate_views_async(zr_session *s, const zr_frame *frames, size_t n_frames,
                                const zr_view *views, const uint32_t *view_frame, size_t n_views,
                                float lo, float hi, float *const *d_outputs, void *hip_stream) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        if (!frames || !views || !d_outputs || n_views == 0)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument or no views");
        Ctx *c = s->acquire();
        if (!c) return set_err(ZR_ERR_DEVICE, "cannot create execution context");
        CtxLock lk(c);
        HIP_TRY(hipSetDevice(s->device));
        return views_common(s, c, frames, n_frames, views, view_frame, n_views, lo, hi, d_outputs,
                            (hipStream_t)hip_stream);
    });
}

// ---- device-resident tracker state (kernels/track.hip)
static_assert(sizeof(zr_track_state) == sizeof(zr::TrackState), "zr_track_state layout");
static_assert(sizeof(zr_view_desc) == sizeof(zr::ViewDesc), "zr_view_desc layout");

static int track_params(zr::TrackParams &p, zr_track_state *d_state, size_t n, const zr_track_cfg *cfg,
                        zr_view_desc *d_views) {
    if (!d_state || !cfg || !d_views || n == 0) return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument or n == 0");
    if (cfg->kind < 0 || cfg->kind > 3 || cfg->num_landmarks <= 0 || cfg->in_w <= 0 || cfg->in_h <= 0 ||
        cfg->aspect_w <= 0 || cfg->aspect_h <= 0 || !(cfg->padding >= 0.f) || n > (1u << 24))
        return set_err(ZR_ERR_INVALID_ARGUMENT, "bad tracker configuration");
    if ((cfg->kind == 0 && cfg->num_landmarks <= 263) || (cfg->kind == 1 && cfg->num_landmarks <= 9))
        return set_err(ZR_ERR_INVALID_ARGUMENT, "angle landmarks out of range");
    p.state = reinterpret_cast<zr::TrackState *>(d_state);
    p.views = reinterpret_cast<zr::ViewDesc *>(d_views);
    p.n = (int)n;
    p.L = cfg->num_landmarks;
    p.kind = cfg->kind;
    p.in_w = cfg->in_w;
    p.in_h = cfg->in_h;
    p.asp_w = cfg->aspect_w;
    p.asp_h = cfg->aspect_h;
    p.loss_thresh = cfg->loss_thresh;
    p.padding = cfg->padding;
    if (cfg->rois_per_frame < 0) return set_err(ZR_ERR_INVALID_ARGUMENT, "rois_per_frame must be >= 0");
    p.rpf = cfg->rois_per_frame > 0 ? cfg->rois_per_frame : 1;
    return ZR_OK;
}

int zr_track_seed_async(zr_track_state *d_state, size_t n, const zr_track_cfg *cfg, zr_view_desc *d_views,
                        void *hip_stream) {
    return guarded([&]() -> int {
        zr::TrackParams p{};
        if (int rc = track_params(p, d_state, n, cfg, d_views)) return rc;
        p.seed = 1;
        zr::launch_track(p, (hipStream_t)hip_stream);
        HIP_TRY(hipGetLastError());
        return ZR_OK;
    });
}

int zr_track_update_async(zr_track_state *d_state, size_t n, const zr_track_cfg *cfg, const float *d_landmarks,
                          size_t lm_stride, const float *d_flag, size_t flag_stride, float *d_lm_out,
                          zr_view_desc *d_views, void *hip_stream) {
    return guarded([&]() -> int {
        zr::TrackParams p{};
        if (int rc = track_params(p, d_state, n, cfg, d_views)) return rc;
        if (!d_landmarks || (cfg->kind <= 2 && (!d_flag || flag_stride == 0)))
            return set_err(ZR_ERR_INVALID_ARGUMENT, "missing landmark / flag outputs");
        if (cfg->kind == 2 && (cfg->num_landmarks <= 5 || flag_stride < 15))
            return set_err(ZR_ERR_INVALID_ARGUMENT, "eye network: output 1 holds the 5 iris points");
        // what each kind's extract reads of output 0 (mediapipe.rs:59-71, hand/landmark.rs:298-322,
        // eye.rs:47-64, multipie68.rs:71,108: outputs[0][..NUM_LANDMARKS * 2])
        const size_t L = (size_t)cfg->num_landmarks;
        const size_t need = cfg->kind == 3 ? 2 * L : cfg->kind == 2 ? 3 * (L - 5) : 3 * L;
        if (lm_stride < need || lm_stride > (size_t)INT32_MAX)
            return set_err(ZR_ERR_SHAPE, "landmark output holds fewer floats per image than the extract reads");
        p.lm = d_landmarks;
        p.lm_stride = (int)lm_stride;
        p.flag = d_flag;
        p.flag_stride = (int)flag_stride;
        p.lm_out = d_lm_out;
        zr::launch_track(p, (hipStream_t)hip_stream);
        HIP_TRY(hipGetLastError());
        return ZR_OK;
    });
}

static int detect_post_impl(const float *d_logits, const float *d_boxes, const float *d_anchors,
                            const float *d_letterbox, size_t n, const zr_detpost_cfg *cfg, int32_t *d_count,
                            float *d_dets, size_t dcap, float *d_records, size_t rmax, uint32_t first_id,
                            uint32_t id_stride, int32_t *d_ties, const int32_t *d_map, const int32_t *d_nact,
                            void *hip_stream) {
    return guarded([&]() -> int {
        if (!d_logits || !d_boxes || !d_anchors || !d_letterbox || !cfg || !d_count || (!d_dets && dcap))
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        if (n == 0) return ZR_OK;
        if (cfg->anchors <= 0 || cfg->keypoints < 3 || cfg->keypoints > 7 ||
            cfg->params < 4 + 2 * cfg->keypoints || cfg->in_w <= 0 || cfg->in_h <= 0 || n > (1u << 24) ||
            dcap > 65536 || rmax > 64 || (d_records && rmax == 0) || cfg->mode < 0 || cfg->mode > 1)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "bad detection post-processing configuration");
        zr::DetPostParams p{};
        p.logits = d_logits;
        p.boxes = d_boxes;
        p.anchors = d_anchors;
        p.letterbox = d_letterbox;
        p.N = (int)n;
        p.A = cfg->anchors;
        p.D = cfg->params;
        p.nkp = cfg->keypoints;
        p.face = cfg->face ? 1 : 0;
        p.in_w = cfg->in_w;
        p.in_h = cfg->in_h;
        p.thresh = cfg->thresh;
        p.iou = cfg->iou;
        p.mode = cfg->mode;
        p.count = d_count;
        p.dets = d_dets;
        p.dcap = (int)dcap;
        p.rec = d_records;
        p.rmax = (int)rmax;
        p.first_id = first_id;
        p.id_stride = id_stride;
        p.ties = d_ties;
        p.map = d_map;
        p.nact = d_nact;
        if (zr::det_post_lds(p.A) > 128 * 1024) return set_err(ZR_ERR_INVALID_ARGUMENT, "too many anchors");
        zr::launch_det_post(p, (hipStream_t)hip_stream);
        HIP_TRY(hipGetLastError());
        return ZR_OK;
    });
}

int zr_detect_post_async(const float *d_logits, const float *d_boxes, const float *d_anchors,
                         const float *d_letterbox, size_t n, const zr_detpost_cfg *cfg, int32_t *d_count,
                         float *d_dets, size_t dcap, float *d_records, size_t rmax, uint32_t first_id,
                         uint32_t id_stride, int32_t *d_ties, void *hip_stream) {
    return detect_post_impl(d_logits, d_boxes, d_anchors, d_letterbox, n, cfg, d_count, d_dets, dcap, d_records, rmax,
                            first_id, id_stride, d_ties, nullptr, nullptr, hip_stream);
}

int zr_detect_post_mapped_async(const float *d_logits, const float *d_boxes, const float *d_anchors,
                                const float *d_letterbox, size_t n, const int32_t *d_map, const int32_t *d_nframes,
                                const zr_detpost_cfg *cfg, int32_t *d_count, float *d_dets, size_t dcap,
                                int32_t *d_ties, void *hip_stream) {
    if (!d_map || !d_nframes) return set_err(ZR_ERR_INVALID_ARGUMENT, "null frame map or count");
    return detect_post_impl(d_logits, d_boxes, d_anchors, d_letterbox, n, cfg, d_count, d_dets, dcap, nullptr, 0, 0, 1,
                            d_ties, d_map, d_nframes, hip_stream);
}

int zr_track_seed_detections_async(const int32_t *d_count, const float *d_dets, size_t dcap, const float *d_forced,
                                   const int32_t *d_nforced, const uint32_t *d_frame_size, size_t n,
                                   const zr_track_cfg *cfg, float roi_grow, int roi_use_angle,
                                   zr_track_state *d_state, zr_track_state *d_seed_copy, zr_view_desc *d_views,
                                   void *hip_stream) {
    return guarded([&]() -> int {
        if (!d_count || !d_dets || !d_frame_size || !cfg || !d_state || !d_views || dcap == 0 ||
            (!d_forced != !d_nforced))
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        if (n == 0) return ZR_OK;
        const int R = cfg->rois_per_frame > 0 ? cfg->rois_per_frame : 1;
        if (cfg->aspect_w <= 0 || cfg->aspect_h <= 0 || R > 64 || (uint64_t)n * R > (1u << 24) || !(roi_grow >= 0.f))
            return set_err(ZR_ERR_INVALID_ARGUMENT, "bad tracker seeding configuration");
        zr::SeedParams p{};
        p.count = d_count;
        p.dets = d_dets;
        p.dcap = (int)dcap;
        p.forced = d_forced;
        p.nforced = d_nforced;
        p.fsize = d_frame_size;
        p.N = (int)n;
        p.R = R;
        p.roi_grow = roi_grow;
        p.roi_use_angle = roi_use_angle ? 1 : 0;
        p.asp_w = cfg->aspect_w;
        p.asp_h = cfg->aspect_h;
        p.state = reinterpret_cast<zr::TrackState *>(d_state);
        p.seed_copy = reinterpret_cast<zr::TrackState *>(d_seed_copy);
        p.views = reinterpret_cast<zr::ViewDesc *>(d_views);
        zr::launch_seed(p, (hipStream_t)hip_stream);
        HIP_TRY(hipGetLastError());
        return ZR_OK;
    });
}

int zr_hand_manage_async(zr_track_state *d_state, uint64_t *d_ids, float *d_hroi, int32_t *d_src, int32_t *d_nhands,
                         uint64_t *d_next_id, double *d_next_det, int32_t *d_det_pending, const int32_t *d_count,
                         const float *d_dets, size_t dcap, const uint32_t *d_frame_size, size_t n,
                         const zr_hand_cfg *cfg, double now_ms, int init_clock, zr_view_desc *d_views,
                         int32_t *d_dropped, void *hip_stream) {
    return guarded([&]() -> int {
        if (!d_state || !d_ids || !d_hroi || !d_src || !d_nhands || !d_next_id || !d_next_det || !d_det_pending ||
            !d_count || !d_dets || !d_frame_size || !cfg || !d_views)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        if (n == 0) return ZR_OK;
        if (cfg->slots <= 0 || cfg->slots > 64 || dcap == 0 || dcap > 65536 || (uint64_t)n * cfg->slots > (1u << 24) ||
            cfg->aspect_w <= 0 || cfg->aspect_h <= 0 || !(cfg->interval_ms >= 0.0) || !(cfg->palm_grow >= 0.f))
            return set_err(ZR_ERR_INVALID_ARGUMENT, "bad hand tracker configuration");
        zr::HandManageParams p{};
        p.state = reinterpret_cast<zr::TrackState *>(d_state);
        p.ids = d_ids;
        p.hroi = d_hroi;
        p.src = d_src;
        p.nhands = d_nhands;
        p.next_id = d_next_id;
        p.dropped = d_dropped;
        p.next_det = d_next_det;
        p.det_pending = d_det_pending;
        p.count = d_count;
        p.dets = d_dets;
        p.fsize = d_frame_size;
        p.views = reinterpret_cast<zr::ViewDesc *>(d_views);
        p.S = (int)n;
        p.H = cfg->slots;
        p.dcap = (int)dcap;
        p.iou = cfg->iou_thresh;
        p.grow = cfg->palm_grow;
        p.now = now_ms;
        p.interval = cfg->interval_ms;
        p.init_clock = init_clock ? 1 : 0;
        p.asp_w = cfg->aspect_w;
        p.asp_h = cfg->aspect_h;
        zr::launch_hand_manage(p, (hipStream_t)hip_stream);
        HIP_TRY(hipGetLastError());
        return ZR_OK;
    });
}

int zr_view_describe(const zr_view *views, size_t n, uint32_t frame, zr_view_desc *out) {
    return guarded([&]() -> int {
        if (!views || !out) return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        for (size_t i = 0; i < n; i++) {
            const zr::ViewDesc d = make_view(views[i], frame);
            std::memcpy(&out[i], &d, sizeof(d));
        }
        return ZR_OK;
    });
}

int zr_debug_glibc_math(int fn, const float *d_a, const float *d_b, float *d_out, size_t n, void *hip_stream) {
    return guarded([&]() -> int {
        if (fn < 0 || fn > 4 || !d_a || !d_out || (fn == 4 && !d_b) || n > (size_t)INT64_MAX / 2)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "bad glibc-math request");
        if (n == 0) return ZR_OK;
        zr::launch_glibc_math(fn, d_a, d_b, d_out, (int64_t)n, (hipStream_t)hip_stream);
        HIP_TRY(hipGetLastError());
        return ZR_OK;
    });
}

int zr_cnn_estimate_device_views_async(zr_session *s, const zr_frame *frames, size_t n_frames,
                                       const zr_view_desc *d_views, size_t n_views, float lo, float hi,
                                       float *const *d_outputs, void *hip_stream) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        if (!frames || !d_views || !d_outputs || n_views == 0 || n_frames == 0)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument or no views");
        Ctx *c = s->acquire();
        if (!c) return set_err(ZR_ERR_DEVICE, "cannot create execution context");
        CtxLock lk(c);
        HIP_TRY(hipSetDevice(s->device));
        return views_common(s, c, frames, n_frames, nullptr, nullptr, n_views, lo, hi, d_outputs,
                            (hipStream_t)hip_stream, reinterpret_cast<const zr::ViewDesc *>(d_views));
    });
}

int zr_cnn_estimate_device_views_count_async(zr_session *s, const zr_frame *frames, size_t n_frames,
                                             const zr_view_desc *d_views, size_t n_views, const int32_t *d_count,
                                             float lo, float hi, float *const *d_outputs, void *hip_stream) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        if (!frames || !d_views || !d_outputs || !d_count || n_views == 0 || n_frames == 0)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument or no views");
        Ctx *c = s->acquire();
        if (!c) return set_err(ZR_ERR_DEVICE, "cannot create execution context");
        CtxLock lk(c);
        HIP_TRY(hipSetDevice(s->device));
        return views_common(s, c, frames, n_frames, nullptr, nullptr, n_views, lo, hi, d_outputs,
                            (hipStream_t)hip_stream, reinterpret_cast<const zr::ViewDesc *>(d_views), d_count);
    });
}

int zr_due_compact_async(const int32_t *d_det_pending, size_t n, const zr_view_desc *view_template, int32_t *d_due,
                         int32_t *d_ndue, zr_view_desc *d_due_views, uint64_t *d_total, void *hip_stream) {
    return guarded([&]() -> int {
        if (!d_det_pending || !view_template || !d_due || !d_ndue || !d_due_views)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        if (n == 0 || n > (1u << 24)) return set_err(ZR_ERR_INVALID_ARGUMENT, "bad stream count");
        zr::launch_due_compact(d_det_pending, nullptr, (int)n, *reinterpret_cast<const zr::ViewDesc *>(view_template),
                               d_due, d_ndue, reinterpret_cast<zr::ViewDesc *>(d_due_views), d_total,
                               (hipStream_t)hip_stream);
        HIP_TRY(hipGetLastError());
        return ZR_OK;
    });
}

int zr_track_lost_compact_async(const zr_track_state *d_state, size_t n, const zr_view_desc *view_template,
                                int32_t *d_due, int32_t *d_ndue, zr_view_desc *d_due_views, uint64_t *d_total,
                                void *hip_stream) {
    return guarded([&]() -> int {
        if (!d_state || !view_template || !d_due || !d_ndue || !d_due_views)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        if (n == 0 || n > (1u << 24)) return set_err(ZR_ERR_INVALID_ARGUMENT, "bad stream count");
        zr::launch_due_compact(nullptr, reinterpret_cast<const zr::TrackState *>(d_state), (int)n,
                               *reinterpret_cast<const zr::ViewDesc *>(view_template), d_due, d_ndue,
                               reinterpret_cast<zr::ViewDesc *>(d_due_views), d_total, (hipStream_t)hip_stream);
        HIP_TRY(hipGetLastError());
        return ZR_OK;
    });
}

int zr_track_reseed_best_async(const int32_t *d_count, const float *d_dets, size_t dcap, const uint32_t *d_frame_size,
                               size_t n, const zr_track_cfg *cfg, zr_track_state *d_state, zr_view_desc *d_views,
                               uint64_t *d_reseeded, void *hip_stream) {
    return guarded([&]() -> int {
        if (!d_count || !d_dets || !d_frame_size || !cfg || !d_state || !d_views || dcap == 0)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument");
        if (n == 0) return ZR_OK;
        if (cfg->aspect_w <= 0 || cfg->aspect_h <= 0 || n > (1u << 24) || dcap > 65536)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "bad re-seeding configuration");
        zr::ReseedParams p{};
        p.count = d_count;
        p.dets = d_dets;
        p.dcap = (int)dcap;
        p.fsize = d_frame_size;
        p.N = (int)n;
        p.asp_w = cfg->aspect_w;
        p.asp_h = cfg->aspect_h;
        p.state = reinterpret_cast<zr::TrackState *>(d_state);
        p.views = reinterpret_cast<zr::ViewDesc *>(d_views);
        p.reseeded = d_reseeded;
        zr::launch_reseed(p, (hipStream_t)hip_stream);
        HIP_TRY(hipGetLastError());
        return ZR_OK;
    });
}

int zr_cnn_estimate_views(zr_session *s, const uint8_t *rgba, uint32_t w, uint32_t h,
                          size_t row_stride, const zr_view *views, size_t n_views, float lo,
                          float hi, float *const *outputs) {
    return guarded([&]() -> int {
        if (int rc = check_session(s)) return rc;
        if (!rgba || !views || !outputs || n_views == 0)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument or no views");
        if (row_stride < (size_t)w * 4) return set_err(ZR_ERR_INVALID_ARGUMENT, "row_stride < 4*width");
        Ctx *c = s->acquire();
        if (!c) return set_err(ZR_ERR_DEVICE, "cannot create execution context");
        CtxLock lk(c);
        HIP_TRY(hipSetDevice(s->device));
        const size_t bytes = row_stride * h;
        if (int rc = ctx_stream(c)) return rc;
        if (int rc = grow(c->image, c->image_bytes, bytes ? bytes : 4)) return rc;
        if (int rc = sync_outputs(s, c, n_views)) return rc;
        HIP_TRY(hipStreamWaitEvent(c->stream, c->done, 0));
        HIP_TRY(hipMemcpyAsync(c->image, rgba, bytes, hipMemcpyHostToDevice, c->stream));
        zr_frame f{c->image, w, h, (uint64_t)row_stride};
        if (int rc = views_common(s, c, &f, 1, views, nullptr, n_views, lo, hi, c->outs.data(), c->stream))
            return rc;
        for (size_t i = 0; i < s->plan.outputs.size(); i++)
            HIP_TRY(hipMemcpyAsync(outputs[i], c->outs[i], s->plan.outputs[i].per_image * n_views * 4,
                                   hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return ZR_OK;
    });
}

int zr_preprocess_views_async(const zr_frame *frames, size_t n_frames, const zr_view *views,
                              const uint32_t *view_frame, size_t n_views, uint32_t ow, uint32_t oh,
                              float lo, float hi, float *d_out, void *hip_stream) {
    return guarded([&]() -> int {
        if (!frames || !views || !d_out || n_views == 0 || ow == 0 || oh == 0)
            return set_err(ZR_ERR_INVALID_ARGUMENT, "null argument or empty shape");
        if (!(hi > lo)) return set_err(ZR_ERR_INVALID_ARGUMENT, "ColorMapper range must satisfy end > start");
        hipStream_t st = (hipStream_t)hip_stream;
        std::vector<zr::ViewDesc> vd(n_views);
        for (size_t i = 0; i < n_views; i++) {
            const uint32_t f = view_frame ? view_frame[i] : 0;
            if (f >= n_frames) return set_err(ZR_ERR_INVALID_ARGUMENT, "view_frame index out of range");
            vd[i] = make_view(views[i], f);
        }
        std::vector<zr::FrameDesc> fd(n_frames);
        for (size_t i = 0; i < n_frames; i++)
            if (!frames[i].rgba || frames[i].width == 0 || frames[i].height == 0)
                return set_err(ZR_ERR_INVALID_ARGUMENT, "empty frame");
        for (size_t i = 0; i < n_frames; i++)
            fd[i] = zr::FrameDesc{frames[i].rgba, frames[i].width, frames[i].height, frames[i].row_stride};
        zr::ViewDesc *dv = nullptr;
        zr::FrameDesc *df = nullptr;
        HIP_TRY(hipMallocAsync((void **)&dv, n_views * sizeof(zr::ViewDesc), st));
        HIP_TRY(hipMallocAsync((void **)&df, n_frames * sizeof(zr::FrameDesc), st));
        HIP_TRY(hipMemcpyAsync(dv, vd.data(), n_views * sizeof(zr::ViewDesc), hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(df, fd.data(), n_frames * sizeof(zr::FrameDesc), hipMemcpyHostToDevice, st));
        zr::PreprocParams p{};
        p.frames = df;
        p.nframes = (int)n_frames;
        p.views = dv;
        p.nviews = (int)n_views;
        p.OW = (int)ow;
        p.OH = (int)oh;
        p.lo = lo;
        p.adjust = (hi - lo) / 255.0f;
        p.out = d_out;
        p.o_sN = 3 * (int64_t)ow * oh;
        p.o_sC = (int64_t)ow * oh;
        zr::launch_preproc(p, st);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipFreeAsync(dv, st));
        HIP_TRY(hipFreeAsync(df, st));
        return ZR_OK;
    });
}

int zr_detection_candidates_async(const float *d_logits, const float *d_boxes, uint32_t n,
                                  uint32_t anchors, uint32_t params, float logit_min,
                                  uint32_t cap, int32_t *d_count, float *d_rec, void *hip_stream) {
    return guarded([&]() -> int {
        if (!d_logits || !d_boxes || !d_count || !d_rec) return set_err(ZR_ERR_INVALID_ARGUMENT, "null pointer");
        if (n == 0) return ZR_OK;
        zr::CandParams p{};
        p.logits = d_logits;
        p.boxes = d_boxes;
        p.N = (int)n;
        p.A = (int)anchors;
        p.D = (int)params;
        p.cap = (int)cap;
        p.logit_min = logit_min;
        p.count = d_count;
        p.rec = d_rec;
        zr::launch_candidates(p, (hipStream_t)hip_stream);
        HIP_TRY(hipGetLastError());
        return ZR_OK;
    });
}

int zr_device_count(int *n) {
    return guarded([&]() -> int {
        if (!n) return set_err(ZR_ERR_INVALID_ARGUMENT, "null n");
        *n = 0;
        if (hipGetDeviceCount(n) != hipSuccess) *n = 0;
        return ZR_OK;
    });
}

int zr_malloc(void **p, size_t bytes) {
    return guarded([&]() -> int {
        if (!p) return set_err(ZR_ERR_INVALID_ARGUMENT, "null p");
        HIP_TRY(hipMalloc(p, bytes ? bytes : 4));
        return ZR_OK;
    });
}

int zr_free(void *p) {
    return guarded([&]() -> int {
        HIP_TRY(hipFree(p));
        return ZR_OK;
    });
}

int zr_host_alloc(void **p, size_t bytes) {
    return guarded([&]() -> int {
        if (!p) return set_err(ZR_ERR_INVALID_ARGUMENT, "null p");
        HIP_TRY(hipHostMalloc(p, bytes ? bytes : 4));
        return ZR_OK;
    });
}

int zr_host_free(void *p) {
    return guarded([&]() -> int {
        HIP_TRY(hipHostFree(p));
        return ZR_OK;
    });
}

int zr_memcpy_async(void *dst, const void *src, size_t bytes, int kind, void *hip_stream) {
    return guarded([&]() -> int {
        hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                        : hipMemcpyDeviceToDevice;
        HIP_TRY(hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)hip_stream));
        return ZR_OK;
    });
}

int zr_memcpy2d_async(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height,
                      int kind, void *hip_stream) {
    return guarded([&]() -> int {
        if (height == 0 || width == 0) return ZR_OK;
        hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                        : hipMemcpyDeviceToDevice;
        HIP_TRY(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, k, (hipStream_t)hip_stream));
        return ZR_OK;
    });
}

int zr_event_create_timing(void **event) {
    return guarded([&]() -> int {
        if (!event) return set_err(ZR_ERR_INVALID_ARGUMENT, "null event");
        HIP_TRY(hipEventCreateWithFlags((hipEvent_t *)event, hipEventDefault));
        return ZR_OK;
    });
}

int zr_event_elapsed(float *ms, void *start, void *end) {
    return guarded([&]() -> int {
        if (!ms) return set_err(ZR_ERR_INVALID_ARGUMENT, "null ms");
        HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end));
        return ZR_OK;
    });
}

int zr_stream_wait_event(void *stream, void *event) {
    return guarded([&]() -> int {
        HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
        return ZR_OK;
    });
}

int zr_event_create(void **event) {
    return guarded([&]() -> int {
        if (!event) return set_err(ZR_ERR_INVALID_ARGUMENT, "null event");
        HIP_TRY(hipEventCreateWithFlags((hipEvent_t *)event, hipEventDisableTiming));
        return ZR_OK;
    });
}

int zr_event_destroy(void *event) {
    return guarded([&]() -> int {
        HIP_TRY(hipEventDestroy((hipEvent_t)event));
        return ZR_OK;
    });
}

int zr_event_record(void *event, void *stream) {
    return guarded([&]() -> int {
        HIP_TRY(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
        return ZR_OK;
    });
}

int zr_event_synchronize(void *event) {
    return guarded([&]() -> int {
        HIP_TRY(hipEventSynchronize((hipEvent_t)event));
        return ZR_OK;
    });
}

int zr_event_query(void *event) {
    return guarded([&]() -> int {
        const hipError_t e = hipEventQuery((hipEvent_t)event);
        if (e == hipSuccess) return ZR_OK;
        (void)hipGetLastError();  // not-ready is no failure; a failure is returned here, once
        if (e == hipErrorNotReady) return 1;
        return set_err(ZR_ERR_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(e));
    });
}

int zr_stream_create(void **stream) {
    return guarded([&]() -> int {
        if (!stream) return set_err(ZR_ERR_INVALID_ARGUMENT, "null stream");
        HIP_TRY(hipStreamCreateWithFlags((hipStream_t *)stream, hipStreamNonBlocking));
        return ZR_OK;
    });
}

int zr_stream_destroy(void *stream) {
    return guarded([&]() -> int {
        HIP_TRY(hipStreamDestroy((hipStream_t)stream));
        return ZR_OK;
    });
}

int zr_stream_synchronize(void *stream) {
    return guarded([&]() -> int {
        HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
        return ZR_OK;
    });
}

}  // extern "C"
