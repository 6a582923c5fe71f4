// plan.h -- a compiled, fused, statically scheduled execution plan for one ONNX CNN.
//
// The compiler (plan.cpp) replaces what tract's into_optimized()/SimplePlan and ORT's
// session do for the reference (crates/zaru/src/nn/mod.rs:259-362): it lowers the graph
// into a short list of HIP kernel launches with
//   * Relu / PRelu / Clip / Sigmoid folded into their producer,
//   * residual Add (+ channel Pad, + 2x2 MaxPool of the shortcut) folded into the 1x1 conv
//     epilogue,
//   * Transpose / Reshape / Squeeze / Concat folded into store addressing of the producer,
//   * every intermediate in the CNHW layout of zr_kernels.h, with arena slots reused by
//     liveness (activations for B images need only arena_per_image * B floats).
#pragma once
#include <string>
#include <vector>

#include "onnx_model.h"
#include "zr_kernels.h"

namespace zr {

// S_DWGAP: a depthwise conv (S_DW fields) whose only consumer was a global average pool; `out`
// is the pooled vector
enum StepKind { S_GEMM, S_DW, S_DIRECT, S_ELT, S_RESIZE, S_GAP, S_DWPW, S_DWGAP };

struct TRef {
    int kind = 0;  // 0 internal storage, 1 graph input, 2 graph output
    int id = -1;
    int C = 0, H = 1, W = 1;
    // kind 2: element (n, c, q) -> out[id] + n*o_sN + off + c*o_sC + q*o_sP
    int64_t off = 0, o_sN = 0, o_sC = 0, o_sP = 1;
    // kind 0: first channel inside the storage (a member of an internal channel Concat)
    int c_off = 0;
};

struct ActDesc {
    int kind = ACT_NONE;
    float lo = 0.f, hi = 0.f;
    int64_t slope_off = -1;  // offset into the weight arena (floats)
};

struct Step {
    StepKind kind;
    std::string name;  // ONNX node that anchors the step (diagnostics / profiling)
    TRef in, in2, out;
    int64_t w_off = -1, b_off = -1;
    ActDesc pre, post;
    int kh = 1, kw = 1, stride = 1, pad_t = 0, pad_l = 0;
    int KK = 1, M = 0, K = 0, Mpad = 0, Kpad = 0;
    int res_mode = 0, r_C = 0;
    int elt_op = 0;
    float scale_y = 1.f, scale_x = 1.f;
    // S_DWPW: the depthwise conv in front of the 1x1 (kh/kw/stride/pads above describe it)
    int64_t dw_w_off = -1, dw_b_off = -1;
    ActDesc dw_act;
    // S_DWGAP: the depthwise output plane (pooled away)
    int dw_oh = 0, dw_ow = 0;
    // S_DIRECT: runs as stem_kernel (Cin = 3, weights padded to 32 output channels)
    bool stem = false;
    // algorithmic traffic / work per image (for roofline accounting); bytes_pre: the same
    // step sampling its input from RGBA frames (4 B per input pixel instead of 12)
    double bytes = 0, flops = 0, bytes_pre = 0;
    // launch grouping (group_siblings): the first step of a group of independent sibling steps
    // holds the group's size (>= 2) and the members follow it; 1 = launched alone, 0 = a member
    int group = 1;
    // mark_inverted_residuals: 1 = this expand (S_GEMM) and the next step (S_DWPW, its only reader)
    // may run as one launch (launch_ir), the expanded tensor never stored
    int ir = 0;
};

struct PlanOutput {
    std::string name;
    std::vector<int64_t> shape;  // with batch dim = 1
    int64_t per_image = 0;
};

struct Plan {
    std::vector<Step> steps;
    std::vector<int64_t> storage_size;  // floats per image
    std::vector<int64_t> storage_off;   // floats per image (slot offset in the arena)
    int64_t arena_per_image = 0;
    std::vector<float> weights;         // uploaded once per session
    std::string input_name;
    int in_C = 0, in_H = 0, in_W = 0;
    std::vector<PlanOutput> outputs;
    double bytes_per_image = 0, flops_per_image = 0;
    // the graph input is read by exactly one step, a stem: view sampling can be fused into it
    bool input_fusable = false;
};

bool compile_plan(const OnnxModel &m, const std::vector<uint32_t> &out_sel, Plan &plan,
                  std::string &err);

struct Binding {
    int N = 0;
    // the batch the arena is laid out for: N rounded up to a multiple of 4, so every internal
    // channel plane (P * Ns floats) starts 16-B aligned whatever N and P are -- the LDS-DMA forms
    // need that (the padding images are never computed or read as results)
    int Ns = 0;
    const float *input = nullptr;
    int64_t in_sN = 0, in_sC = 0;   // input strides (NCHW user tensor or CNHW preproc output)
    float *const *outputs = nullptr;  // device pointers, one per plan output
    float *arena = nullptr;
    const float *weights = nullptr;
    // when set, the input comes from RGBA frames through these views (plan.input_fusable)
    const PreprocParams *pre = nullptr;
    // device image count (may be null): images >= *nact need not be computed (GemmParams::nact)
    const int *nact = nullptr;
};

// Optional per-launch hook (profiling): called before and after every kernel launch with the
// step index, the launched kernel's symbol (after only) and the launch's algorithmic work.
struct LaunchHook {
    virtual ~LaunchHook() = default;
    virtual void before(hipStream_t s) = 0;
    virtual void after(hipStream_t s, const char *kernel, double bytes, double flops) = 0;
    virtual void cancel() {}  // the launch announced by before() did not happen
};

void run_plan(const Plan &plan, const Binding &b, hipStream_t stream, LaunchHook *hook = nullptr);

}  // namespace zr
