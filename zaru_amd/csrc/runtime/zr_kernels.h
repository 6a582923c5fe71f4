// zr_kernels.h -- launch descriptors shared by the graph runtime and the gfx950 kernels.
//
// Activation layout in HBM ("CNHW"): element (n, c, p) of an internal tensor with
// N images, C channels and P = H*W positions lives at  c*(N*P) + n*P + p.  Every
// 1x1 convolution is then a plain GEMM  out[Cout][N*P] = W[Cout][Cin] . X[Cin][N*P]
// with both operands contiguous along the column axis, whatever the spatial size.
// Graph outputs are written directly in the reference's row-major layout (batch in
// dim 0) through explicit (sN, sC, sP) strides, so no transpose/reshape/concat ever
// runs as a separate pass.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zr {

enum ActKind : int { ACT_NONE = 0, ACT_RELU = 1, ACT_CLIP = 2, ACT_PRELU = 3, ACT_SIGMOID = 4 };

struct Act {
    int kind = ACT_NONE;
    float lo = 0.f, hi = 0.f;        // Clip bounds
    const float *slope = nullptr;    // PReLU per-channel slope (device)
};

// Generic strided view of a 4-D activation: element (n, c, y, x) at
// base + n*sN + c*sC + y*sY + x  (x is always unit stride).
struct Plane {
    const float *p;
    int64_t sN, sC;
    int C, H, W;
};

// ---------------------------------------------------------------- GEMM (1x1 conv / Gemm /
// full-plane conv).  Column j = n*P + q  (P output positions per image).
// B operand X(k, j): x + n*x_sN + (k / KK)*x_sC + (k % KK)*x_sK + q   (KK = 1 except for a
// convolution whose kernel covers its whole input plane, where KK = kh*kw and P = 1).
struct GemmParams {
    const float *x;
    int64_t x_sN, x_sC;
    int KK, x_sK;
    // KK > 1 im2col addressing (gemm_kernel<., true>): k = ci*KK + ky*pk + kx reads
    // x[ci*x_sC + (oy*ph + ky)*x_W + ox*pk + kx] for output q = oy*out_W + ox -- full-plane
    // convs (ph x pk = the plane, one output; ph may differ from pk) and non-overlapping
    // patches (ph == pk)
    int pk, ph, x_W;
    int P, ncols;        // positions per image, N*P
    int M, K;            // Cout, reduction length (Cin*KK)
    int Mpad, Kpad;      // weights zero-padded to multiples of 32 / 8
    const float *wt;     // [Kpad][Mpad]  (transposed)
    const float *bias;   // [Mpad]
    Act pre, post;       // y = post( pre(acc + bias) + residual )
    // residual (channel-padded, optionally 2x2 max-pooled) source
    int res_mode;        // 0 none, 1 direct, 2 maxpool 2x2/2
    const float *r;
    int64_t r_sN, r_sC;
    int r_C, r_W;        // channels present in the residual (rest are zero); source width
    int out_W;           // output width (to split q into y, x for pooling)
    // output (m, j) at out + n*o_sN + m*o_sC + q*o_sP
    float *out;
    int64_t o_sN, o_sC, o_sP;
    // device image count (may be null): workgroups whose columns all lie in images >= *nact may
    // skip their work -- those images' outputs are then undefined (the BlazePalm launches of the
    // device HandTracker run over the streams due for detection only, hand/tracking.rs:210-218)
    const int *nact;
};

// ---------------------------------------------------------------- depthwise conv
struct DwParams {
    Plane in;
    float *out;
    int64_t o_sN, o_sC;
    int OH, OW, N;
    int k, stride, pad_t, pad_l;
    const float *w;      // [C][k*k]
    const float *bias;   // [C]
    Act act;
};

// ---------------------------------------------------------------- dense direct conv
struct DirectParams {
    Plane in;
    float *out;
    int64_t o_sN, o_sC;
    int OH, OW, N, Cout;
    int kh, kw, stride, pad_t, pad_l;
    const float *w;      // [Cout][Cin][kh][kw]
    const float *bias;   // [Cout]
    Act act;
};

// ---------------------------------------------------------------- elementwise family
struct EltParams {
    int op;              // 0 act-copy, 1 add(a,b), 2 maxpool2 of a, 3 channel-pad of a
    Plane a, b;          // sources (b only for add)
    float *out;
    int64_t o_sN, o_sC;
    int N, C, H, W;      // output geometry
    Act act;
};

struct ResizeParams {    // bilinear, half_pixel, edge clamp
    Plane in;
    float *out;
    int64_t o_sN, o_sC;
    int N, OH, OW;
    float scale_y, scale_x;  // in/out ratio
    const int *nact;         // as GemmParams::nact
};

struct GapParams {
    Plane in;
    float *out;
    int64_t o_sN, o_sC;
    int N;
};

// ---------------------------------------------------------------- preprocessing
// One view: a RotatedRect in root-image coordinates (image/mod.rs:188-192) with its
// host-computed (glibc) cos/sin and the derived f32 quantities the reference recomputes
// per sample.  All arithmetic in the kernel is IEEE f32 without contraction.
struct ViewDesc {
    float half_w, half_h;    // rect.size() * 0.5
    float tl_x, tl_y;        // rect.top_left() = centre - size * 0.5
    float view_w, view_h;    // rect.size()
    float cos_r, sin_r;      // cosf(rad), sinf(rad)
    uint32_t frame;          // index into the frame array
    uint32_t pad_;
};

struct FrameDesc {
    const uint8_t *rgba;
    uint32_t w, h;
    uint64_t stride;         // bytes per row
};

struct PreprocParams {
    const FrameDesc *frames;
    const ViewDesc *views;
    int nviews, OW, OH;
    int nframes;             // a view whose frame index is >= nframes samples Color::NONE
    float lo, adjust;        // ColorMapper: c * adjust + lo
    float *out;              // (view v, channel c, position q) at out + v*o_sN + c*o_sC + q
    int64_t o_sN, o_sC;
};

// ---------------------------------------------------------------- detection candidates
// Per image: anchors whose logit >= logit_min (a conservative bound below logit(thresh))
// are compacted as {anchor index, logit, raw box params} for the exact host decode.
struct CandParams {
    const float *logits;     // [N][A]
    const float *boxes;      // [N][A][D]
    int N, A, D, cap;
    float logit_min;
    int *count;              // [N]
    float *rec;              // [N][cap][2 + D]
};

// ---------------------------------------------------------------- fused kernels (fused.hip)
// Dense KxK stride-S stem conv with Cin = 3 (every model's first layer).  With `pre` the
// kernel samples its input from RGBA frames through per-image views (K1 fused in front);
// otherwise it reads the f32 tensor `in`.
struct StemParams {
    Plane in;
    PreprocParams pre;   // frames / views / lo / adjust (used with pre)
    float *out;
    int64_t o_sN, o_sC;
    int IH, IW, OH, OW, N, Cout;
    int k, stride, pad_t, pad_l;
    const float *w;      // [3][k][k][32] (output channel innermost, zero-padded to 32)
    const float *bias;   // [>= 32]
    Act act;
    const int *nact;     // as GemmParams::nact
};

// Depthwise KxK conv feeding a 1x1 conv (BlazeBlock / inverted-residual tail) in one launch.
// `g` describes the 1x1 conv exactly as for launch_gemm (its x is unused: the depthwise output
// of each column tile is computed into LDS), `in` is the depthwise input.
struct DwPwParams {
    GemmParams g;
    Plane in;
    int OW;              // depthwise output width (= positions per row of g's columns)
    int k, stride, pad_t, pad_l;
    const float *dw_w;   // [Cin][k*k]
    const float *dw_b;   // [Cin]
    Act dw_act;
};

// Kernel forms the launchers and the plan compiler choose between.  Every form computes the same
// arithmetic in the same order, so switching one changes no output bit (tests/test_gpu_forms.py).
// ZARU_HIP_FORMS, read once per process, switches forms off ("-dma,-v4"), for verification and
// A/B runs.
//   dma: LDS-DMA staged MFMA dwpw (dwpw_dma_kernel)   v4: windowed depthwise taps (dwpw_kernel)
//   valu: VALU dwpw for few-channel high-resolution layers   valu_db: its double-buffered staging
//   rows: image-row head GEMM (gemm_rows_kernel)
//   vres: VALU dwpw taking the block's residual from the staged depthwise taps
//   vstore: 16-B row-segment GEMM epilogue
//   ws: warp-specialized persistent MFMA dwpw (dwpw_ws.hip)
//   groups: sibling steps launched as one grid (plan.cpp group_siblings, kernels/group.h)
//   dwgap: depthwise + global average pool in one launch (plan.cpp fuse_dw_gap)
//   rt: row-task depthwise inside the LDS-DMA MFMA dwpw (dwpw_dma_body, RT > 0)
//   ir: expand 1x1 + depthwise + projection in one launch (plan.cpp mark_inverted_residuals, ir.hip)
//   bneck: FaceMesh V2's reduction 1x1 + depthwise + 1x1 + residual in one launch (bneck.hip)
//   pin: the row-task depthwise's window reads at full width (ds_read_b64 / b128, dwpw_dma_pin_kernel)
enum Form : int { FORM_DMA, FORM_V4, FORM_VALU, FORM_VALU_DB, FORM_ROWS, FORM_VRES, FORM_VSTORE, FORM_WS, FORM_GROUPS, FORM_DWGAP, FORM_RT, FORM_IR, FORM_IRL, FORM_IRL2, FORM_BNECK, FORM_PIN, FORM_COUNT };
bool form_on(Form f);

bool stem_supported(int cin, int k, int stride, int cout);
bool dwpw_supported(int k, int stride);

// launchers (kernels/*.hip); each returns the symbol of the kernel it launched
// The symbol a launch ran, as rocprofv3 prints it (spaces removed), for the profiler: printf
// formatting interned in a mutex-guarded set, so the pointer stays valid and concurrent
// launches from several threads are safe.
const char *kernel_name(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

const char *launch_gemm(const GemmParams &p, hipStream_t s);
const char *launch_dw(const DwParams &p, hipStream_t s);
const char *launch_direct(const DirectParams &p, hipStream_t s);
const char *launch_elt(const EltParams &p, hipStream_t s);
const char *launch_resize(const ResizeParams &p, hipStream_t s);
const char *launch_gap(const GapParams &p, hipStream_t s);
// depthwise + activation + global average pool in one launch (out / o_sN / o_sC: the pooled
// vector); planes of <= 512 floats (64 of them staged in LDS)
const char *launch_dwgap(const DwParams &p, hipStream_t s);
const char *launch_preproc(const PreprocParams &p, hipStream_t s);
const char *launch_candidates(const CandParams &p, hipStream_t s);
const char *launch_stem(const StemParams &p, bool pre, hipStream_t s);
const char *launch_dwpw(const DwPwParams &p, hipStream_t s);
const char *launch_dwpw_mfma(const DwPwParams &p, hipStream_t s);  // the MFMA forms (dwpw_mfma.hip)
const char *launch_dwpw_ws(const DwPwParams &p, hipStream_t s, bool launch);  // nullptr: the layer does not fit it
constexpr int ZR_GROUP_MAX = 4;  // steps per launch group
// Sibling steps (independent, same kernel instance) in one launch (kernels/group.h); nullptr
// when the parts would not run the same grouped instance: the caller launches them one by one.
const char *launch_gemm_group(const GemmParams *p, int n, hipStream_t s);
const char *launch_dwpw_group(const DwPwParams *p, int n, hipStream_t s);
const char *launch_dwpw_mfma_group(const DwPwParams *p, int n, hipStream_t s);
// An expand 1x1 (e) and the depthwise + 1x1 step reading its output (d) in one launch (ir.hip);
// nullptr when the shapes do not fit (the caller launches both).
const char *launch_ir(const GemmParams &e, const DwPwParams &d, hipStream_t s);
// the same for the low-resolution blocks (irl.hip: a workgroup per image plane)
const char *launch_irl(const GemmParams &e, const DwPwParams &d, hipStream_t s);
// FaceMesh V2's bottleneck pair (a C -> C/2 reduction feeding a 3x3 dwpw back to C with the
// reduction's input as residual) in one launch (bneck.hip); nullptr when the shapes do not fit
const char *launch_bneck(const GemmParams &e, const DwPwParams &d, hipStream_t s);

}  // namespace zr
