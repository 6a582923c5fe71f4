// preproc.hip -- K1 on its own: batched view sampling + ColorMapper, bit-exact with the
// reference (the arithmetic is sample.h's, shared with the stem kernel that samples frames
// itself).  Used when the network input is read by more than the stem, and by
// zr_preprocess_views_async.  The tensor is written straight into the consumer's layout
// (CNHW for the HIP runtime, NCHW for the standalone entry point).
#include "../runtime/zr_kernels.h"
#include "sample.h"

namespace zr {

__global__ __launch_bounds__(256) void preproc_kernel(const PreprocParams P) {
    const int v = blockIdx.y;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P.OW * P.OH) return;
    const int y = q / P.OW, x = q - y * P.OW;
    const ViewDesc d = P.views[v];
    const FrameDesc f = frame_of(P, d);
    const uint32_t rgba = sample_view(d, f, x, y, P.OW, P.OH);
    float *o = P.out + (int64_t)v * P.o_sN + q;
    o[0] = color_map(rgba, 0, P.adjust, P.lo);
    o[P.o_sC] = color_map(rgba, 1, P.adjust, P.lo);
    o[2 * P.o_sC] = color_map(rgba, 2, P.adjust, P.lo);
}

const char *launch_preproc(const PreprocParams &p, hipStream_t s) {
    if (p.nviews == 0) return "preproc_kernel";
    dim3 grid((p.OW * p.OH + 255) / 256, p.nviews);
    hipLaunchKernelGGL(preproc_kernel, grid, dim3(256), 0, s, p);
    return "preproc_kernel";
}

}  // namespace zr
