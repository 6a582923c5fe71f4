// group.h -- independent launches of one kernel instance fused into one grid.  The plan
// compiler groups sibling steps (same form, no data dependency between them: the two FaceMesh
// head branches, the four hand-landmark heads) so the GPU runs them side by side in one launch
// instead of back to back -- those launches are a few dozen workgroups each, latency chains
// that leave most CUs idle.  Each part keeps its own parameters and grid; a workgroup finds its
// part from the flattened block index (wave-uniform), and the kernel body runs unchanged, so a
// grouped step computes exactly what it computes alone.
#pragma once
#include <hip/hip_runtime.h>

#include "../runtime/zr_kernels.h"

namespace zr {

template <class T>
struct LaunchGroup {
    T p[ZR_GROUP_MAX];
    int a0[ZR_GROUP_MAX], a1[ZR_GROUP_MAX], a2[ZR_GROUP_MAX];  // per-part scalar kernel arguments
    int gx[ZR_GROUP_MAX];                                      // per-part grid.x (blocks gx * gy)
    int start[ZR_GROUP_MAX + 1];                               // first flattened block of each part
    int n;
};

// the part of this workgroup and its (bx, by) inside the part's own grid
struct GroupSlot {
    int g, bx, by;
};
template <class T>
__device__ __forceinline__ GroupSlot group_slot(const LaunchGroup<T> &G) {
    const int b = (int)blockIdx.x;
    int g = 0;
#pragma unroll
    for (int i = 1; i < ZR_GROUP_MAX; ++i) g += (i < G.n && b >= G.start[i]) ? 1 : 0;
    const int local = b - G.start[g], gx = G.gx[g];
    return {g, local % gx, local / gx};
}

}  // namespace zr
