// detpost.hip -- Detector::detect_impl after inference, on the device (crates/zaru/src/
// detection.rs:231-267): extract_outputs (sigmoid, threshold, decode: face/detection.rs:96-157,
// hand/detection.rs:108-179), weighted NMS (detection/nms.rs:59-145, Average mode) and the map
// back into frame pixels (detection.rs:245-267).  One wave per frame; the host restatement
// (host/detection.cpp) is matched bit for bit:
//   * conf = 1 / (1 + expf(-logit)) with glibc's expf (glibc_math.h), kept unless conf < thresh;
//   * the decode, IoU, weighted sums and map are f32 in the host's operation order (no
//     contraction: -ffp-contract=off), the angle with glibc's atan2f;
//   * the NMS order is ascending total_cmp of the confidence, ties in anchor order (the host's
//     stable sort, = Rust's sort_unstable on <= 20 elements), seeds popped from the top, each
//     group summed seed first then in ascending order.  Above 20 candidates Rust sorts with
//     ipnsort, which is not stable: a frame with more than 20 candidates and an exact confidence
//     tie (sigmoid saturates to 1.0f above logit ~16.6) has an order the reference does not pin;
//     `ties` reports each frame's candidate and tied-candidate counts so callers can count them.
// Candidates (anchor, conf) and their rects live in LDS; the group sums re-decode a member's
// keypoints from the raw outputs, which is the same arithmetic as decoding it once.
#include "../runtime/zr_track.h"
#include "geom_dev.h"

namespace zr {
namespace {

using namespace geo;

__device__ __forceinline__ int32_t total_key(float f) {  // f32::total_cmp (zaru-image/src/num.rs:7-27)
    const int32_t i = (int32_t)glibc::asuint(f);
    return i ^ (int32_t)(((uint32_t)(i >> 31)) >> 1);
}

struct Decoded {
    float cx, cy, w, h, angle;
};

// extract_detection for anchor a: centre, size, and the angle from two keypoints
__device__ __forceinline__ Decoded decode(const DetPostParams &P, const float *b, int a) {
    const float iw = (float)P.in_w, ih = (float)P.in_h;
    Decoded d;
    d.cx = b[0] + P.anchors[2 * a] * iw;
    d.cy = b[1] + P.anchors[2 * a + 1] * ih;
    d.w = b[2];
    d.h = b[3];
    const float cxi = d.cx * iw, cyi = d.cy * ih;  // the keypoint offset (quirk kept, face/detection.rs:135)
    auto kp = [&](int k) -> V2 { return {b[4 + 2 * k] + cxi, b[5 + 2 * k] + cyi}; };
    if (P.face) {  // left eye -> right eye against +X (face/detection.rs:151-154)
        const V2 k0 = kp(0), k1 = kp(1);
        d.angle = signed_angle_to({k1.x - k0.x, k1.y - k0.y}, {1.f, 0.f});
    } else {  // wrist - middle finger MCP against +Y (hand/detection.rs:172-176)
        const V2 k0 = kp(0), k2 = kp(2);
        d.angle = signed_angle_to({k0.x - k2.x, k0.y - k2.y}, {0.f, 1.f});
    }
    return d;
}

__global__ __launch_bounds__(64) void det_post_kernel(const DetPostParams P) {
    extern __shared__ float lds_dp[];
    const int f = blockIdx.x, lane = threadIdx.x;
    if (P.nact && f >= *P.nact) return;  // (whole wave)
    const int fo = P.map ? P.map[f] : f;  // the output slot
    const int A = P.A;
    int *ca = (int *)lds_dp;               // candidate anchors, anchor order    [A]
    float *cc = lds_dp + A;                // their confidences                  [A]
    int *ord = (int *)(lds_dp + 2 * A);    // candidate ids in NMS order          [A]
    float *cr = lds_dp + 3 * A;            // their rects (cx, cy, w, h)           [4A]
    int *grp = (int *)(lds_dp + 7 * A);    // the current group                   [A]
    const float *logits = P.logits + (int64_t)f * A;
    const float *boxes = P.boxes + (int64_t)f * A * P.D;

    // 1. extract_outputs: anchors in order, compacted with a wave ballot
    int n = 0;
    for (int a0 = 0; a0 < A; a0 += 64) {
        const int a = a0 + lane;
        float conf = 0.f;
        bool keep = false;
        if (a < A) {
            conf = sigmoid(logits[a]);
            keep = !(conf < P.thresh);
        }
        const uint64_t m = __ballot(keep);
        if (keep) {
            const int at = n + (int)__popcll(m & ((1ull << lane) - 1ull));
            ca[at] = a;
            cc[at] = conf;
        }
        n += (int)__popcll(m);
    }
    __syncthreads();
    // 2. rects, and 3. the ascending stable order: rank = #smaller keys + #equal keys before
    __shared__ int s_tied;  // candidates whose key another candidate shares (NonMaxSuppression::TieCount)
    if (lane == 0) s_tied = 0;
    __syncthreads();
    for (int i = lane; i < n; i += 64) {
        const float *b = boxes + (int64_t)ca[i] * P.D;
        cr[4 * i] = b[0] + P.anchors[2 * ca[i]] * (float)P.in_w;
        cr[4 * i + 1] = b[1] + P.anchors[2 * ca[i] + 1] * (float)P.in_h;
        cr[4 * i + 2] = b[2];
        cr[4 * i + 3] = b[3];
        const int32_t ki = total_key(cc[i]);
        int r = 0, eq = 0;
        for (int j = 0; j < n; ++j) {
            const int32_t kj = total_key(cc[j]);
            r += (kj < ki || (kj == ki && j < i)) ? 1 : 0;
            eq += (kj == ki && j != i) ? 1 : 0;
        }
        ord[r] = i;
        if (eq) atomicAdd(&s_tied, 1);
    }
    __syncthreads();

    // 4. NMS: pop the most confident, group everything within the IoU threshold (keeping order),
    // average the group weighted by confidence, map into the frame
    const float *lb = P.letterbox + 4 * fo;
    const float scale = lb[2] / (float)P.in_w;
    const float tlx = lb[0] - lb[2] * 0.5f, tly = lb[1] - lb[3] * 0.5f;
    const int rw = 2 + 20 * P.rmax;
    float *rec = P.rec ? P.rec + (int64_t)fo * rw : nullptr;
    int rem = n, out = 0;
    while (rem > 0) {
        const int seed = ord[--rem];
        const float sx = cr[4 * seed], sy = cr[4 * seed + 1], sw = cr[4 * seed + 2], sh = cr[4 * seed + 3];
        int ng = 0, nk = 0;
        for (int i0 = 0; i0 < rem; i0 += 64) {
            const int i = i0 + lane;
            int id = 0;
            bool in = false;
            if (i < rem) {
                id = ord[i];
                in = iou(sx, sy, sw, sh, cr[4 * id], cr[4 * id + 1], cr[4 * id + 2], cr[4 * id + 3]) >= P.iou;
            }
            const uint64_t mg = __ballot(i < rem && in), mk = __ballot(i < rem && !in);
            const uint64_t below = (1ull << lane) - 1ull;
            __syncthreads();  // every lane has read ord[i0 .. i0 + 63] before the in-place compaction
            if (i < rem) {
                if (in) grp[ng + (int)__popcll(mg & below)] = id;
                else ord[nk + (int)__popcll(mk & below)] = id;  // retain: order kept, nk <= i
            }
            ng += (int)__popcll(mg);
            nk += (int)__popcll(mk);
            __syncthreads();
        }
        rem = nk;
        if (lane == 0 && P.mode == 1) {
            // SuppressionMode::Remove (nms.rs:70-76): the group is dropped, the seed kept as decoded
            const float *b = boxes + (int64_t)ca[seed] * P.D;
            const Decoded d = decode(P, b, ca[seed]);
            const float cxi = d.cx * (float)P.in_w, cyi = d.cy * (float)P.in_h;
            float e[20];
            e[0] = cc[seed];
            e[1] = d.angle;
            e[2] = d.cx * scale + tlx;
            e[3] = d.cy * scale + tly;
            e[4] = d.w * scale;
            e[5] = d.h * scale;
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                e[6 + 2 * k] = k < P.nkp ? (b[4 + 2 * k] + cxi) * scale + tlx : 0.f;
                e[7 + 2 * k] = k < P.nkp ? (b[5 + 2 * k] + cyi) * scale + tly : 0.f;
            }
            if (out < P.dcap) {
                float *o = P.dets + ((int64_t)fo * P.dcap + out) * 20;
#pragma unroll
                for (int k = 0; k < 20; ++k) o[k] = e[k];
            }
            if (rec && out < P.rmax) {
#pragma unroll
                for (int k = 0; k < 20; ++k) rec[2 + 20 * out + k] = e[k];
            }
        } else if (lane == 0) {
            // the weighted average over [seed] + group, each accumulator summed in that order
            float divisor = 0.f, ax = 0.f, ay = 0.f, aw = 0.f, ah = 0.f, aa = 0.f;
            float kx[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, ky[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            for (int g = -1; g < ng; ++g) {
                const int id = g < 0 ? seed : grp[g];
                const float *b = boxes + (int64_t)ca[id] * P.D;
                const Decoded d = decode(P, b, ca[id]);
                const float c = cc[id];
                divisor += c;
                const float cxi = d.cx * (float)P.in_w, cyi = d.cy * (float)P.in_h;
#pragma unroll
                for (int k = 0; k < 7; ++k)  // (static indices: the sums stay in registers)
                    if (k < P.nkp) {
                        kx[k] += (b[4 + 2 * k] + cxi) * c;
                        ky[k] += (b[5 + 2 * k] + cyi) * c;
                    }
                ax += d.cx * c;
                ay += d.cy * c;
                aw += d.w * c;
                ah += d.h * c;
                aa += d.angle * c;
            }
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                kx[k] /= divisor;
                ky[k] /= divisor;
            }
            ax /= divisor;
            ay /= divisor;
            aw /= divisor;
            ah /= divisor;
            aa /= divisor;
            // map_detections: scale, then move by the letterbox's top left
            float e[20];
            e[0] = cc[seed];
            e[1] = aa;
            e[2] = ax * scale + tlx;
            e[3] = ay * scale + tly;
            e[4] = aw * scale;
            e[5] = ah * scale;
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                e[6 + 2 * k] = k < P.nkp ? kx[k] * scale + tlx : 0.f;
                e[7 + 2 * k] = k < P.nkp ? ky[k] * scale + tly : 0.f;
            }
            if (out < P.dcap) {
                float *o = P.dets + ((int64_t)fo * P.dcap + out) * 20;
#pragma unroll
                for (int k = 0; k < 20; ++k) o[k] = e[k];
            }
            if (rec && out < P.rmax) {
#pragma unroll
                for (int k = 0; k < 20; ++k) rec[2 + 20 * out + k] = e[k];
            }
        }
        ++out;
    }
    if (lane == 0) {
        P.count[fo] = out;
        if (P.ties) {
            P.ties[2 * fo] = n;
            P.ties[2 * fo + 1] = s_tied;
        }
        if (rec) {
            const uint32_t id = P.first_id + (uint32_t)fo * P.id_stride;
            rec[0] = __builtin_bit_cast(float, id);
            rec[1] = __builtin_bit_cast(float, (uint32_t)out);
            for (int k = 20 * min(out, P.rmax); k < 20 * P.rmax; ++k) rec[2 + k] = 0.f;
        }
    }
}

}  // namespace

size_t det_post_lds(int anchors) { return sizeof(float) * 8 * (size_t)anchors; }

const char *launch_det_post(const DetPostParams &p, hipStream_t s) {
    hipLaunchKernelGGL(det_post_kernel, dim3(p.N), dim3(64), det_post_lds(p.A), s, p);
    return "det_post_kernel";
}

}  // namespace zr
