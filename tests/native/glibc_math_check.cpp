// glibc_math_check.cpp -- test helper (not product code): the host build of
// zaru_amd/csrc/kernels/glibc_math.h next to this machine's glibc, for
// tests/test_glibc_math_cpu.py (host restatement vs glibc) and tests/test_gpu_glibc_math.py
// (device restatement vs glibc).  fn: 0 sinf, 1 cosf, 2 expf, 3 atanf, 4 atan2f(a, b).
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../zaru_amd/csrc/kernels/glibc_math.h"

static float eval_glibc(int fn, float a, float b) {
    switch (fn) {
        case 0: return sinf(a);
        case 1: return cosf(a);
        case 2: return expf(a);
        case 3: return atanf(a);
        default: return atan2f(a, b);
    }
}

static float eval_mine(int fn, float a, float b) {
    switch (fn) {
        case 0: return zr::glibc::sinf(a);
        case 1: return zr::glibc::cosf(a);
        case 2: return zr::glibc::expf(a);
        case 3: return zr::glibc::atanf(a);
        default: return zr::glibc::atan2f(a, b);
    }
}

static bool same(float x, float y) {
    if (x != x && y != y) return true;
    return memcmp(&x, &y, 4) == 0;
}

extern "C" {
void gm_glibc(int fn, const float *a, const float *b, float *out, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] = eval_glibc(fn, a[i], b ? b[i] : 0.f);
}

void gm_mine(int fn, const float *a, const float *b, float *out, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] = eval_mine(fn, a[i], b ? b[i] : 0.f);
}

// mismatches of the restatement over the bit patterns start + k * stride (k < count, mod 2^32)
uint64_t gm_sweep(int fn, uint64_t start, uint64_t count, uint64_t stride) {
    uint64_t bad = 0;
    for (uint64_t k = 0; k < count; k++) {
        const uint32_t u = (uint32_t)(start + k * stride);
        float x;
        memcpy(&x, &u, 4);
        if (!same(eval_mine(fn, x, 1.f), eval_glibc(fn, x, 1.f))) ++bad;
    }
    return bad;
}
}
