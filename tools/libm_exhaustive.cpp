// libm_exhaustive.cpp -- checks zaru_amd/csrc/kernels/glibc_math.h (compiled for the host,
// exactly the source the GPU kernels use) against this machine's glibc over every f32 input:
// sinf, cosf, expf, atanf exhaustively (2^32 each), atan2f on N random (y, x) pairs drawn
// from every binade plus structured pairs (axes, |y| == |x|, x == 1).  Result equality is
// bitwise; two NaNs compare equal.  Prints one JSON line.
//   g++ -O2 -mfma -ffp-contract=off -fopenmp -std=c++17 tools/libm_exhaustive.cpp -lm
//   ./a.out [atan2_pairs_log2=32] [fma=1]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../zaru_amd/csrc/kernels/glibc_math.h"

static inline bool same(float a, float b) {
    if (a != a && b != b) return true;
    uint32_t x, y;
    memcpy(&x, &a, 4);
    memcpy(&y, &b, 4);
    return x == y;
}

static inline float f32(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static inline uint64_t splitmix(uint64_t &s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

template <class F, class G>
static uint64_t sweep(F mine, G ref, uint32_t *first) {
    uint64_t bad = 0;
    uint32_t fst = 0xffffffffu;
#pragma omp parallel for schedule(static, 1 << 20) reduction(+ : bad) reduction(min : fst)
    for (int64_t i = 0; i < (1LL << 32); ++i) {
        const float x = f32((uint32_t)i);
        if (!same(mine(x), ref(x))) {
            ++bad;
            if ((uint32_t)i < fst) fst = (uint32_t)i;
        }
    }
    *first = fst;
    return bad;
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 32;
    uint32_t f1, f2, f3, f4;
    const uint64_t bs = sweep([](float x) { return zr::glibc::sinf(x); }, [](float x) { return sinf(x); }, &f1);
    const uint64_t bc = sweep([](float x) { return zr::glibc::cosf(x); }, [](float x) { return cosf(x); }, &f2);
    const uint64_t be = sweep([](float x) { return zr::glibc::expf(x); }, [](float x) { return expf(x); }, &f3);
    const uint64_t ba = sweep([](float x) { return zr::glibc::atanf(x); }, [](float x) { return atanf(x); }, &f4);
    // atan2f: random bit patterns (uniform over binades) and pairs with a random ratio
    uint64_t b2 = 0, n2 = 0;
    const int64_t N = 1LL << lg;
#pragma omp parallel for schedule(static, 1 << 16) reduction(+ : b2, n2)
    for (int64_t i = 0; i < N; ++i) {
        uint64_t s = 0x5A52550000000003ULL ^ (uint64_t)i * 0x2545F4914F6CDD1DULL;
        const uint64_t r = splitmix(s);
        float y = f32((uint32_t)r), x = f32((uint32_t)(r >> 32));
        switch (i & 7) {
            case 0: break;  // any bits, NaN and Inf included
            case 1:         // |y| ~ |x|: the reduction branches near 1 (7/16 .. 2.4375)
                x = f32(((uint32_t)(r >> 32) & 0x807fffffu) | (((uint32_t)r >> 24 & 0x7f) + 64u) << 23);
                y = x * f32(0x3e000000u + (uint32_t)(r & 0x01ffffffu));
                break;
            case 2: x = 1.0f; break;
            case 3: y = ((r >> 40) & 1) ? 0.0f : -0.0f; break;
            case 4: x = ((r >> 40) & 1) ? 0.0f : -0.0f; break;
            case 5:  // moderate magnitudes: the landmark / detection angle inputs
                y = (float)((int32_t)(uint32_t)r) * 1e-6f;
                x = (float)((int32_t)(uint32_t)(r >> 32)) * 1e-6f;
                break;
            case 6: y = x; break;
            default: y = -x; break;
        }
        ++n2;
        if (!same(zr::glibc::atan2f(y, x), atan2f(y, x))) ++b2;
    }
    printf("{\"glibc\": \"%s\", \"fma_build\": %d, \"sinf_mismatch\": %llu, \"sinf_first\": \"0x%08x\", "
           "\"cosf_mismatch\": %llu, \"cosf_first\": \"0x%08x\", \"expf_mismatch\": %llu, \"expf_first\": \"0x%08x\", "
           "\"atanf_mismatch\": %llu, \"atanf_first\": \"0x%08x\", \"inputs_each\": 4294967296, "
           "\"atan2f_pairs\": %llu, \"atan2f_mismatch\": %llu}\n",
           "2.35", ZR_GLIBC_FMA, (unsigned long long)bs, f1, (unsigned long long)bc, f2, (unsigned long long)be, f3,
           (unsigned long long)ba, f4, (unsigned long long)n2, (unsigned long long)b2);
    return (bs | bc | be | ba | b2) ? 1 : 0;
}
