// libm_variants.cpp -- the f32 inputs on which glibc 2.35's two x86_64 builds of sinf / cosf /
// expf (the -mfma IFUNC variants and the baseline SSE2 ones) round differently, found by running
// both builds of zaru_amd/csrc/kernels/glibc_math.h (ZR_GLIBC_FMA=1 / 0) over every f32 input.
// Output: tests/golden/glibc_fma_variant_inputs.json, which tests/test_glibc_math_cpu.py uses to
// show which build the host's glibc resolved and that each restatement matches its build.
//   g++ -O2 -mfma -ffp-contract=off -fopenmp -std=c++17 -DZR_GLIBC_FMA=1 -c -o v1.o tools/libm_variants.cpp -DVARIANT
//   g++ -O2 -mfma -ffp-contract=off -fopenmp -std=c++17 -DZR_GLIBC_FMA=0 -c -o v0.o tools/libm_variants.cpp -DVARIANT
//   g++ -O2 -fopenmp -std=c++17 tools/libm_variants.cpp v1.o v0.o -o variants && ./variants
#ifdef VARIANT
#include "../zaru_amd/csrc/kernels/glibc_math.h"
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
extern "C" float CAT(eval_, ZR_GLIBC_FMA)(int fn, float x) {
    switch (fn) {
        case 0: return zr::glibc::sinf(x);
        case 1: return zr::glibc::cosf(x);
        default: return zr::glibc::expf(x);
    }
}
#else
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

extern "C" float eval_1(int, float);
extern "C" float eval_0(int, float);

int main() {
    const char *names[3] = {"sinf", "cosf", "expf"};
    printf("{");
    for (int fn = 0; fn < 3; fn++) {
        std::vector<uint32_t> all;
#pragma omp parallel
        {
            std::vector<uint32_t> mine;
#pragma omp for schedule(static)
            for (int64_t u = 0; u < (int64_t)1 << 32; u++) {
                const uint32_t v = (uint32_t)u;
                float x;
                memcpy(&x, &v, 4);
                const float a = eval_1(fn, x), b = eval_0(fn, x);
                if (memcmp(&a, &b, 4) != 0 && !(a != a && b != b)) mine.push_back(v);
            }
#pragma omp critical
            all.insert(all.end(), mine.begin(), mine.end());
        }
        std::sort(all.begin(), all.end());
        printf("%s\"%s\": [", fn ? ", " : "", names[fn]);
        for (size_t i = 0; i < all.size(); i++) printf("%s%u", i ? ", " : "", all[i]);
        printf("]");
    }
    printf("}\n");
}
#endif
