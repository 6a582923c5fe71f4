// mfma_order.hip -- do v_mfma_f32_16x16x4_f32 and v_mfma_f32_32x32x2_f32 accumulate a K = 16
// dot product in the same order (= an fmaf chain over k ascending)?  Prints mismatch counts of
// each against the fmaf chain on random inputs (with cancellation so the order matters).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int K = 16;
// A [32][K], B [K][32] row-major; C32 [32][32] from 32x32x2; C16 [32][32] from four 16x16x4 tiles
__global__ void k32(const float *A, const float *B, float *C) {
    const int lane = threadIdx.x, col = lane & 31, kh = lane >> 5;
    f32x16 acc = {};
    for (int s = 0; s < K / 2; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[col * K + 2 * s + kh], B[(2 * s + kh) * 32 + col], acc, 0, 0, 0);
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * kh;
        C[row * 32 + col] = acc[r];
    }
}
__global__ void k16(const float *A, const float *B, float *C) {
    const int lane = threadIdx.x, col = lane & 15, kq = lane >> 4;
    for (int tm = 0; tm < 2; ++tm)
        for (int tn = 0; tn < 2; ++tn) {
            f32x4 acc = {};
            for (int s = 0; s < K / 4; ++s)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[(tm * 16 + col) * K + 4 * s + kq],
                                                         B[(4 * s + kq) * 32 + tn * 16 + col], acc, 0, 0, 0);
            for (int r = 0; r < 4; ++r) C[(tm * 16 + 4 * kq + r) * 32 + tn * 16 + col] = acc[r];
        }
}
int main() {
    std::vector<float> A(32 * K), B(K * 32), C32(1024), C16(1024), R(1024);
    srand(7);
    auto rnd = [] { return (float)((rand() / (double)RAND_MAX) * 2 - 1) * (float)(1 << (rand() % 20)); };
    for (auto &x : A) x = rnd();
    for (auto &x : B) x = rnd();
    for (int m = 0; m < 32; ++m)
        for (int n = 0; n < 32; ++n) {
            float a = 0.f;
            for (int k = 0; k < K; ++k) a = fmaf(A[m * K + k], B[k * 32 + n], a);
            R[m * 32 + n] = a;
        }
    float *dA, *dB, *dC;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dC, 4096);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k32, 1, 64, 0, 0, dA, dB, dC);
    hipMemcpy(C32.data(), dC, 4096, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k16, 1, 64, 0, 0, dA, dB, dC);
    hipMemcpy(C16.data(), dC, 4096, hipMemcpyDeviceToHost);
    int m32 = 0, m16 = 0, m3216 = 0;
    for (int i = 0; i < 1024; ++i) {
        m32 += memcmp(&C32[i], &R[i], 4) != 0;
        m16 += memcmp(&C16[i], &R[i], 4) != 0;
        m3216 += memcmp(&C16[i], &C32[i], 4) != 0;
    }
    printf("{\"k\": %d, \"mfma32x32x2_vs_fmaf_chain\": %d, \"mfma16x16x4_vs_fmaf_chain\": %d, \"mfma16_vs_mfma32\": %d}\n", K, m32, m16, m3216);
    return 0;
}
