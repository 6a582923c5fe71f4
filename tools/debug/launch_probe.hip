// launch_probe.hip -- fixed costs on the box: kernel duration of an empty / barrier-only /
// one-load workgroup grid at several grid and LDS sizes, and the latency of a dependent chain of
// global loads (L2-resident and HBM-resident).  hipcc --offload-arch=gfx950 -O3 -o lp launch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_empty(float *out) {
    extern __shared__ float lds[];
    if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) out[0] = lds[0];
}
__global__ __launch_bounds__(256) void k_barriers(float *out, int n) {
    extern __shared__ float lds[];
    float a = 0.f;
    for (int i = 0; i < n; ++i) {
        lds[(threadIdx.x + i) & 255] = a;
        __syncthreads();
        a += lds[(threadIdx.x * 7 + i) & 255];
        __syncthreads();
    }
    if (a == 12345.f) out[0] = a;
}
__global__ __launch_bounds__(256) void k_loads(const float *in, float *out, int n, int stride) {
    // n dependent rounds: each round loads one float per lane, then a barrier
    float a = 0.f;
    int idx = (blockIdx.x * 256 + threadIdx.x) * stride;
    for (int i = 0; i < n; ++i) {
        a += in[idx];
        idx = (idx + (int)a + 4096 * 256) & ((1 << 26) - 1);
        __syncthreads();
    }
    if (a == 12345.f) out[0] = a;
}
__global__ void k_chase(const int *next, int *out, int n) {
    int p = 0;
    for (int i = 0; i < n; ++i) p = next[p];
    out[0] = p;
}


// straight-line code of N dependent-free VALU ops (cold instruction cache per CU) vs the same op
// count as a loop over a short body
template <int N>
__global__ __launch_bounds__(256) void k_straight(float *out, float x) {
    float a = x + threadIdx.x, b = x * 2.f, c = x - 1.f, d = x * x;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(d) : "v"(b), "v"(a));
    }
    if (a + d == 12345.f) out[0] = a;
}
__global__ __launch_bounds__(256) void k_looped(float *out, float x, int n) {
    float a = x + threadIdx.x, b = x * 2.f, c = x - 1.f, d = x * x;
    for (int i = 0; i < n; i += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
            asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(d) : "v"(b), "v"(a));
        }
    }
    if (a + d == 12345.f) out[0] = a;
}

static float time_ms(hipEvent_t a, hipEvent_t b) { float ms; hipEventElapsedTime(&ms, a, b); return ms; }

int main() {
    float *buf, *out;
    int *chase, *iout;
    const size_t N = 1 << 26;  // 256 MB of floats
    CK(hipMalloc(&buf, N * 4));
    CK(hipMalloc(&out, 1024));
    CK(hipMalloc(&chase, N * 4));
    CK(hipMalloc(&iout, 64));
    CK(hipMemset(buf, 0, N * 4));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    CK(hipFuncSetAttribute((const void *)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void *)k_barriers, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const int reps = 200;
    for (int warm = 0; warm < 2000; ++warm) hipLaunchKernelGGL(k_empty, dim3(1536), dim3(256), 0, 0, out);
    CK(hipDeviceSynchronize());
    for (int grid : {24, 96, 384, 1536, 6144}) {
        for (int lds : {0, 16 * 1024, 44 * 1024, 96 * 1024}) {
            hipEventRecord(e0);
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), lds, 0, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float te = time_ms(e0, e1) * 1000 / reps;
            hipEventRecord(e0);
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_barriers, dim3(grid), dim3(256), lds, 0, out, 8);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float tb = time_ms(e0, e1) * 1000 / reps;
            printf("{\"probe\":\"grid\",\"grid\":%d,\"lds_kb\":%d,\"empty_us\":%.2f,\"barriers8x2_us\":%.2f}\n", grid, lds / 1024, te, tb);
        }
        for (int n : {1, 4, 8}) {
            hipEventRecord(e0);
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_loads, dim3(grid), dim3(256), 0, 0, buf, out, n, 1);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            printf("{\"probe\":\"loads\",\"grid\":%d,\"rounds\":%d,\"us\":%.2f}\n", grid, n, time_ms(e0, e1) * 1000 / reps);
        }
    }
    for (int grid : {256, 1536}) {
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_straight<2048>, dim3(grid), dim3(256), 0, 0, out, 1.f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ts = time_ms(e0, e1) * 1000 / reps;
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_looped, dim3(grid), dim3(256), 0, 0, out, 1.f, 2048);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        printf("{\"probe\":\"icache\",\"grid\":%d,\"straight_4096_us\":%.2f,\"looped_4096_us\":%.2f}\n", grid, ts, time_ms(e0, e1) * 1000 / reps);
    }
    // dependent load chain: a random cycle over `span` ints
    for (size_t span : {(size_t)1 << 12, (size_t)1 << 18, (size_t)1 << 26}) {
        std::vector<int> h(span);
        std::vector<int> perm(span);
        for (size_t i = 0; i < span; ++i) perm[i] = (int)i;
        unsigned s = 12345;
        for (size_t i = span - 1; i > 0; --i) { s = s * 1103515245u + 12345u; size_t j = (s >> 4) % (i + 1); std::swap(perm[i], perm[j]); }
        for (size_t i = 0; i < span; ++i) h[perm[i]] = perm[(i + 1) % span];
        CK(hipMemcpy(chase, h.data(), span * 4, hipMemcpyHostToDevice));
        const int n = 2000;
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(1), 0, 0, chase, iout, n);
        CK(hipDeviceSynchronize());
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(1), 0, 0, chase, iout, n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        printf("{\"probe\":\"chase\",\"span_bytes\":%zu,\"ns_per_load\":%.1f}\n", span * 4, time_ms(e0, e1) * 1e6 / n);
    }
    return 0;
}
