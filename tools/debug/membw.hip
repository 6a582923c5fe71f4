// HBM write / read / copy ceilings on this GPU for the store-bound expand GEMMs: 16-B vector
// stores and loads over buffers far larger than L2 + MALL, one grid-stride kernel per pattern.
// Build: hipcc --offload-arch=gfx950 -O3 tools/debug/membw.hip -o tools/debug/membw
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void fill4(float4 *o, size_t n4, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        o[i] = make_float4(v, v, v, v);
}
__global__ void read4(const float4 *a, size_t n4, float *sink) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 x = a[i];
        s += x.x + x.y + x.z + x.w;
    }
    if (s == 12345.f) sink[0] = s;
}
__global__ void copy4(const float4 *a, float4 *o, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) o[i] = a[i];
}
// the expand GEMM's store pattern without the GEMM: each workgroup writes M rows x 128 columns
// of a [M][ncols] matrix (512 B per row), rows ncols * 4 B apart
__global__ void rows4(float *o, int M, size_t ncols, float v) {
    const size_t c0 = (size_t)blockIdx.x * 128;
    const int lane = threadIdx.x & 31, r0 = threadIdx.x >> 5;  // 8 rows per pass, 32 float4 per row
    for (int r = r0; r < M; r += 8)
        if (c0 + 4 * lane < ncols) *(float4 *)(o + (size_t)r * ncols + c0 + 4 * lane) = make_float4(v, v, v, v);
}

int main() {
    const size_t bytes = (size_t)4 << 30, n4 = bytes / 16;
    float4 *a, *b;
    float *sink;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMalloc(&sink, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grids[] = {1024, 4096, 16384};
    for (int g : grids) {
        float ms;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            fill4<<<g, 256>>>(a, n4, 1.f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
        }
        hipEventElapsedTime(&ms, e0, e1);
        printf("write  grid %5d: %.2f TB/s\n", g, bytes / ms / 1e9);
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            read4<<<g, 256>>>(a, n4, sink);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
        }
        hipEventElapsedTime(&ms, e0, e1);
        printf("read   grid %5d: %.2f TB/s\n", g, bytes / ms / 1e9);
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            copy4<<<g, 256>>>(a, b, n4 / 2);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
        }
        hipEventElapsedTime(&ms, e0, e1);
        printf("copy   grid %5d: %.2f TB/s (read + write)\n", g, bytes / ms / 1e9);
    }
    // expand-GEMM-shaped stores: 64 rows x 4.26 M columns (the hand 112^2 expand at 340 ROIs)
    const int M = 64;
    const size_t ncols = 4264960;
    for (int rep = 0; rep < 3; ++rep) {
        float ms;
        hipEventRecord(e0);
        rows4<<<(unsigned)((ncols + 127) / 128), 256>>>((float *)a, M, ncols, 2.f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        if (rep == 2) printf("rows   64 x %zu (512-B row segments per workgroup): %.1f us, %.2f TB/s\n", ncols, ms * 1e3,
                             (double)M * ncols * 4 / ms / 1e9);
    }
    hipFree(a);
    hipFree(b);
    return 0;
}
