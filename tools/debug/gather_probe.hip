// what FETCH_SIZE counts for the stems' 4-byte RGBA gathers.  BlazeFace's
// fused preprocessing samples a 1920x1080 frame letterboxed into 1920x1920 at 128x128: one
// 4-byte pixel every 15 pixels (60 B apart in a row, 15 rows apart), 128 x 72 samples inside the
// frame.  Three kernels over 341 distinct frames (2.8 GB, far past the 256 MiB MALL):
//   seq4:   every u32 of the frames once, 4-byte loads, lanes contiguous (known bytes: the
//           calibration of FETCH_SIZE for 4-byte accesses)
//   gather: the stem's sample pattern, one u32 per sample (known bytes: 4 per sample; the lines
//           touched: 128 B per sample, none shared)
//   dense:  FaceMesh-like sampling of a 512x512 ROI at 192x192 (2.67 px apart: several samples
//           per line)
// Run under rocprofv3 --pmc FETCH_SIZE --kernel-trace and divide FETCH_SIZE per dispatch by the
// counts printed here.  Build: hipcc --offload-arch=gfx950 -O3 tools/debug/gather_probe.hip -o tools/debug/gather_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int FW = 1920, FH = 1080, NF = 341;

__global__ void seq4(const unsigned *f, size_t n, unsigned *sink) {
    unsigned s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += f[i];
    if (s == 0x12345u) sink[0] = s;
}

// one workgroup per frame and sample row: 128 samples, 15 px apart (x = 15 i + 7, y = 15 r + 7)
__global__ void gather(const unsigned *f, unsigned *out) {
    const int fr = blockIdx.y, r = blockIdx.x, i = threadIdx.x;
    const size_t y = 15 * (size_t)r + 7, x = 15 * (size_t)i + 7;
    const unsigned v = f[(size_t)fr * FW * FH + y * FW + x];
    out[((size_t)fr * 72 + r) * 128 + i] = v;
}

// 192 samples per row over a 512-px ROI at (600, 300): 2.67 px apart
__global__ void dense(const unsigned *f, unsigned *out) {
    const int fr = blockIdx.y, r = blockIdx.x, i = threadIdx.x;
    const size_t y = 300 + (size_t)(r * 512 / 192), x = 600 + (size_t)(i * 512 / 192);
    const unsigned v = f[(size_t)fr * FW * FH + y * FW + x];
    out[((size_t)fr * 192 + r) * 192 + i] = v;
}

int main() {
    const size_t npx = (size_t)NF * FW * FH;
    unsigned *f, *out, *sink;
    if (hipMalloc(&f, npx * 4) != hipSuccess || hipMalloc(&out, (size_t)NF * 192 * 192 * 4) != hipSuccess ||
        hipMalloc(&sink, 4) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(f, 1, npx * 4);
    hipDeviceSynchronize();
    for (int rep = 0; rep < 2; ++rep) {
        seq4<<<4096, 256>>>(f, npx, sink);
        gather<<<dim3(72, NF), 128>>>(f, out);
        dense<<<dim3(192, NF), 192>>>(f, out);
    }
    hipDeviceSynchronize();
    printf("seq4 bytes %zu\n", npx * 4);
    printf("gather samples %d bytes %d lines_128B %d\n", NF * 72 * 128, NF * 72 * 128 * 4, NF * 72 * 128 * 128);
    // dense: distinct 128-B lines touched per frame (the ROI's rows and 32-px line spans)
    printf("dense samples %d bytes %d lines_128B_approx %d\n", NF * 192 * 192, NF * 192 * 192 * 4, NF * 192 * 17 * 128);
    return 0;
}
