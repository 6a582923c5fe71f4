// hip_lasterr.cpp -- which HIP calls leave a value behind for hipGetLastError(): an event query
// on in-flight work, a query on a never-recorded event, a launch after them.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O2 tools/hip_lasterr.cpp -o gpurun_out/hip_lasterr
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(long long cycles, int *out) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

static void show(const char *what, hipError_t e) {
    const hipError_t last = hipGetLastError();
    std::printf("%-44s ret=%d (%s)  last=%d (%s)\n", what, (int)e, hipGetErrorString(e), (int)last,
                hipGetErrorString(last));
}

int main() {
    int *d = nullptr;
    hipStream_t s1, s2;
    hipEvent_t ev, fresh;
    show("hipMalloc", hipMalloc(&d, 4096));
    show("hipStreamCreateWithFlags", hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    show("hipStreamCreateWithFlags", hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    show("hipEventCreateWithFlags", hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    show("hipEventCreateWithFlags", hipEventCreateWithFlags(&fresh, hipEventDisableTiming));
    show("hipEventQuery(never recorded)", hipEventQuery(fresh));
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s1, 200000000LL, d);
    show("launch spin", hipSuccess);
    show("hipEventRecord(s1)", hipEventRecord(ev, s1));
    show("hipEventQuery(in flight)", hipEventQuery(ev));
    show("hipStreamWaitEvent(s2, ev)", hipStreamWaitEvent(s2, ev, 0));
    const hipError_t q = hipEventQuery(ev);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s2, 1000LL, d);
    show("query(in flight) then launch on s2", q);
    show("hipStreamSynchronize(s1)", hipStreamSynchronize(s1));
    show("hipEventQuery(done)", hipEventQuery(ev));
    show("hipDeviceSynchronize", hipDeviceSynchronize());
    return 0;
}
