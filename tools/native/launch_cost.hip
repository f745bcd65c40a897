// Host cost of the HIP calls the scan loop issues per keyframe (kernel launch, event record, stream wait), measured
// back to back on one stream without synchronisation.  Build: hipcc --offload-arch=gfx950 -O2 launch_cost.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty(int* p, int n) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0 && n < 0) p[0] = n;
}

int main() {
    hipStream_t s, s2;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    int* d = nullptr;
    hipMalloc(&d, 64);
    const int N = 20000;
    for (int rep = 0; rep < 3; ++rep) {
        hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(128), dim3(256), 0, s, d, i);
        auto t1 = std::chrono::steady_clock::now();
        hipStreamSynchronize(s);
        auto t2 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; ++i) hipEventRecord(ev, s);
        auto t3 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; ++i) hipStreamWaitEvent(s2, ev, 0);
        auto t4 = std::chrono::steady_clock::now();
        hipDeviceSynchronize();
        auto t5 = std::chrono::steady_clock::now();
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        std::printf("launch %.2f us (host issue), %.2f us/kernel (GPU drain incl.), eventRecord %.2f us, streamWaitEvent %.2f us\n",
                    us(t0, t1) / N, us(t0, t2) / N, us(t2, t3) / N, us(t3, t4) / N);
    }
    return 0;
}
