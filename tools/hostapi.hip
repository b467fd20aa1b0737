// GPU box: host-side cost of the HIP calls the iteration loop makes (kernel
// launch, launch with start/stop events, event record, cross-stream wait).
//   hipcc --offload-arch=gfx950 -O3 tools/hostapi.hip -o tools/hostapi && tools/hostapi
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

struct Big { long long w[24]; };                 // a kernel-argument block of ~200 bytes

__global__ void k_empty(Big b, int *p) { if (b.w[0] == 12345 && p) p[threadIdx.x] = 1; }

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    hipStream_t s, s2;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t e, e0, e1;
    (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    Big b = {};
    const int N = 2000;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipStreamSynchronize(s);
        double t = now_us();
        for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, b, (int *)nullptr);
        const double launch = (now_us() - t) / N;
        (void)hipStreamSynchronize(s);
        t = now_us();
        for (int i = 0; i < N; ++i)
            hipExtLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, e0, e1, 0, b, (int *)nullptr);
        const double xlaunch = (now_us() - t) / N;
        (void)hipStreamSynchronize(s);
        t = now_us();
        for (int i = 0; i < N; ++i) (void)hipEventRecord(e, s);
        const double rec = (now_us() - t) / N;
        (void)hipStreamSynchronize(s);
        t = now_us();
        for (int i = 0; i < N; ++i) { (void)hipEventRecord(e, s); (void)hipStreamWaitEvent(s2, e, 0); }
        const double recwait = (now_us() - t) / N;
        (void)hipDeviceSynchronize();
        // device-side: back-to-back empty kernels, gap per kernel
        (void)hipEventRecord(e0, s);
        for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, b, (int *)nullptr);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("launch %.2f us, ext launch+events %.2f us, event record %.2f us, record+wait %.2f us | "
               "device time per empty 1024-block kernel %.2f us\n", launch, xlaunch, rec, recwait, ms * 1e3 / N);
    }
    return 0;
}
