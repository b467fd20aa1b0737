// Wave-dispatch rate probe (gfx950): how long does a grid of single-wave blocks
// that do (almost) nothing take, per grid size and block size?  Tells whether
// k_rootwalk's 65 536-wave grid-stride grid has a dispatch floor.
//   hipcc --offload-arch=gfx950 -O3 tools/dispatch_probe.hip -o tools/_dispatch_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int *sink, int n)
{
    if ((int)blockIdx.x >= n && threadIdx.x == 0) sink[0] = 1;   // never true: keeps the kernel
}

int main()
{
    int *sink;
    hipMalloc(&sink, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grids[] = {1024, 4096, 8192, 16384, 32768, 65536, 131072, 262144};
    const int blocks[] = {64, 256};
    printf("{\"rows\": [\n");
    bool first = true;
    for (int bs : blocks)
        for (int g : grids) {
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_empty, dim3(g), dim3(bs), 0, 0, sink, 1 << 30);
            hipDeviceSynchronize();
            hipEventRecord(a, 0);
            const int reps = 20;
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_empty, dim3(g), dim3(bs), 0, 0, sink, 1 << 30);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0.0f;
            hipEventElapsedTime(&ms, a, b);
            const double us = ms * 1e3 / reps;
            printf("%s{\"block\": %d, \"grid\": %d, \"waves\": %lld, \"us_per_launch\": %.2f, \"ns_per_wave\": %.3f}",
                   first ? "" : ",\n", bs, g, (long long)g * bs / 64, us, us * 1e3 / ((double)g * bs / 64));
            first = false;
        }
    printf("\n]}\n");
    return 0;
}
