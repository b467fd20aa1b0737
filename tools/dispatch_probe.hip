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

// the same with k_rootwalk's LDS per block (5 412 B)
__global__ void k_empty_lds(int *sink, int n)
{
    __shared__ int buf[1353];
    buf[threadIdx.x] = (int)blockIdx.x;
    __syncthreads();
    if ((int)blockIdx.x >= n && threadIdx.x == 0) sink[0] = buf[(threadIdx.x + 1) & 63];
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
    for (int lds = 0; lds < 2; ++lds)
    for (int bs : blocks)
        for (int g : grids) {
            if (lds && bs != 64) continue;
            auto K = lds ? k_empty_lds : k_empty;
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(K, dim3(g), dim3(bs), 0, 0, sink, 1 << 30);
            hipDeviceSynchronize();
            hipEventRecord(a, 0);
            const int reps = 20;
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(K, dim3(g), dim3(bs), 0, 0, sink, 1 << 30);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0.0f;
            hipEventElapsedTime(&ms, a, b);
            const double us = ms * 1e3 / reps;
            printf("%s{\"lds\": %d, \"block\": %d, \"grid\": %d, \"waves\": %lld, \"us_per_launch\": %.2f, \"ns_per_wave\": %.3f}",
                   first ? "" : ",\n", lds, bs, g, (long long)g * bs / 64, us, us * 1e3 / ((double)g * bs / 64));
            first = false;
        }
    printf("\n]}\n");
    return 0;
}
