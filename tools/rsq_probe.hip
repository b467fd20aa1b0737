// Probe: are gfx950's v_rsq_f32 / v_sqrt_f32 correctly rounded?  (The reference's
// OpenCL normalize() / length() from ROCm's device library use them.)  Writes
// the raw results for every float in [1, 4) (2^24 inputs; other binades scale by
// exact powers of 4) to the file given as argv[1]: rsq[2^24], sqrt[2^24] (uint32).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k_probe(uint32_t *rsq, uint32_t *sq, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = __uint_as_float(0x3f800000u + i);
    rsq[i] = __float_as_uint(__builtin_amdgcn_rsqf(x));
    sq[i] = __float_as_uint(__builtin_amdgcn_sqrtf(x));
}

int main(int argc, char **argv)
{
    const uint32_t n = 1u << 24;
    uint32_t *d = nullptr;
    if (hipMalloc(&d, (size_t)2 * n * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_probe, dim3(n / 256), dim3(256), 0, 0, d, d + n, n);
    std::vector<uint32_t> h((size_t)2 * n);
    if (hipMemcpy(h.data(), d, (size_t)2 * n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    FILE *f = fopen(argc > 1 ? argv[1] : "rsq_probe.bin", "wb");
    if (!f) return 3;
    fwrite(h.data(), 4, h.size(), f);
    fclose(f);
    hipFree(d);
    printf("ok %u\n", n);
    return 0;
}
