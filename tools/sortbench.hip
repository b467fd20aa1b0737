// GPU box: rocPRIM onesweep configurations on the coherence sort's shape (1 Mi
// (key, index) pairs, 16 key bits), hipEvent timing of the whole radix_sort_pairs
// call (its fills, histogram and digit passes).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sortbench.hip -o tools/sortbench && tools/sortbench [n]
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <class Cfg>
static void run(const char *name, size_t n, const unsigned *kin0, const int *vin0, hipStream_t s)
{
    unsigned *kin, *kout;
    int *vin, *vout;
    CK(hipMalloc(&kin, n * 4)); CK(hipMalloc(&kout, n * 4)); CK(hipMalloc(&vin, n * 4)); CK(hipMalloc(&vout, n * 4));
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, kin, kout, vin, vout, n, 0, 16, s));
    void *tmp;
    CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e9f, sum = 0.0f;
    const int reps = 30;
    for (int r = 0; r < reps + 3; ++r) {
        CK(hipMemcpyAsync(kin, kin0, n * 4, hipMemcpyDeviceToDevice, s));
        CK(hipMemcpyAsync(vin, vin0, n * 4, hipMemcpyDeviceToDevice, s));
        CK(hipEventRecord(a, s));
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, kin, kout, vin, vout, n, 0, 16, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 3) { best = ms < best ? ms : best; sum += ms; }
    }
    // sortedness check
    std::vector<unsigned> h(n);
    CK(hipMemcpy(h.data(), kout, n * 4, hipMemcpyDeviceToHost));
    bool ok = true;
    for (size_t i = 1; i < n; ++i) ok = ok && h[i - 1] <= h[i];
    printf("%-44s best %7.1f us  mean %7.1f us  %s\n", name, best * 1e3f, sum / reps * 1e3f, ok ? "sorted" : "NOT SORTED");
    CK(hipFree(kin)); CK(hipFree(kout)); CK(hipFree(vin)); CK(hipFree(vout)); CK(hipFree(tmp));
}

using namespace rocprim;
template <unsigned B, unsigned I, unsigned HB, unsigned HI, unsigned R>
using OS = radix_sort_config<default_config, default_config,
                             radix_sort_onesweep_config<kernel_config<HB, HI>, kernel_config<B, I>, R>, 0>;

int main(int argc, char **argv)
{
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1u << 20);
    std::vector<unsigned> hk(n);
    std::vector<int> hv(n);
    unsigned x = 12345u;
    for (size_t i = 0; i < n; ++i) { x = x * 1664525u + 1013904223u; hk[i] = x >> 16; hv[i] = (int)i; }
    unsigned *dk; int *dv;
    CK(hipMalloc(&dk, n * 4)); CK(hipMalloc(&dv, n * 4));
    CK(hipMemcpy(dk, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, hv.data(), n * 4, hipMemcpyHostToDevice));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    printf("n = %zu pairs, 16 key bits\n", n);
    run<radix_sort_config<default_config, default_config, default_config, 0>>("default onesweep (LPC RaySortCfg16)", n, dk, dv, s);
    run<OS<256, 12, 256, 12, 8>>("onesweep 256x12, 8 bits", n, dk, dv, s);
    run<OS<256, 16, 256, 16, 8>>("onesweep 256x16, 8 bits", n, dk, dv, s);
    run<OS<256, 24, 256, 24, 8>>("onesweep 256x24, 8 bits", n, dk, dv, s);
    run<OS<128, 16, 128, 16, 8>>("onesweep 128x16, 8 bits", n, dk, dv, s);
    run<OS<256, 12, 256, 12, 4>>("onesweep 256x12, 4 bits", n, dk, dv, s);
    run<default_config>("default_config (merge sort below 1 Mi)", n, dk, dv, s);
    return 0;
}
