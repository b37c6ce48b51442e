// Radix-sort pass-width experiment for the SDBG edge sort: 1.01e9 (u64 key < 2^57, u16)
// pairs, rocprim onesweep with 8/10/11/12 bits per pass. Prints ms per sort.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void fill(uint64_t *k, uint16_t *v, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9e3779b97f4a7c15ULL;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        k[i] = (z ^ (z >> 31)) >> 7;
        v[i] = (uint16_t)i;
    }
}

template <unsigned Bits, unsigned BS, unsigned IPT>
float run(uint64_t *k, uint64_t *k2, uint16_t *v, uint16_t *v2, size_t n) {
    using cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                           rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>,
                                                                               rocprim::kernel_config<BS, IPT>, Bits>>;
    size_t tmp = 0;
    CK(rocprim::radix_sort_pairs<cfg>(nullptr, tmp, k, k2, v, v2, n, 0, 57, 0));
    void *t;
    CK(hipMalloc(&t, tmp));
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
        hipEventRecord(a, 0);
        CK(rocprim::radix_sort_pairs<cfg>(t, tmp, k, k2, v, v2, n, 0, 57, 0));
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    hipFree(t);
    return best;
}

float run_default(uint64_t *k, uint64_t *k2, uint16_t *v, uint16_t *v2, size_t n) {
    size_t tmp = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tmp, k, k2, v, v2, n, 0, 57, 0));
    void *t; CK(hipMalloc(&t, tmp));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
        hipEventRecord(a, 0);
        CK(rocprim::radix_sort_pairs(t, tmp, k, k2, v, v2, n, 0, 57, 0));
        hipEventRecord(b, 0); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    hipFree(t);
    return best;
}

int main(int argc, char **argv) {
    size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1010000000ULL;
    uint64_t *k, *k2; uint16_t *v, *v2;
    CK(hipMalloc(&k, 8 * n)); CK(hipMalloc(&k2, 8 * n)); CK(hipMalloc(&v, 2 * n)); CK(hipMalloc(&v2, 2 * n));
    fill<<<4096, 256>>>(k, v, n);
    CK(hipDeviceSynchronize());
    printf("default    %.2f ms\n", run_default(k, k2, v, v2, n));
    printf("8b 256x16  %.2f ms\n", run<8, 256, 16>(k, k2, v, v2, n));
    printf("10b 256x16 %.2f ms\n", run<10, 256, 16>(k, k2, v, v2, n));
    printf("11b 256x16 %.2f ms\n", run<11, 256, 16>(k, k2, v, v2, n));
    printf("11b 512x16 %.2f ms\n", run<11, 512, 16>(k, k2, v, v2, n));
    printf("12b 512x16 %.2f ms\n", run<12, 512, 16>(k, k2, v, v2, n));
    return 0;
}
