// membench.hip — HBM write/read rate by access granularity on one MI355X (tools only, not the
// product): every 16-B lane store/load goes to a chunk of C bytes at a pseudo-random
// chunk-aligned position of an 8-GiB buffer (odd-multiplier permutation of the chunk index),
// C = 64 .. 4096, plus the sequential case. Tells what the scatter kernels (pass A flush, pass B,
// MSD levels 1/2) can expect from 64-B line writes against longer runs.
//   hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o tools/membench && tools/membench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

// lanes of a wave cover consecutive 16-B pieces; piece p belongs to chunk p / (C/16)
template <bool WRITE>
__global__ void __launch_bounds__(256) k_chunks(uint4 *buf, uint64_t n_pieces, uint32_t lg_per, uint64_t chunk_mask,
                                                int seq, unsigned long long *sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_pieces; p += stride) {
        const uint64_t chunk = p >> lg_per, within = p & ((1ull << lg_per) - 1);
        const uint64_t dst = seq ? chunk : ((chunk * 0x9E3779B97F4A7C15ull) & chunk_mask);
        uint4 *q = buf + (dst << lg_per) + within;
        if (WRITE) {
            *q = make_uint4((uint32_t)p, 1, 2, 3);
        } else {
            const uint4 v = *q;
            acc ^= v.x ^ v.w;
        }
    }
    if (!WRITE && acc == 0x12345678u) atomicAdd(sink, 1ull);
}

int main() {
    const uint64_t bytes = 8ull << 30, n_pieces = bytes / 16;
    uint4 *buf;
    unsigned long long *sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(buf, 0, bytes));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned grid = (unsigned)ncu * 32;
    printf("%-6s %-10s %10s %10s\n", "op", "chunk", "GB/s", "ms");
    for (int w = 1; w >= 0; --w)
        for (int c = 0; c <= 7; ++c) {
            const int seq = c == 7;
            const uint32_t lg_per = seq ? 2 : (uint32_t)c + 2;  // 16-B pieces per chunk: 4 .. 256
            const uint64_t chunk_mask = (n_pieces >> lg_per) - 1;
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipEventRecord(a));
                if (w)
                    hipLaunchKernelGGL(k_chunks<true>, dim3(grid), dim3(256), 0, 0, buf, n_pieces, lg_per, chunk_mask, seq, sink);
                else
                    hipLaunchKernelGGL(k_chunks<false>, dim3(grid), dim3(256), 0, 0, buf, n_pieces, lg_per, chunk_mask, seq, sink);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep && ms < best) best = ms;
            }
            char name[32];
            if (seq) snprintf(name, sizeof name, "seq");
            else snprintf(name, sizeof name, "%u B", 16u << lg_per);
            printf("%-6s %-10s %10.1f %10.3f\n", w ? "write" : "read", name, bytes / 1e6 / best, best);
        }
    return 0;
}
