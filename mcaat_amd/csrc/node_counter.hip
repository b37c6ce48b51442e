// node_counter.hip — exact canonical (k+1)-mer (edge) multiplicity counting on gfx950.
//
// Replaces the counting inside MEGAHIT Read2SdbgS2::Run (reference sdbg_build.cpp:171-187,
// "-m 1": every edge kept). Layout and roofline: DESIGN.md §node_counter.
//
// v1 design: one open-addressing table in HBM (keys u64 + counts u32, linear probing).
// Each lane owns one (k+1)-mer position; the window is a funnel shift of two packed
// words (coalesced: a wave reads ~40 consecutive bytes per 64 k-mers of a read).
// Existing keys cost one load + one atomic add; new keys one CAS. The table is sized
// from the occurrence count and regrown (x4) if the load factor passes 0.7.
#include <hipcub/hipcub.hpp>

#include "internal.h"

namespace mcaat {

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kMaxProbe = 1u << 14;

// one 16-byte slot: key+1 (0 = empty, so a plain memset clears the table) and count,
// in the same cache line so a hit costs one line
struct __attribute__((aligned(16))) Slot {
    unsigned long long key1;
    unsigned int cnt;
    unsigned int pad;
};

__device__ __forceinline__ void table_insert(uint64_t key, Slot *tab, uint64_t mask, unsigned long long *n_new,
                                             int *overflow) {
    const unsigned long long k1 = key + 1;
    uint64_t slot = mix64(key) & mask;
    for (uint32_t probe = 0; probe < kMaxProbe; ++probe) {
        unsigned long long cur = __hip_atomic_load(&tab[slot].key1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == 0) {
            cur = atomicCAS(&tab[slot].key1, 0ull, k1);
            if (cur == 0) {
                atomicAdd(&tab[slot].cnt, 1u);
                atomicAdd(n_new, 1ull);
                return;
            }
        }
        if (cur == k1) {
            atomicAdd(&tab[slot].cnt, 1u);
            return;
        }
        slot = (slot + 1) & mask;
    }
    atomicExch(overflow, 1);
}

// fixed-length reads: thread i -> (read i / npos, position i % npos)
__global__ void __launch_bounds__(kBlock) k_count_fixed(const uint64_t *__restrict__ packed, uint64_t n_reads,
                                                        uint64_t L, int E, Slot *tab, uint64_t mask,
                                                        unsigned long long *n_new, int *overflow) {
    const uint64_t npos = L - E + 1;
    const uint64_t total = n_reads * npos;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const uint64_t r = i / npos, p = i - r * npos;
        const uint64_t lsb = window_at(packed, r * L + p, E);
        const uint64_t rc = lsb_rc(lsb, E);
        table_insert(lsb < rc ? lsb : rc, tab, mask, n_new, overflow);
    }
}

// variable-length reads: one wave per read, lanes stride over positions
__global__ void __launch_bounds__(kBlock) k_count_var(const uint64_t *__restrict__ packed,
                                                      const uint64_t *__restrict__ offsets, uint64_t n_reads, int E,
                                                      Slot *tab, uint64_t mask, unsigned long long *n_new,
                                                      int *overflow) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t r = wave; r < n_reads; r += nwaves) {
        const uint64_t a = offsets[r], b = offsets[r + 1];
        if (b - a < (uint64_t)E) continue;
        const uint64_t npos = b - a - E + 1;
        for (uint64_t p = lane; p < npos; p += 64) {
            const uint64_t lsb = window_at(packed, a + p, E);
            const uint64_t rc = lsb_rc(lsb, E);
            table_insert(lsb < rc ? lsb : rc, tab, mask, n_new, overflow);
        }
    }
}

struct Occupied {
    __device__ __forceinline__ bool operator()(const Slot &s) const { return s.key1 != 0; }
};

__global__ void __launch_bounds__(kBlock) k_split(const Slot *in, uint64_t n, uint64_t *keys, uint32_t *cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const Slot s = in[i];
        keys[i] = s.key1 - 1;
        cnt[i] = s.cnt;
    }
}

}  // namespace

void node_counter(mcaat_ctx *ctx, const mcaat_reads *r, int k, CountResult &out) {
    const int E = k + 1;
    hipStream_t st = ctx->stream;
    uint64_t n_occ = 0;
    if (r->fixed_len) {
        n_occ = r->fixed_len >= (uint64_t)E ? r->n_reads * (r->fixed_len - E + 1) : 0;
    } else {
        std::vector<uint64_t> off(r->n_reads + 1);
        HIP_OK(hipMemcpyAsync(off.data(), r->offsets.p, 8 * (r->n_reads + 1), hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        for (uint64_t i = 0; i < r->n_reads; ++i)
            if (off[i + 1] - off[i] >= (uint64_t)E) n_occ += off[i + 1] - off[i] - E + 1;
    }
    uint64_t cap = next_pow2(n_occ / 8 + 1);
    if (cap < (1u << 16)) cap = 1u << 16;
    if (cap > (1ull << 31)) cap = 1ull << 31;

    DevBuf<unsigned long long> dcnt(2);
    DevBuf<int> dover(1);
    for (;;) {
        DevBuf<Slot> tab(cap);
        HIP_OK(hipMemsetAsync(tab.p, 0, tab.bytes(), st));
        HIP_OK(hipMemsetAsync(dcnt.p, 0, dcnt.bytes(), st));
        HIP_OK(hipMemsetAsync(dover.p, 0, dover.bytes(), st));
        {
            // algorithmic bytes per launch: 2-bit reads once + 16 B per occurrence
            KernelTimer kt(ctx, "node_counter", 0.25 * (double)r->n_bases + 16.0 * (double)n_occ);
            if (r->fixed_len) {
                hipLaunchKernelGGL(k_count_fixed, dim3(grid_for(n_occ, kBlock, 256 * 64)), dim3(kBlock), 0, st,
                                   r->packed.p, r->n_reads, r->fixed_len, E, tab.p, cap - 1, dcnt.p, dover.p);
            } else {
                hipLaunchKernelGGL(k_count_var, dim3(grid_for(r->n_reads * 64, kBlock, 256 * 64)), dim3(kBlock), 0,
                                   st, r->packed.p, r->offsets.p, r->n_reads, E, tab.p, cap - 1, dcnt.p, dover.p);
            }
            LAUNCH_OK();
            kt.stop();
        }
        unsigned long long n_new = 0;
        int over = 0;
        HIP_OK(hipMemcpyAsync(&n_new, dcnt.p, 8, hipMemcpyDeviceToHost, st));
        HIP_OK(hipMemcpyAsync(&over, dover.p, 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        if (over || n_new > cap / 10 * 7) {
            if (cap >= (1ull << 34)) throw Error(MCAAT_E_CAPACITY, "node_counter: hash table cannot grow further");
            cap <<= 2;
            continue;
        }
        DevBuf<Slot> packed_slots(n_new);
        size_t tmp = 0;
        HIP_OK(hipcub::DeviceSelect::If(nullptr, tmp, tab.p, packed_slots.p, dcnt.p, (size_t)cap, Occupied(), st));
        {
            DevBuf<uint8_t> t(tmp);
            HIP_OK(hipcub::DeviceSelect::If(t.p, tmp, tab.p, packed_slots.p, dcnt.p, (size_t)cap, Occupied(), st));
        }
        tab.release();
        out.n = n_new;
        out.keys.alloc(n_new);
        out.counts.alloc(n_new);
        hipLaunchKernelGGL(k_split, dim3(grid_for(n_new, kBlock)), dim3(kBlock), 0, st, packed_slots.p, n_new,
                           out.keys.p, out.counts.p);
        LAUNCH_OK();
        HIP_OK(hipStreamSynchronize(st));
        break;
    }
}

void sort_counts(mcaat_ctx *ctx, CountResult &c, int k) {
    if (c.n < 2) return;
    const int E = k + 1;
    DevBuf<uint64_t> k2(c.n);
    DevBuf<uint32_t> c2(c.n);
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, c.keys.p, k2.p, c.counts.p, c2.p, (size_t)c.n, 0, 2 * E,
                                              ctx->stream));
    DevBuf<uint8_t> t(tmp);
    HIP_OK(hipcub::DeviceRadixSort::SortPairs(t.p, tmp, c.keys.p, k2.p, c.counts.p, c2.p, (size_t)c.n, 0, 2 * E,
                                              ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    c.keys = std::move(k2);
    c.counts = std::move(c2);
}

}  // namespace mcaat
