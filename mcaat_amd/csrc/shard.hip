// shard.hip — the per-rank pieces of the multi-GPU build:
// local canonical counts -> BOSS-key histogram (for balanced owner ranges) -> oriented
// (BOSS key, partial count) pairs grouped by owner rank -> [caller's all-to-all over RCCL]
// -> owner-side sort + sum per key -> [caller's all-gather] -> graph from the globally
// sorted keys. Owner ranges are contiguous in BOSS order, so the ranks' reduced arrays
// concatenated in rank order are the single-GPU edge array (edge ids bit-identical).
#include <hipcub/hipcub.hpp>

#include "internal.h"

namespace mcaat {

namespace {

constexpr int kBlock = 256;
constexpr int kMaxOwners = 64;
constexpr uint32_t kTile = 65536;  // canonical entries per workgroup tile in the partition

// the one or two oriented edges of a canonical count: BOSS keys and partial counts
// (a palindrome is one oriented edge seen from both strands: 2*c)
__device__ __forceinline__ int oriented(uint64_t a, uint32_t c, int k, uint64_t *K, uint32_t *m) {
    const int E = k + 1;
    const uint64_t b = lsb_rc(a, E);
    K[0] = boss_key(a, k);
    if (a == b) {
        m[0] = 2 * c;
        return 1;
    }
    m[0] = m[1] = c;
    K[1] = boss_key(b, k);
    return 2;
}

__device__ __forceinline__ int owner_of(uint64_t K, const uint64_t *splits, int ns) {
    int o = 0;
    while (o < ns && splits[o] <= K) ++o;
    return o;
}

__global__ void __launch_bounds__(kBlock) k_boss_hist(const uint64_t *keys, const uint32_t *cnt, uint64_t n, int k,
                                                      int shift, int nbins, unsigned long long *hist) {
    extern __shared__ uint32_t lh[];
    for (int i = threadIdx.x; i < nbins; i += kBlock) lh[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uint64_t K[2];
        uint32_t m[2];
        const int no = oriented(keys[i], cnt[i], k, K, m);
        for (int j = 0; j < no; ++j) atomicAdd(&lh[K[j] >> shift], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nbins; i += kBlock)
        if (lh[i]) atomicAdd(&hist[i], (unsigned long long)lh[i]);
}

// per tile: count per owner in LDS, reserve one run per owner, write the tile's edges
__global__ void __launch_bounds__(kBlock) k_partition(const uint64_t *keys, const uint32_t *cnt, uint64_t n, int k,
                                                      const uint64_t *splits, int ns, unsigned long long *cursor,
                                                      uint64_t *okeys, uint32_t *ocnt, int count_only) {
    __shared__ uint32_t lc[kMaxOwners];
    __shared__ unsigned long long lbase[kMaxOwners];
    __shared__ uint64_t sp[kMaxOwners];
    const int no_owners = ns + 1;
    for (int i = threadIdx.x; i < ns; i += kBlock) sp[i] = splits[i];
    for (uint64_t t0 = (uint64_t)blockIdx.x * kTile; t0 < n; t0 += (uint64_t)gridDim.x * kTile) {
        const uint64_t t1 = t0 + kTile < n ? t0 + kTile : n;
        for (int i = threadIdx.x; i < no_owners; i += kBlock) lc[i] = 0;
        __syncthreads();
        for (uint64_t i = t0 + threadIdx.x; i < t1; i += kBlock) {
            uint64_t K[2];
            uint32_t m[2];
            const int no = oriented(keys[i], cnt[i], k, K, m);
            for (int j = 0; j < no; ++j) atomicAdd(&lc[owner_of(K[j], sp, ns)], 1u);
        }
        __syncthreads();
        if (count_only) {
            for (int i = threadIdx.x; i < no_owners; i += kBlock)
                if (lc[i]) atomicAdd(&cursor[i], (unsigned long long)lc[i]);
            __syncthreads();
            continue;
        }
        for (int i = threadIdx.x; i < no_owners; i += kBlock) {
            lbase[i] = lc[i] ? atomicAdd(&cursor[i], (unsigned long long)lc[i]) : 0;
            lc[i] = 0;
        }
        __syncthreads();
        for (uint64_t i = t0 + threadIdx.x; i < t1; i += kBlock) {
            uint64_t K[2];
            uint32_t m[2];
            const int no = oriented(keys[i], cnt[i], k, K, m);
            for (int j = 0; j < no; ++j) {
                const int o = owner_of(K[j], sp, ns);
                const uint64_t pos = lbase[o] + atomicAdd(&lc[o], 1u);
                okeys[pos] = K[j];
                ocnt[pos] = m[j];
            }
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(kBlock) k_saturate(const uint32_t *agg, uint64_t n, uint16_t *mult) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        mult[i] = (uint16_t)(agg[i] > 65535u ? 65535u : agg[i]);
}

// ---- canonical-pair exchange (the native multi-GPU build, dist.hip) ----
// A canonical edge goes once, with its partial count saturated to 16 bits, to the owner of
// the smaller of its two BOSS keys; that owner sums it, expands it to its oriented edges and
// routes each to the owner of its range (usually another rank). At high coverage every
// rank's reads hold nearly every edge, so this halves both the first exchange and the
// owner's sort against sending both orientations. Saturating a partial count changes no
// multiplicity: any partial at 65535 already saturates the total (a palindrome's 2x too).
__device__ __forceinline__ uint64_t min_boss(uint64_t a, int k) {
    const uint64_t b = lsb_rc(a, k + 1);
    const uint64_t Ka = boss_key(a, k), Kb = boss_key(b, k);
    return Ka < Kb ? Ka : Kb;
}

__global__ void __launch_bounds__(kBlock) k_partition_canon(const uint64_t *keys, const uint32_t *cnt, uint64_t n,
                                                            int k, const uint64_t *splits, int ns,
                                                            unsigned long long *cursor, uint64_t *okeys, uint16_t *ocnt,
                                                            int count_only) {
    __shared__ uint32_t lc[kMaxOwners];
    __shared__ unsigned long long lbase[kMaxOwners];
    __shared__ uint64_t sp[kMaxOwners];
    const int no_owners = ns + 1;
    for (int i = threadIdx.x; i < ns; i += kBlock) sp[i] = splits[i];
    for (uint64_t t0 = (uint64_t)blockIdx.x * kTile; t0 < n; t0 += (uint64_t)gridDim.x * kTile) {
        const uint64_t t1 = t0 + kTile < n ? t0 + kTile : n;
        for (int i = threadIdx.x; i < no_owners; i += kBlock) lc[i] = 0;
        __syncthreads();
        for (uint64_t i = t0 + threadIdx.x; i < t1; i += kBlock) atomicAdd(&lc[owner_of(min_boss(keys[i], k), sp, ns)], 1u);
        __syncthreads();
        if (count_only) {
            for (int i = threadIdx.x; i < no_owners; i += kBlock)
                if (lc[i]) atomicAdd(&cursor[i], (unsigned long long)lc[i]);
            __syncthreads();
            continue;
        }
        for (int i = threadIdx.x; i < no_owners; i += kBlock) {
            lbase[i] = lc[i] ? atomicAdd(&cursor[i], (unsigned long long)lc[i]) : 0;
            lc[i] = 0;
        }
        __syncthreads();
        for (uint64_t i = t0 + threadIdx.x; i < t1; i += kBlock) {
            const uint64_t a = keys[i];
            const int o = owner_of(min_boss(a, k), sp, ns);
            const uint64_t pos = lbase[o] + atomicAdd(&lc[o], 1u);
            okeys[pos] = a;
            ocnt[pos] = (uint16_t)(cnt[i] > 65535u ? 65535u : cnt[i]);
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(kBlock) k_widen16(const uint16_t *in, uint64_t n, uint32_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

// the summed canonical edges -> their oriented edges (multiplicity saturated), owner-major
__global__ void __launch_bounds__(kBlock) k_route_oriented(const uint64_t *keys, const uint32_t *tot, uint64_t n, int k,
                                                           const uint64_t *splits, int ns, unsigned long long *cursor,
                                                           uint64_t *okeys, uint16_t *omult, int count_only) {
    __shared__ uint32_t lc[kMaxOwners];
    __shared__ unsigned long long lbase[kMaxOwners];
    __shared__ uint64_t sp[kMaxOwners];
    const int no_owners = ns + 1;
    for (int i = threadIdx.x; i < ns; i += kBlock) sp[i] = splits[i];
    for (uint64_t t0 = (uint64_t)blockIdx.x * kTile; t0 < n; t0 += (uint64_t)gridDim.x * kTile) {
        const uint64_t t1 = t0 + kTile < n ? t0 + kTile : n;
        for (int i = threadIdx.x; i < no_owners; i += kBlock) lc[i] = 0;
        __syncthreads();
        for (uint64_t i = t0 + threadIdx.x; i < t1; i += kBlock) {
            uint64_t K[2];
            uint32_t m[2];
            const int no = oriented(keys[i], tot[i], k, K, m);
            for (int j = 0; j < no; ++j) atomicAdd(&lc[owner_of(K[j], sp, ns)], 1u);
        }
        __syncthreads();
        if (count_only) {
            for (int i = threadIdx.x; i < no_owners; i += kBlock)
                if (lc[i]) atomicAdd(&cursor[i], (unsigned long long)lc[i]);
            __syncthreads();
            continue;
        }
        for (int i = threadIdx.x; i < no_owners; i += kBlock) {
            lbase[i] = lc[i] ? atomicAdd(&cursor[i], (unsigned long long)lc[i]) : 0;
            lc[i] = 0;
        }
        __syncthreads();
        for (uint64_t i = t0 + threadIdx.x; i < t1; i += kBlock) {
            uint64_t K[2];
            uint32_t m[2];
            const int no = oriented(keys[i], tot[i], k, K, m);
            for (int j = 0; j < no; ++j) {
                const int o = owner_of(K[j], sp, ns);
                const uint64_t pos = lbase[o] + atomicAdd(&lc[o], 1u);
                okeys[pos] = K[j];
                omult[pos] = (uint16_t)(m[j] > 65535u ? 65535u : m[j]);
            }
        }
        __syncthreads();
    }
}

// owner-major two-pass partition driver shared by the canonical and the oriented routes
template <class Launch>
uint64_t owner_major(mcaat_ctx *ctx, uint64_t n, int n_owners, const uint64_t *splits_host, uint64_t *sizes_host,
                     uint64_t cap, Launch launch) {
    hipStream_t st = ctx->stream;
    const int ns = n_owners - 1;
    DevBuf<uint64_t> sp(ns > 0 ? ns : 1);
    DevBuf<unsigned long long> cur(n_owners);
    if (ns > 0) HIP_OK(hipMemcpyAsync(sp.p, splits_host, 8 * (uint64_t)ns, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(cur.p, 0, cur.bytes(), st));
    const unsigned grid = grid_for(n, kTile, (unsigned)ctx->n_cu * 8);
    if (n) {
        launch(grid, sp.p, ns, cur.p, 1);
        LAUNCH_OK();
    }
    std::vector<unsigned long long> h(n_owners);
    HIP_OK(hipMemcpyAsync(h.data(), cur.p, 8 * (uint64_t)n_owners, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    uint64_t total = 0;
    std::vector<unsigned long long> base(n_owners);
    for (int o = 0; o < n_owners; ++o) {
        base[o] = total;
        sizes_host[o] = h[o];
        total += h[o];
    }
    if (total > cap) throw Error(MCAAT_E_CAPACITY, "partition: output buffers smaller than the routed edges");
    if (!total) return 0;
    HIP_OK(hipMemcpyAsync(cur.p, base.data(), 8 * (uint64_t)n_owners, hipMemcpyHostToDevice, st));
    launch(grid, sp.p, ns, cur.p, 0);
    LAUNCH_OK();
    HIP_OK(hipStreamSynchronize(st));
    return total;
}

}  // namespace

void counts_histogram(mcaat_ctx *ctx, const CountResult &c, int k, int bits, uint64_t *hist_host) {
    hipStream_t st = ctx->stream;
    const int shift = 2 * (k + 1) - bits;
    const int nbins = 1 << bits;
    DevBuf<unsigned long long> h(nbins);
    HIP_OK(hipMemsetAsync(h.p, 0, h.bytes(), st));
    if (c.n) {
        hipLaunchKernelGGL(k_boss_hist, dim3(grid_for(c.n, kBlock, (unsigned)ctx->n_cu * 8)), dim3(kBlock),
                           4 * nbins, st, c.keys.p, c.counts.p, c.n, k, shift, nbins, h.p);
        LAUNCH_OK();
    }
    HIP_OK(hipMemcpyAsync(hist_host, h.p, 8 * (uint64_t)nbins, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
}

void counts_partition(mcaat_ctx *ctx, const CountResult &c, int k, int n_owners, const uint64_t *splits_host,
                      uint64_t *sizes_host, uint64_t *okeys, uint32_t *ocnt, uint64_t cap) {
    hipStream_t st = ctx->stream;
    const int ns = n_owners - 1;
    DevBuf<uint64_t> sp(ns > 0 ? ns : 1);
    DevBuf<unsigned long long> cur(n_owners);
    if (ns > 0) HIP_OK(hipMemcpyAsync(sp.p, splits_host, 8 * (uint64_t)ns, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(cur.p, 0, cur.bytes(), st));
    const unsigned grid = grid_for(c.n, kTile, (unsigned)ctx->n_cu * 8);
    if (c.n) {
        hipLaunchKernelGGL(k_partition, dim3(grid), dim3(kBlock), 0, st, c.keys.p, c.counts.p, c.n, k, sp.p, ns, cur.p,
                           (uint64_t *)nullptr, (uint32_t *)nullptr, 1);
        LAUNCH_OK();
    }
    std::vector<unsigned long long> h(n_owners);
    HIP_OK(hipMemcpyAsync(h.data(), cur.p, 8 * (uint64_t)n_owners, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    uint64_t total = 0;
    std::vector<unsigned long long> base(n_owners);
    for (int o = 0; o < n_owners; ++o) {
        base[o] = total;
        sizes_host[o] = h[o];
        total += h[o];
    }
    if (total > cap) throw Error(MCAAT_E_CAPACITY, "partition: output buffers smaller than the oriented edges");
    if (!total) return;
    HIP_OK(hipMemcpyAsync(cur.p, base.data(), 8 * (uint64_t)n_owners, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_partition, dim3(grid), dim3(kBlock), 0, st, c.keys.p, c.counts.p, c.n, k, sp.p, ns, cur.p,
                       okeys, ocnt, 0);
    LAUNCH_OK();
    HIP_OK(hipStreamSynchronize(st));
}

uint64_t edges_reduce(mcaat_ctx *ctx, int k, const uint64_t *keys, const uint32_t *cnt, uint64_t n, uint64_t *keys_out,
                      uint16_t *mult_out) {
    if (!n) return 0;
    hipStream_t st = ctx->stream;
    const int E = k + 1;
    DevBuf<uint64_t> sk(n);
    DevBuf<uint32_t> sc(n), agg(n);
    DevBuf<unsigned long long> nrun(1);
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, keys, sk.p, cnt, sc.p, (size_t)n, 0, 2 * E, st));
    {
        DevBuf<uint8_t> t(tmp);
        HIP_OK(hipcub::DeviceRadixSort::SortPairs(t.p, tmp, keys, sk.p, cnt, sc.p, (size_t)n, 0, 2 * E, st));
    }
    tmp = 0;
    HIP_OK(hipcub::DeviceReduce::ReduceByKey(nullptr, tmp, sk.p, keys_out, sc.p, agg.p, nrun.p, hipcub::Sum(),
                                             (size_t)n, st));
    {
        DevBuf<uint8_t> t(tmp);
        HIP_OK(hipcub::DeviceReduce::ReduceByKey(t.p, tmp, sk.p, keys_out, sc.p, agg.p, nrun.p, hipcub::Sum(),
                                                 (size_t)n, st));
    }
    unsigned long long u = 0;
    HIP_OK(hipMemcpyAsync(&u, nrun.p, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    hipLaunchKernelGGL(k_saturate, dim3(grid_for(u, kBlock)), dim3(kBlock), 0, st, agg.p, (uint64_t)u, mult_out);
    LAUNCH_OK();
    HIP_OK(hipStreamSynchronize(st));
    return u;
}

uint64_t counts_partition_canon(mcaat_ctx *ctx, const CountResult &c, int k, int n_owners, const uint64_t *splits_host,
                                uint64_t *sizes_host, uint64_t *okeys, uint16_t *ocnt, uint64_t cap) {
    hipStream_t st = ctx->stream;
    return owner_major(ctx, c.n, n_owners, splits_host, sizes_host, cap,
                       [&](unsigned grid, const uint64_t *sp, int ns, unsigned long long *cur, int count_only) {
                           hipLaunchKernelGGL(k_partition_canon, dim3(grid), dim3(kBlock), 0, st, c.keys.p, c.counts.p,
                                              c.n, k, sp, ns, cur, okeys, ocnt, count_only);
                       });
}

uint64_t canon_reduce(mcaat_ctx *ctx, int k, const uint64_t *keys, const uint16_t *cnt16, uint64_t n, uint64_t *keys_out,
                      uint32_t *tot_out) {
    if (!n) return 0;
    hipStream_t st = ctx->stream;
    const int E = k + 1;
    DevBuf<uint32_t> cnt(n);
    hipLaunchKernelGGL(k_widen16, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, cnt16, n, cnt.p);
    LAUNCH_OK();
    DevBuf<uint64_t> sk(n);
    DevBuf<uint32_t> sc(n);
    DevBuf<unsigned long long> nrun(1);
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, keys, sk.p, cnt.p, sc.p, (size_t)n, 0, 2 * E, st));
    {
        DevBuf<uint8_t> t(tmp);
        HIP_OK(hipcub::DeviceRadixSort::SortPairs(t.p, tmp, keys, sk.p, cnt.p, sc.p, (size_t)n, 0, 2 * E, st));
    }
    cnt.release();
    tmp = 0;
    HIP_OK(hipcub::DeviceReduce::ReduceByKey(nullptr, tmp, sk.p, keys_out, sc.p, tot_out, nrun.p, hipcub::Sum(),
                                             (size_t)n, st));
    {
        DevBuf<uint8_t> t(tmp);
        HIP_OK(hipcub::DeviceReduce::ReduceByKey(t.p, tmp, sk.p, keys_out, sc.p, tot_out, nrun.p, hipcub::Sum(),
                                                 (size_t)n, st));
    }
    unsigned long long u = 0;
    HIP_OK(hipMemcpyAsync(&u, nrun.p, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    return u;
}

uint64_t route_oriented(mcaat_ctx *ctx, int k, const uint64_t *keys, const uint32_t *tot, uint64_t n, int n_owners,
                        const uint64_t *splits_host, uint64_t *sizes_host, uint64_t *okeys, uint16_t *omult, uint64_t cap) {
    hipStream_t st = ctx->stream;
    return owner_major(ctx, n, n_owners, splits_host, sizes_host, cap,
                       [&](unsigned grid, const uint64_t *sp, int ns, unsigned long long *cur, int count_only) {
                           hipLaunchKernelGGL(k_route_oriented, dim3(grid), dim3(kBlock), 0, st, keys, tot, n, k, sp,
                                              ns, cur, okeys, omult, count_only);
                       });
}

void sort_oriented(mcaat_ctx *ctx, int k, const uint64_t *keys, const uint16_t *mult, uint64_t n, uint64_t *keys_out,
                   uint16_t *mult_out) {
    if (!n) return;
    hipStream_t st = ctx->stream;
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, keys, keys_out, mult, mult_out, (size_t)n, 0, 2 * (k + 1), st));
    DevBuf<uint8_t> t(tmp);
    HIP_OK(hipcub::DeviceRadixSort::SortPairs(t.p, tmp, keys, keys_out, mult, mult_out, (size_t)n, 0, 2 * (k + 1), st));
    HIP_OK(hipStreamSynchronize(st));
}

void graph_from_sorted(mcaat_ctx *ctx, int k, const uint64_t *keys, const uint16_t *mult, uint64_t D, mcaat_graph *g) {
    hipStream_t st = ctx->stream;
    g->k = k;
    g->D = D;
    g->key.alloc(D ? D : 1);
    g->mult.alloc(mcaat_graph::mult_entries(D));
    if (D) {
        HIP_OK(hipMemcpyAsync(g->key.p, keys, 8 * D, hipMemcpyDeviceToDevice, st));
        HIP_OK(hipMemcpyAsync(g->mult.p, mult, 2 * D, hipMemcpyDeviceToDevice, st));
    }
    sdbg_finish(ctx, g);
}

void preload_shard() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, (const void *)k_boss_hist);
}

}  // namespace mcaat
