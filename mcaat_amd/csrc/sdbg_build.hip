// sdbg_build.hip — canonical counts -> succinct-order de Bruijn graph resident in HBM.
//
// Replaces MEGAHIT's BOSS construction inside Read2SdbgS2::Run + SDBG::LoadFromFile
// (reference sdbg_build.cpp:183-187, main.cpp:522-530). Conventions: DESIGN.md
// "SDBG conventions" (edge ids in colex-label-then-W order, both orientations,
// mult = occ(e)+occ(rc e), palindromes 2*occ, saturating at 65535; no '$' dummies).
//
// Steps: expand each canonical edge to its two orientations (BOSS keys) -> radix sort
// (key, mult) -> radix directory over the top key bits -> per-edge adjacency words
// (first out-edge + W mask of the target node; first edge of the predecessor group +
// position mask) -> valid bitmap.
#include <hipcub/hipcub.hpp>

#include "internal.h"

namespace mcaat {

namespace {

constexpr int kBlock = 256;

__global__ void __launch_bounds__(kBlock) k_expand(const uint64_t *ckeys, const uint32_t *ccnt, uint64_t n, int k,
                                                   uint64_t *okeys, uint16_t *omult, unsigned long long *n_pal) {
    const int E = k + 1;
    const uint64_t sentinel = 1ULL << (2 * E);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t a = ckeys[i], b = lsb_rc(a, E);
        const uint64_t c = ccnt[i];
        if (a == b) {
            const uint64_t m = 2 * c;
            okeys[2 * i] = boss_key(a, k);
            omult[2 * i] = (uint16_t)(m > 65535 ? 65535 : m);
            okeys[2 * i + 1] = sentinel;
            omult[2 * i + 1] = 0;
            atomicAdd(n_pal, 1ull);
        } else {
            const uint16_t m = (uint16_t)(c > 65535 ? 65535 : c);
            okeys[2 * i] = boss_key(a, k);
            omult[2 * i] = m;
            okeys[2 * i + 1] = boss_key(b, k);
            omult[2 * i + 1] = m;
        }
    }
}

// dir[p] = first index whose key prefix (top B of 2E bits) >= p, p in [0, 2^B]
__global__ void __launch_bounds__(kBlock) k_dir(const uint64_t *key, uint64_t D, int shift, uint64_t nprefix,
                                                uint64_t *dir) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= nprefix; p += stride) {
        const uint64_t q = p << shift;
        uint64_t lo = 0, hi = D;
        if (p == nprefix) {
            lo = D;
        } else {
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (key[mid] < q) lo = mid + 1; else hi = mid;
            }
        }
        dir[p] = lo;
    }
}

__device__ __forceinline__ uint64_t lower_bound_dir(const uint64_t *key, const uint64_t *dir, int shift, uint64_t q) {
    const uint64_t p = q >> shift;
    uint64_t lo = dir[p], hi = dir[p + 1];
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (key[mid] < q) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(kBlock) k_adjacency(const uint64_t *key, uint64_t D, int k, const uint64_t *dir,
                                                      int shift, uint64_t *out_info, uint64_t *in_info) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t gmask = mask_bits(2 * (k - 1));
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < D; e += stride) {
        const uint64_t K = key[e];
        const uint64_t W = K & 3, R = K >> 2;
        // out: edges of node target(e) = label s[1..k-1]W
        const uint64_t Rt = (W << (2 * (k - 1))) | (R >> 2);
        uint64_t lo = lower_bound_dir(key, dir, shift, Rt << 2);
        unsigned m = 0;
        for (uint64_t i = lo; i < D && (key[i] >> 2) == Rt; ++i) m |= 1u << (key[i] & 3);
        out_info[e] = lo | ((uint64_t)m << kIdxBits);
        // in: group of labels x s[0..k-2], edges with W == s[k-1]
        const uint64_t c = (K >> (2 * k)) & 3;
        const uint64_t G = R & gmask;
        lo = lower_bound_dir(key, dir, shift, G << 4);
        unsigned pm = 0;
        int j = 0;
        for (uint64_t i = lo; i < D && (key[i] >> 4) == G && j < 16; ++i, ++j)
            if ((key[i] & 3) == c) pm |= 1u << j;
        in_info[e] = lo | ((uint64_t)pm << kIdxBits);
    }
}

__global__ void __launch_bounds__(kBlock) k_valid_init(uint64_t *valid, uint64_t D) {
    const uint64_t nw = (D + 63) / 64;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
        const uint64_t rem = D - w * 64;
        valid[w] = rem >= 64 ? ~0ULL : ((1ULL << rem) - 1);
    }
}

}  // namespace

void sdbg_build(mcaat_ctx *ctx, CountResult &c, int k, mcaat_graph *g) {
    hipStream_t st = ctx->stream;
    const int E = k + 1;
    const uint64_t n2 = 2 * c.n;
    g->k = k;
    DevBuf<unsigned long long> npal(1);
    HIP_OK(hipMemsetAsync(npal.p, 0, 8, st));
    DevBuf<uint64_t> ek(n2);
    DevBuf<uint16_t> em(n2);
    if (c.n) {
        hipLaunchKernelGGL(k_expand, dim3(grid_for(c.n, kBlock)), dim3(kBlock), 0, st, c.keys.p, c.counts.p, c.n, k,
                           ek.p, em.p, npal.p);
        LAUNCH_OK();
    }
    // release the counting table output before sorting
    c.keys.release();
    c.counts.release();
    unsigned long long n_pal = 0;
    HIP_OK(hipMemcpyAsync(&n_pal, npal.p, 8, hipMemcpyDeviceToHost, st));
    g->key.alloc(n2);
    g->mult.alloc(n2);
    if (n2) {
        size_t tmp = 0;
        HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, ek.p, g->key.p, em.p, g->mult.p, (size_t)n2, 0,
                                                  2 * E + 1, st));
        DevBuf<uint8_t> t(tmp);
        HIP_OK(hipcub::DeviceRadixSort::SortPairs(t.p, tmp, ek.p, g->key.p, em.p, g->mult.p, (size_t)n2, 0, 2 * E + 1,
                                                  st));
    }
    HIP_OK(hipStreamSynchronize(st));
    ek.release();
    em.release();
    g->D = n2 - n_pal;
    sdbg_finish(ctx, g);
}

// sorted unique (key, mult) in g -> directory, adjacency words, valid bitmap
void sdbg_finish(mcaat_ctx *ctx, mcaat_graph *g) {
    hipStream_t st = ctx->stream;
    const int k = g->k, E = k + 1;
    const uint64_t D = g->D;

    // radix directory: B top bits of the 2E-bit key, ~8-16 edges per bucket
    int lg = 0;
    while ((1ULL << (lg + 1)) <= (D ? D : 1)) ++lg;
    int B = lg - 3;
    if (B < 1) B = 1;
    if (B > 2 * E) B = 2 * E;
    if (B > 30) B = 30;
    const int shift = 2 * E - B;
    const uint64_t nprefix = 1ULL << B;
    DevBuf<uint64_t> dir(nprefix + 1);
    hipLaunchKernelGGL(k_dir, dim3(grid_for(nprefix + 1, kBlock)), dim3(kBlock), 0, st, g->key.p, D, shift, nprefix,
                       dir.p);
    LAUNCH_OK();
    g->out_info.alloc(D);
    g->in_info.alloc(D);
    if (D) {
        hipLaunchKernelGGL(k_adjacency, dim3(grid_for(D, kBlock)), dim3(kBlock), 0, st, g->key.p, D, k, dir.p, shift,
                           g->out_info.p, g->in_info.p);
        LAUNCH_OK();
    }
    g->valid.alloc((D + 63) / 64);
    hipLaunchKernelGGL(k_valid_init, dim3(grid_for((D + 63) / 64, kBlock)), dim3(kBlock), 0, st, g->valid.p, D);
    LAUNCH_OK();
    HIP_OK(hipStreamSynchronize(st));
}

}  // namespace mcaat
