// shard_cf.hip — the per-shard CycleFinder of a multi-GPU run (round 5; BASELINE north_star:
// "cycle_finder then runs per-shard with a boundary-edge exchange").
//
// The sharded build leaves every rank its BOSS-key range of the edges ([id_lo, id_lo + D_local)
// of the global ids; mcaat_graph::sharded) instead of all-gathering the whole graph. Everything
// D-wide then runs on the rank's own range, and what crosses a range boundary is a message:
//   adjacency (sdbg_finish_sharded): out_info / in_info of every local edge by one request /
//       response exchange with the owners of its target node and its predecessor group
//       (SDBG construction, MEGAHIT; the neighbour queries of cycle_finder.cpp:58-123);
//   CollectTips + InvalidateMultiplicityOneNodes (cycle_finder.cpp:346-357, 372-382): local;
//   the post-filter out-degree, ChunkStartNodes' in-degree filter (:29-36, 387-427): windows of
//       the owners' filtered bitmaps, one request / response;
//   RecursiveReduction (:359-371, 440-442), the monotone least fixpoint: a distributed list
//       ranking — predecessor flags as messages, rulers walking their chains in bulk-synchronous
//       rounds (a step onto another owner's edge is a message), pointer jumping over the rulers,
//       branch resolution rounds — then removal (Router below carries every exchange);
//   the valid count and tips recount (:443-452): local, summed;
//   DepthLevelSearch (:248-343, 394-419) and FindCycle (:140-243, 468-487): on a search-region
//       replica. A search only follows valid edges, at most cycle_max_length deep, and the lock
//       relaxation walks in-edges at most as many steps back, so every rank gathers the groups
//       within that radius of the starts (bulk-synchronous BFS rounds over the owners) into a
//       compact graph; the existing search kernels run on it unchanged (gid keeps FindCycle's
//       libstdc++ frame order), split over the ranks as before.
// No rank holds, scans or peels the whole graph; results equal the one-GPU path bit for bit
// (tests/test_native_multi.py).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <map>

#include "comm.h"

namespace mcaat {

namespace {

constexpr int kBlk = 256;
constexpr uint64_t kNo = ~0ULL;
constexpr uint64_t kRef = 1ULL << 62;        // a jump / reference to a ruler (its edge id below)
constexpr uint64_t kIdM = (1ULL << 40) - 1;  // edge ids
// kind byte of a local edge: post-filter valid out-edges (4-bit window over the out_info
// positions), a unary predecessor exists, a branch predecessor exists, ruler
constexpr uint8_t kUpred = 0x10, kBpred = 0x20, kRuler = 0x40;
constexpr uint8_t kStUnk = 0, kStRem = 1, kStSurv = 2;
constexpr uint64_t kPad = kNo - 1;  // an unused successor slot of a branch

bool verbose() {
    static const bool v = getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1';
    return v;
}

// ---------------------------------------------------------------- owners
struct Owners {  // N <= 64 (Comm limits)
    int N;
    int R;
    uint64_t id_lo;
    uint64_t n;  // D_local
    uint64_t rank_lo[65];
    uint64_t split[64];
};
__device__ __forceinline__ int owner_of_id(const Owners &o, uint64_t x) {
    int r = 0;
    while (r + 1 < o.N && o.rank_lo[r + 1] <= x) ++r;
    return r;
}
__device__ __forceinline__ int owner_of_key(const Owners &o, uint64_t K) {
    int r = 0;
    while (r < o.N - 1 && o.split[r] <= K) ++r;
    return r;
}

Owners owners_of(const mcaat_graph *g, const Comm &comm) {
    Owners o{};
    o.N = comm.world;
    o.R = comm.rank;
    o.id_lo = g->id_lo;
    o.n = g->D_local;
    for (int r = 0; r <= o.N; ++r) o.rank_lo[r] = g->rank_lo[r];
    for (int r = 0; r + 1 < o.N; ++r) o.split[r] = g->key_split[r];
    return o;
}

__device__ __forceinline__ bool bit_of(const uint64_t *bm, uint64_t i) { return (bm[i >> 6] >> (i & 63)) & 1; }

// ---------------------------------------------------------------- Router
// Records of W 64-bit words with a destination rank each go to their ranks in one all-to-all
// (grouped by destination on the device: a block reserves its per-destination ranges with one
// atomic per destination). perm keeps, for a request / response pattern, which record went out
// at each send position, so the answers (in the order the owner received them) come back to
// their requests. Order within a destination is not fixed; nothing here depends on it.
__global__ void __launch_bounds__(kBlk) k_dest_count(const uint8_t *dest, uint64_t n, unsigned long long *cnt, int N) {
    __shared__ unsigned int h[64];
    for (int i = threadIdx.x; i < N; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) atomicAdd(&h[dest[i]], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < N; i += blockDim.x)
        if (h[i]) atomicAdd(&cnt[i], (unsigned long long)h[i]);
}

__global__ void __launch_bounds__(kBlk) k_dest_scatter(const uint64_t *rec, int W, const uint8_t *dest, uint64_t n,
                                                       const uint64_t *off, unsigned long long *cur, uint64_t *out,
                                                       uint32_t *perm, int N) {
    __shared__ unsigned int h[64];
    __shared__ unsigned long long base[64];
    for (uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x; t0 < n; t0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = t0 + threadIdx.x;
        for (int q = threadIdx.x; q < N; q += blockDim.x) h[q] = 0;
        __syncthreads();
        const int d = i < n ? dest[i] : 0;
        const unsigned int r = i < n ? atomicAdd(&h[d], 1u) : 0u;
        __syncthreads();
        for (int q = threadIdx.x; q < N; q += blockDim.x) base[q] = h[q] ? atomicAdd(&cur[q], (unsigned long long)h[q]) : 0ull;
        __syncthreads();
        if (i < n) {
            const uint64_t pos = off[d] + base[d] + r;
            for (int w = 0; w < W; ++w) out[pos * W + w] = rec[i * W + w];
            if (perm) perm[pos] = (uint32_t)i;
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(kBlk) k_unperm(const uint64_t *ans, int W, const uint32_t *perm, uint64_t n, uint64_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride)
        for (int w = 0; w < W; ++w) out[(uint64_t)perm[k] * W + w] = ans[k * W + w];
}

struct Routed {
    int W = 1;
    uint64_t n = 0, n_in = 0, total = 0;  // sent, received, sent by all ranks
    std::vector<uint64_t> out_cnt, in_cnt;
    DevBuf<uint32_t> perm;
    DevBuf<uint64_t> in;  // received records, sources in rank order
};

struct Router {
    mcaat_ctx *ctx;
    Comm &comm;
    uint64_t rounds = 0, records = 0;  // collectives and records moved (diagnostics)
    Router(mcaat_ctx *c, Comm &cm) : ctx(c), comm(cm) {}

    void send(const uint64_t *rec, int W, const uint8_t *dest, uint64_t n, Routed &rt, bool keep_perm) {
        hipStream_t st = ctx->stream;
        const int N = comm.world, R = comm.rank;
        if (n >= (1ULL << 32)) throw Error(MCAAT_E_CAPACITY, "shard router: 2^32 or more records in one exchange");
        rt.W = W;
        rt.n = n;
        rt.out_cnt.assign(N, 0);
        DevBuf<unsigned long long> cnt(2 * N);
        HIP_OK(hipMemsetAsync(cnt.p, 0, 16 * N, st));
        if (n) {
            hipLaunchKernelGGL(k_dest_count, dim3(grid_for(n, kBlk, (unsigned)ctx->n_cu * 8)), dim3(kBlk), 0, st, dest, n,
                               cnt.p, N);
            LAUNCH_OK();
            d2h(ctx, rt.out_cnt.data(), cnt.p, 8 * N);
        }
        std::vector<uint64_t> off(N + 1, 0);
        for (int q = 0; q < N; ++q) off[q + 1] = off[q] + rt.out_cnt[q];
        DevBuf<uint64_t> sendb((n ? n : 1) * W);
        if (keep_perm) rt.perm.alloc(n ? n : 1);
        if (n) {
            DevBuf<uint64_t> doff(N);
            HIP_OK(hipMemcpyAsync(doff.p, off.data(), 8 * N, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_dest_scatter, dim3(grid_for(n, kBlk, (unsigned)ctx->n_cu * 8)), dim3(kBlk), 0, st, rec, W,
                               dest, n, doff.p, cnt.p + N, sendb.p, keep_perm ? rt.perm.p : nullptr, N);
            LAUNCH_OK();
        }
        const std::vector<uint64_t> mat = comm.allgather_vec(rt.out_cnt);
        rt.in_cnt.assign(N, 0);
        rt.n_in = rt.total = 0;
        for (int s = 0; s < N; ++s) {
            rt.in_cnt[s] = mat[(uint64_t)s * N + R];
            rt.n_in += rt.in_cnt[s];
            for (int d = 0; d < N; ++d) rt.total += mat[(uint64_t)s * N + d];
        }
        rt.in.alloc((rt.n_in ? rt.n_in : 1) * W);
        std::vector<uint64_t> sb(N), rb(N);
        for (int q = 0; q < N; ++q) sb[q] = 8ULL * W * rt.out_cnt[q], rb[q] = 8ULL * W * rt.in_cnt[q];
        HIP_OK(hipStreamSynchronize(st));
        if (rt.total) comm.alltoallv_dev(sendb.p, sb.data(), rt.in.p, rb.data());
        ++rounds;
        records += n;
    }
    // answers (Wa words per received record, in received order) back to the requests: out[i * Wa ..]
    void reply(Routed &rt, const uint64_t *ans, int Wa, uint64_t *out) {
        hipStream_t st = ctx->stream;
        const int N = comm.world;
        DevBuf<uint64_t> back((rt.n ? rt.n : 1) * Wa);
        std::vector<uint64_t> sb(N), rb(N);
        for (int q = 0; q < N; ++q) sb[q] = 8ULL * Wa * rt.in_cnt[q], rb[q] = 8ULL * Wa * rt.out_cnt[q];
        HIP_OK(hipStreamSynchronize(st));
        if (rt.total) comm.alltoallv_dev(ans, sb.data(), back.p, rb.data());
        if (rt.n) {
            hipLaunchKernelGGL(k_unperm, dim3(grid_for(rt.n, kBlk, (unsigned)ctx->n_cu * 16)), dim3(kBlk), 0, st,
                               (const uint64_t *)back.p, Wa, (const uint32_t *)rt.perm.p, rt.n, out);
            LAUNCH_OK();
        }
        HIP_OK(hipStreamSynchronize(st));
        ++rounds;
    }
};

// Appends to a list with one cursor atomic per wave (ballot + mbcnt); entries past cap are
// counted, not written (callers size lists so that cannot happen: cap = every possible entry).
__device__ __forceinline__ uint64_t wave_reserve(bool f, unsigned long long *cursor, unsigned long long &mask) {
    mask = __ballot(f);
    const int lane = threadIdx.x & 63;
    unsigned long long base = 0;
    if (mask) {
        if (lane == __ffsll((long long)mask) - 1) base = atomicAdd(cursor, (unsigned long long)__popcll(mask));
        base = __shfl(base, __ffsll((long long)mask) - 1);
    }
    const unsigned long long below = lane ? mask & (~0ull >> (64 - lane)) : 0ull;
    return base + (uint64_t)__popcll(below);
}

uint64_t read_u64(mcaat_ctx *ctx, const unsigned long long *d) {
    uint64_t h = 0;
    d2h(ctx, &h, d, 8);
    return h;
}

// ---------------------------------------------------------------- sharded adjacency
// local radix directory: dir[p] = first local index whose (key - base) >> shift >= p, p in [0, np]
__global__ void __launch_bounds__(kBlk) k_sdir(const uint64_t *key, uint64_t n, uint64_t base, int shift, uint64_t np,
                                               uint64_t *dir) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e <= n; e += stride) {
        uint64_t p = e < n ? (key[e] - base) >> shift : np;
        p = p < np ? p : np;
        const uint64_t first = e ? ((key[e - 1] - base) >> shift) + 1 : 0;
        for (uint64_t q = first; q <= p; ++q) dir[q] = e;
    }
}

__device__ __forceinline__ uint64_t lb_local(const uint64_t *key, uint64_t n, const uint64_t *dir, uint64_t base, int shift,
                                             uint64_t np, uint64_t q) {
    if (q < base) return 0;
    const uint64_t p = (q - base) >> shift;
    if (p >= np) return n;
    uint64_t lo = dir[p], hi = dir[p + 1];
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (key[mid] < q) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// two queries per edge: [2i] the target node's first edge (key prefix of s[1..k-1]W), [2i+1]
// (bit 63) the predecessors' group (s[0..k-2]) and the W they carry (s[k-1])
__global__ void __launch_bounds__(kBlk) k_adj_queries(const uint64_t *key, uint64_t i0, uint64_t m, int k, Owners o,
                                                      uint64_t *q, uint8_t *dest) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t gmask = (1ULL << (2 * (k - 1))) - 1;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        const uint64_t K = key[i0 + j], W = K & 3, R = K >> 2;
        const uint64_t Qo = ((W << (2 * (k - 1))) | (R >> 2)) << 2;
        const uint64_t G = R & gmask, x = R >> (2 * (k - 1));
        q[2 * j] = Qo;
        dest[2 * j] = (uint8_t)owner_of_key(o, Qo);
        q[2 * j + 1] = (G << 4) | x | (1ULL << 63);
        dest[2 * j + 1] = (uint8_t)owner_of_key(o, G << 4);
    }
}

__global__ void __launch_bounds__(kBlk) k_adj_answer(const uint64_t *key, uint64_t n, uint64_t id_lo, const uint64_t *dir,
                                                     uint64_t base, int shift, uint64_t np, const uint64_t *q, uint64_t m,
                                                     uint64_t *ans) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        const uint64_t Q = q[j] & ~(1ULL << 63);
        if (!(q[j] >> 63)) {  // out_info: the target node's first edge and its W set
            const uint64_t lo = lb_local(key, n, dir, base, shift, np, Q);
            uint64_t mask = 0;
            for (int i = 0; i < 4; ++i)
                if (lo + i < n && (key[lo + i] >> 2) == (Q >> 2)) mask |= 1ULL << (key[lo + i] & 3);
            ans[j] = (id_lo + lo) | (mask << kIdxBits);
        } else {  // in_info: the group start and the positions of its edges with W == x
            const uint64_t G = Q >> 4, x = Q & 3;
            const uint64_t lo = lb_local(key, n, dir, base, shift, np, G << 4);
            uint64_t mask = 0;
            for (int i = 0; i < 16; ++i)
                if (lo + i < n && (key[lo + i] >> 4) == G && (key[lo + i] & 3) == x) mask |= 1ULL << i;
            ans[j] = mask ? (id_lo + lo) | (mask << kIdxBits) : 0;  // no predecessors: 0, as the one-GPU build
        }
    }
}

__global__ void __launch_bounds__(kBlk) k_adj_store(const uint64_t *a, uint64_t i0, uint64_t m, uint64_t *out_info,
                                                    uint64_t *in_info) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        out_info[i0 + j] = a[2 * j];
        in_info[i0 + j] = a[2 * j + 1];
    }
}

__global__ void __launch_bounds__(kBlk) k_fill(uint64_t *x, uint64_t n, uint64_t v) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = v;
}

__global__ void __launch_bounds__(kBlk) k_ones(uint64_t *bm, uint64_t n) {
    const uint64_t nw = (n + 63) / 64, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride)
        bm[w] = (w + 1) * 64 <= n ? ~0ULL : (~0ULL >> (64 - (n - w * 64)));
}

// ---------------------------------------------------------------- CycleFinder, D-wide
// CollectTips (fresh graph: an edge without out-edges) and InvalidateMultiplicityOneNodes,
// one wave per 64 local edges
__global__ void __launch_bounds__(kBlk) k_sh_filter(const uint16_t *mult, const uint64_t *out_info, uint64_t n,
                                                    uint64_t *post, uint64_t *seed, unsigned long long *cnt) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (n + 63) / 64, wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    unsigned long long tips = 0, low = 0;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += wstride) {
        const uint64_t i = w * 64 + lane;
        const bool in = i < n;
        const uint32_t m = in ? mult[i] : 0;
        const bool t = in && ((out_info[i] >> kIdxBits) & 0xF) == 0;
        const unsigned long long pm = __ballot(in && m > 1), tm = __ballot(t), lm = __ballot(in && m <= 1);
        if (lane == 0) {
            post[w] = pm;
            seed[w] = tm;
            tips += __popcll(tm);
            low += __popcll(lm);
        }
    }
    block_add(cnt, tips);
    block_add(cnt + 1, low);
}

// window requests: every filter-valid edge with out-edges asks the 16 filtered bits at its
// target node's first edge; filter-valid edges above the threshold ask their predecessor group's
// (ChunkStartNodes' in-degree); src = local index | 1 << 63 for the in-window
__global__ void __launch_bounds__(kBlk) k_win_req(const uint64_t *post, const uint16_t *mult, const uint64_t *out_info,
                                                  const uint64_t *in_info, uint64_t a0, uint64_t n, uint64_t thr, Owners o,
                                                  uint64_t *q, uint8_t *dest, uint64_t *src, unsigned long long *cur) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i0 = a0 + (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
        const uint64_t i = i0 + threadIdx.x;
        const bool pv = i < n && bit_of(post, i);
        const uint64_t oi = pv ? out_info[i] : 0;
        const bool wo = pv && ((oi >> kIdxBits) & 0xF);
        const uint64_t ii = pv && (uint64_t)mult[i] > thr ? in_info[i] : 0;
        const bool wi = (ii >> kIdxBits) != 0;
        unsigned long long m;
        uint64_t at = wave_reserve(wo, cur, m);
        if (wo) {
            q[at] = oi & kIdM;
            dest[at] = (uint8_t)owner_of_id(o, oi & kIdM);
            src[at] = i;
        }
        at = wave_reserve(wi, cur, m);
        if (wi) {
            q[at] = ii & kIdM;
            dest[at] = (uint8_t)owner_of_id(o, ii & kIdM);
            src[at] = i | (1ULL << 63);
        }
    }
}

// 16 bits of a local bitmap from global id x (bits outside the range read 0; the bitmap has a
// padding word)
__device__ __forceinline__ uint32_t bits16_local(const uint64_t *bm, uint64_t n, uint64_t li) {
    if (li >= n) return 0;
    const uint64_t w = li >> 6;
    const int sh = (int)(li & 63);
    const uint64_t v = (bm[w] >> sh) | (sh ? bm[w + 1] << (64 - sh) : 0);
    return (uint32_t)(v & 0xFFFF);
}

__global__ void __launch_bounds__(kBlk) k_win_ans(const uint64_t *bm, uint64_t n, uint64_t id_lo, const uint64_t *q,
                                                  uint64_t m, uint64_t *ans) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride)
        ans[j] = bits16_local(bm, n, q[j] - id_lo);
}

// the answers: kind (filtered out-window), unary successor, candidates (in-window)
__global__ void __launch_bounds__(kBlk) k_win_apply(const uint64_t *src, const uint64_t *ans, uint64_t m,
                                                    const uint64_t *out_info, const uint64_t *in_info, uint64_t id_lo,
                                                    uint8_t *kind, uint64_t *nx, uint64_t *cand, unsigned long long *ncand) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < m; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        bool c = false;
        uint64_t e = 0;
        if (j < m) {
            const uint64_t s = src[j], i = s & ~(1ULL << 63);
            const uint32_t b = (uint32_t)ans[j];
            if (!(s >> 63)) {
                const uint64_t oi = out_info[i];
                const int cnt = __popc((unsigned)(oi >> kIdxBits) & 0xF);
                const uint32_t pm = b & ((1u << cnt) - 1);
                kind[i] = (uint8_t)pm;  // the flag bits come later (k_flag_apply)
                if (__popc(pm) == 1) nx[i] = (oi & kIdM) + (uint64_t)(__ffs(pm) - 1);
            } else {
                const uint64_t ii = in_info[i], l = ii & kIdM;
                const uint32_t in = b & (uint32_t)((ii >> kIdxBits) & 0xFFFF);
                e = id_lo + i;
                const bool self = e >= l && e - l < 16 && ((in >> (e - l)) & 1);
                c = __popc(in) >= 2 && !self;  // _IncomingNotEqualToCurrentNode, indegree >= 2
            }
        }
        unsigned long long mk;
        const uint64_t at = wave_reserve(c, ncand, mk);
        if (c) cand[at] = e;
    }
}

// post-filter tips that are not seeds (counts[2]); predecessor flags as messages to the
// successors: id | 1 << 62 from a unary edge, id | 1 << 63 from a branch edge
__global__ void __launch_bounds__(kBlk) k_flag_msgs(const uint64_t *post, const uint64_t *seed, const uint8_t *kind,
                                                    const uint64_t *out_info, uint64_t a0, uint64_t n, Owners o, uint64_t *q,
                                                    uint8_t *dest, unsigned long long *cur, unsigned long long *cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long tpf = 0;
    for (uint64_t i0 = a0 + (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
        const uint64_t i = i0 + threadIdx.x;
        const bool pv = i < n && bit_of(post, i);
        const uint32_t pm = pv ? kind[i] & 0xF : 0;
        const int od = __popc(pm);
        if (pv && od == 0 && !bit_of(seed, i)) ++tpf;
        const uint64_t lo = pv ? out_info[i] & kIdM : 0;
        for (int b = 0; b < 4; ++b) {
            const bool f = (pm >> b) & 1;
            unsigned long long mk;
            const uint64_t at = wave_reserve(f, cur, mk);
            if (f) {
                const uint64_t y = lo + b;
                q[at] = y | (od == 1 ? (1ULL << 62) : (1ULL << 63));
                dest[at] = (uint8_t)owner_of_id(o, y);
            }
        }
    }
    block_add(cnt + 2, tpf);
}

__device__ __forceinline__ void or_byte(uint8_t *a, uint64_t i, uint32_t v) {
    atomicOr((unsigned int *)(a + (i & ~3ULL)), v << (8 * (i & 3)));
}

__global__ void __launch_bounds__(kBlk) k_flag_apply(const uint64_t *q, uint64_t m, uint64_t id_lo, uint8_t *kind) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        const uint64_t x = q[j];
        or_byte(kind, (x & kIdM) - id_lo, (x >> 62) == 1 ? kUpred : kBpred);
    }
}

// rulers (unary chain heads and 1 in rmask + 1 unary edges by the hash of their id), states of
// the non-unary edges (dead ends: removed iff a seed; branches unresolved); lists of rulers
// and branches (local indices)
__global__ void __launch_bounds__(kBlk) k_prep(const uint64_t *post, const uint64_t *seed, uint8_t *kind, uint8_t *st,
                                               uint64_t n, uint64_t id_lo, uint64_t rmask, uint64_t *rl,
                                               unsigned long long *nr, uint64_t *bl, unsigned long long *nb) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
        const uint64_t i = i0 + threadIdx.x;
        const bool pv = i < n && bit_of(post, i);
        const uint8_t k = pv ? kind[i] : 0;
        const int od = __popc(k & 0xF);
        const bool ruler = pv && od == 1 && (!(k & kUpred) || (mix64((id_lo + i) ^ 0x5eed) & rmask) == 0);
        const bool branch = pv && od >= 2;
        if (pv) {
            if (ruler) kind[i] = k | kRuler;
            st[i] = od == 0 ? (bit_of(seed, i) ? kStRem : kStSurv) : kStUnk;
        }
        unsigned long long mk;
        uint64_t at = wave_reserve(ruler, nr, mk);
        if (ruler) rl[at] = i;
        at = wave_reserve(branch, nb, mk);
        if (branch) bl[at] = i;
    }
}

// walkers: {ruler, edge, tortoise, power << 32 | lam}; results: {ruler, reached, 0, 1 << 63}
// (reached: a non-unary edge, kRef | a ruler, or kNo on a ruler-less unary cycle)
constexpr uint64_t kResult = 1ULL << 63;

__global__ void __launch_bounds__(kBlk) k_walk_init(const uint64_t *rl, uint64_t nr, const uint64_t *nx, uint64_t id_lo,
                                                    uint64_t *w) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nr; j += stride) {
        const uint64_t i = rl[j];
        w[4 * j] = id_lo + i;
        w[4 * j + 1] = nx[i];
        w[4 * j + 2] = id_lo + i;
        w[4 * j + 3] = (1ULL << 32) | 1;
    }
}

// one round: results land in their rulers' jump words (nx of the ruler, no longer read: a walk
// stops at a ruler before reading its successor); walkers advance over this rank's edges and
// leave for the owner of the next one (Brent's cycle check as the one-GPU k_peel_walk)
__global__ void __launch_bounds__(kBlk) k_walk(const uint64_t *in, uint64_t m, const uint8_t *kind, uint64_t *nx,
                                               uint64_t *own, Owners o, uint64_t *out, uint8_t *dest,
                                               unsigned long long *cur) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < m; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        bool emit = false;
        uint64_t r = 0, x = 0, tort = 0, pl = 0;
        int to = 0;
        if (j < m) {
            r = in[4 * j];
            x = in[4 * j + 1];
            tort = in[4 * j + 2];
            pl = in[4 * j + 3];
            if (pl & kResult) {
                nx[r - o.id_lo] = x;
            } else {
                uint64_t power = pl >> 32, lam = pl & 0xFFFFFFFFu;
                for (;;) {
                    if (x < o.id_lo || x >= o.id_lo + o.n) {  // leaves for the owner of x
                        emit = true;
                        to = owner_of_id(o, x);
                        pl = (power << 32) | lam;
                        break;
                    }
                    const uint64_t li = x - o.id_lo;
                    const uint8_t k = kind[li];
                    uint64_t res = 0;
                    bool done = true;
                    if (__popc(k & 0xF) != 1) res = x;
                    else if (k & kRuler) res = kRef | x;
                    else if (x == tort) res = kNo;
                    else done = false;
                    if (done) {
                        emit = true;
                        to = owner_of_id(o, r);
                        x = res;
                        tort = 0;
                        pl = kResult;
                        break;
                    }
                    own[li] = r;
                    if (power == lam) {
                        tort = x;
                        power <<= 1;
                        lam = 0;
                    }
                    x = nx[li];
                    ++lam;
                }
            }
        }
        unsigned long long mk;
        const uint64_t at = wave_reserve(emit, cur, mk);
        if (emit) {
            out[4 * at] = r;
            out[4 * at + 1] = x;
            out[4 * at + 2] = tort;
            out[4 * at + 3] = pl;
            dest[at] = (uint8_t)to;
        }
    }
}

// pointer jumping: requests of the rulers still pointing at a ruler
__global__ void __launch_bounds__(kBlk) k_jump_req(const uint64_t *al, uint64_t na, const uint64_t *nx, Owners o, uint64_t *q,
                                                   uint8_t *dest) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < na; j += stride) {
        const uint64_t t = nx[al[j]] & kIdM;
        q[j] = t;
        dest[j] = (uint8_t)owner_of_id(o, t);
    }
}
__global__ void __launch_bounds__(kBlk) k_jump_ans(const uint64_t *q, uint64_t m, const uint64_t *nx, uint64_t id_lo, uint64_t *ans) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) ans[j] = nx[q[j] - id_lo];
}
// the new jumps; the rulers still pointing at a ruler stay listed
__global__ void __launch_bounds__(kBlk) k_jump_apply(const uint64_t *al, uint64_t na, const uint64_t *a, uint64_t *nx,
                                                     uint64_t *al2, unsigned long long *na2) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < na; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        bool keep = false;
        if (j < na) {
            nx[al[j]] = a[j];
            keep = a[j] != kNo && (a[j] & kRef);
        }
        unsigned long long mk;
        const uint64_t at = wave_reserve(keep, na2, mk);
        if (keep) al2[at] = al[j];
    }
}
__global__ void __launch_bounds__(kBlk) k_jump_cycle(const uint64_t *al, uint64_t na, uint64_t *nx) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < na; j += stride) nx[al[j]] = kNo;
}
// the rulers whose jump still points at a ruler (kept in `al`) after the walks
__global__ void __launch_bounds__(kBlk) k_active_rulers(const uint64_t *rl, uint64_t nr, const uint64_t *nx, uint64_t *al,
                                                        unsigned long long *na) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < nr; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        const bool a = j < nr && nx[rl[j]] != kNo && (nx[rl[j]] & kRef);
        unsigned long long mk;
        const uint64_t at = wave_reserve(a, na, mk);
        if (a) al[at] = rl[j];
    }
}

// the references of branch successors: request y (4 slots per branch, kNo past its successors)
__global__ void __launch_bounds__(kBlk) k_bref_req(const uint64_t *bl, uint64_t nb, const uint8_t *kind,
                                                   const uint64_t *out_info, Owners o, uint64_t *q, uint8_t *dest,
                                                   uint64_t *src, unsigned long long *cur) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < nb; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        const uint32_t pm = j < nb ? kind[bl[j]] & 0xF : 0;
        const uint64_t lo = j < nb ? out_info[bl[j]] & kIdM : 0;
        for (int b = 0; b < 4; ++b) {
            const bool f = (pm >> b) & 1;
            unsigned long long mk;
            const uint64_t at = wave_reserve(f, cur, mk);
            if (f) {
                q[at] = lo + b;
                dest[at] = (uint8_t)owner_of_id(o, lo + b);
                src[at] = 4 * j + b;
            }
        }
    }
}
// a successor's reference: itself (non-unary), its ruler's terminal (a ruler), or kRef | the
// ruler whose walk passed it (kNo: none did — a ruler-less unary cycle)
__global__ void __launch_bounds__(kBlk) k_bref_ans(const uint64_t *q, uint64_t m, const uint8_t *kind, const uint64_t *nx,
                                                   const uint64_t *own, uint64_t id_lo, uint64_t *ans) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        const uint64_t y = q[j], li = y - id_lo;
        const uint8_t k = kind[li];
        if (__popc(k & 0xF) != 1) ans[j] = y;
        else if (k & kRuler) ans[j] = nx[li];
        else ans[j] = own[li] == kNo ? kNo : (kRef | own[li]);
    }
}
__global__ void __launch_bounds__(kBlk) k_scatter_ref(const uint64_t *src, const uint64_t *a, uint64_t m, uint64_t *ref) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) ref[src[j]] = a[j];
}
// second step for successors owned by a passing ruler: that ruler's terminal
__global__ void __launch_bounds__(kBlk) k_bref_req2(const uint64_t *ref, uint64_t nslots, Owners o, uint64_t *q, uint8_t *dest,
                                                    uint64_t *src, unsigned long long *cur) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < nslots; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        const bool f = j < nslots && ref[j] < kPad && (ref[j] & kRef);
        unsigned long long mk;
        const uint64_t at = wave_reserve(f, cur, mk);
        if (f) {
            q[at] = ref[j] & kIdM;
            dest[at] = (uint8_t)owner_of_id(o, ref[j] & kIdM);
            src[at] = j;
        }
    }
}

// branch resolution: a branch with a surviving reference (kNo: a unary cycle) survives at once;
// otherwise its references' states are requested
__global__ void __launch_bounds__(kBlk) k_res_req(const uint64_t *bl, const uint64_t *ref, uint64_t nb, uint8_t *st,
                                                  Owners o, uint64_t *q, uint8_t *dest, uint64_t *src,
                                                  unsigned long long *cur, unsigned long long *changed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long ch = 0;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < nb; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        bool unk = j < nb && st[bl[j]] == kStUnk;
        if (unk) {
            for (int b = 0; b < 4; ++b)
                if (ref[4 * j + b] == kNo) unk = false;
            if (!unk) {
                st[bl[j]] = kStSurv;
                ++ch;
            }
        }
        for (int b = 0; b < 4; ++b) {
            const uint64_t t = unk ? ref[4 * j + b] : kPad;
            const bool f = t != kPad;
            unsigned long long mk;
            const uint64_t at = wave_reserve(f, cur, mk);
            if (f) {
                q[at] = t;
                dest[at] = (uint8_t)owner_of_id(o, t);
                src[at] = 4 * j + b;
            }
        }
    }
    block_add(changed, ch);
}
__global__ void __launch_bounds__(kBlk) k_st_ans(const uint64_t *q, uint64_t m, const uint8_t *st, uint64_t id_lo, uint64_t *ans) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) ans[j] = st[q[j] - id_lo];
}
// per branch slot: the state of its reference (written by the answers; kStRem for padding)
__global__ void __launch_bounds__(kBlk) k_res_apply(const uint64_t *bl, uint64_t nb, const uint8_t *slot_st, uint8_t *st,
                                                    unsigned long long *changed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long ch = 0;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nb; j += stride) {
        if (st[bl[j]] != kStUnk) continue;
        bool all_rem = true, any_surv = false;
        for (int b = 0; b < 4; ++b) {
            const uint8_t s = slot_st[4 * j + b];
            if (s == kStSurv) any_surv = true;
            if (s != kStRem) all_rem = false;
        }
        if (any_surv) { st[bl[j]] = kStSurv; ++ch; }
        else if (all_rem) { st[bl[j]] = kStRem; ++ch; }
    }
    block_add(changed, ch);
}
__global__ void __launch_bounds__(kBlk) k_slot_st(const uint64_t *src, const uint64_t *a, uint64_t m, uint8_t *slot_st) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) slot_st[src[j]] = (uint8_t)a[j];
}

// removal of the non-unary edges resolved kRem (valid starts as the filtered bitmap)
__global__ void __launch_bounds__(kBlk) k_rm_nonunary(const uint64_t *post, const uint8_t *kind, const uint8_t *st, uint64_t n,
                                                      uint64_t *valid) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (n + 63) / 64, wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += wstride) {
        const uint64_t i = w * 64 + lane;
        const bool rm = i < n && bit_of(post, i) && __popc(kind[i] & 0xF) != 1 && st[i] == kStRem;
        const unsigned long long m = __ballot(rm);
        if (lane == 0) valid[w] = post[w] & ~m;
    }
}
// rulers: the state of their terminal (kNo: survive)
__global__ void __launch_bounds__(kBlk) k_term_req(const uint64_t *rl, uint64_t nr, const uint64_t *nx, Owners o, uint64_t *q,
                                                   uint8_t *dest, uint64_t *src, unsigned long long *cur) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < nr; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        const uint64_t t = j < nr ? nx[rl[j]] : kNo;
        const bool f = t != kNo;
        unsigned long long mk;
        const uint64_t at = wave_reserve(f, cur, mk);
        if (f) {
            q[at] = t;
            dest[at] = (uint8_t)owner_of_id(o, t);
            src[at] = rl[j];
        }
    }
}
// removed rulers: their own valid bit cleared, their ids listed
__global__ void __launch_bounds__(kBlk) k_rm_rulers(const uint64_t *src, const uint64_t *a, uint64_t m, uint64_t id_lo,
                                                    uint64_t *valid, uint64_t *rm, unsigned long long *nrm) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < m; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        const bool r = j < m && a[j] == kStRem;
        if (r) atomicAnd((unsigned long long *)&valid[src[j] >> 6], ~(1ULL << (src[j] & 63)));
        unsigned long long mk;
        const uint64_t at = wave_reserve(r, nrm, mk);
        if (r) rm[at] = id_lo + src[j];
    }
}
// open-addressing set of the removed rulers (every rank holds all of them)
__global__ void __launch_bounds__(kBlk) k_set_build(const uint64_t *ids, uint64_t m, uint64_t *tab, uint64_t cap) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride)
        for (uint64_t h = mix64(ids[j]) & (cap - 1);; h = (h + 1) & (cap - 1)) {
            const unsigned long long prev = atomicCAS((unsigned long long *)&tab[h], kNo, ids[j]);
            if (prev == kNo || prev == ids[j]) break;
        }
}
// non-ruler unary edges passed by a removed ruler's walk
__global__ void __launch_bounds__(kBlk) k_rm_chains(const uint64_t *post, const uint8_t *kind, const uint64_t *own, uint64_t n,
                                                    const uint64_t *tab, uint64_t cap, uint64_t *valid) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (n + 63) / 64, wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += wstride) {
        const uint64_t i = w * 64 + lane;
        bool rm = false;
        if (i < n && bit_of(post, i)) {
            const uint8_t k = kind[i];
            if (__popc(k & 0xF) == 1 && !(k & kRuler) && own[i] != kNo) {
                const uint64_t r = own[i];
                for (uint64_t h = mix64(r) & (cap - 1);; h = (h + 1) & (cap - 1)) {
                    const uint64_t x = tab[h];
                    if (x == r) { rm = true; break; }
                    if (x == kNo) break;
                }
            }
        }
        const unsigned long long m = __ballot(rm);
        if (lane == 0 && m) valid[w] &= ~m;
    }
}

__global__ void __launch_bounds__(kBlk) k_popc(const uint64_t *bm, uint64_t nw, unsigned long long *out) {
    unsigned long long c = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) c += __popcll(bm[w]);
    block_add(out, c);
}

// the candidates still valid after the peel (global ids -> local test)
__global__ void __launch_bounds__(kBlk) k_cand_keep(const uint64_t *cand, uint64_t m, const uint64_t *valid, uint64_t id_lo,
                                                    uint64_t *out, unsigned long long *n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < m; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        const bool k = j < m && bit_of(valid, cand[j] - id_lo);
        unsigned long long mk;
        const uint64_t at = wave_reserve(k, n, mk);
        if (k) out[at] = cand[j];
    }
}

// ---------------------------------------------------------------- search regions
// group starts: the first edge of every (k-1)-suffix group (key >> 4); a rank's range starts one
__global__ void __launch_bounds__(kBlk) k_gstart(const uint64_t *key, uint64_t n, uint64_t *gs) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (n + 63) / 64, wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += wstride) {
        const uint64_t i = w * 64 + lane;
        const bool s = i < n && (i == 0 || (key[i] >> 4) != (key[i - 1] >> 4));
        const unsigned long long m = __ballot(s);
        if (lane == 0) gs[w] = m;
    }
}

// marks the group of local edge li in reg (groups hold at most 16 edges)
__device__ __forceinline__ void mark_group(const uint64_t *gs, uint64_t n, uint64_t li, uint64_t *reg) {
    uint64_t a = li;
    while (a > 0 && !bit_of(gs, a)) --a;
    uint64_t b = li + 1;
    while (b < n && !bit_of(gs, b)) ++b;
    for (uint64_t x = a; x < b;) {
        const uint64_t w = x >> 6, e = min(b, (w + 1) * 64);
        const uint64_t lo = x & 63, cnt = e - x;
        const uint64_t m = (cnt == 64 ? ~0ULL : ((1ULL << cnt) - 1)) << lo;
        if ((reg[w] & m) != m) atomicOr((unsigned long long *)&reg[w], m);
        x = e;
    }
}

// the starts of a BFS: their groups marked, themselves seen and listed (local indices)
__global__ void __launch_bounds__(kBlk) k_bfs_seed(const uint64_t *ids, uint64_t m, uint64_t id_lo, uint64_t n, const uint64_t *gs,
                                                   uint64_t *reg, uint64_t *seen, uint64_t *front) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        const uint64_t li = ids[j] - id_lo;
        mark_group(gs, n, li, reg);
        atomicOr((unsigned long long *)&seen[li >> 6], 1ULL << (li & 63));
        front[j] = li;
    }
}
// one BFS hop request per frontier edge: its successors' window (forward) or its
// predecessors' (backward): first id | position mask << 40
__global__ void __launch_bounds__(kBlk) k_bfs_req(const uint64_t *front, uint64_t nf, const uint64_t *out_info,
                                                  const uint64_t *in_info, int backward, Owners o, uint64_t *q,
                                                  uint8_t *dest, unsigned long long *cur) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < nf; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        uint64_t lo = 0, pos = 0;
        if (j < nf) {
            const uint64_t li = front[j];
            if (backward) {
                const uint64_t ii = in_info[li];
                lo = ii & kIdM;
                pos = (ii >> kIdxBits) & 0xFFFF;
            } else {
                const uint64_t oi = out_info[li];
                lo = oi & kIdM;
                pos = (1ULL << __popc((unsigned)(oi >> kIdxBits) & 0xF)) - 1;
            }
        }
        const bool f = pos != 0;
        unsigned long long mk;
        const uint64_t at = wave_reserve(f, cur, mk);
        if (f) {
            q[at] = lo | (pos << kIdxBits);
            dest[at] = (uint8_t)owner_of_id(o, lo);
        }
    }
}
// the owner: the window's group joins the region; its valid, unseen positions join the next frontier
__global__ void __launch_bounds__(kBlk) k_bfs_claim(const uint64_t *q, uint64_t m, uint64_t id_lo, uint64_t n, const uint64_t *gs,
                                                    const uint64_t *valid, uint64_t *reg, uint64_t *seen, uint64_t *next,
                                                    unsigned long long *nn) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        const uint64_t li = (q[j] & kIdM) - id_lo;
        uint32_t pos = (uint32_t)(q[j] >> kIdxBits) & 0xFFFF;
        mark_group(gs, n, li, reg);
        while (pos) {
            const int b = __ffs(pos) - 1;
            pos &= pos - 1;
            const uint64_t y = li + b;
            if (y >= n || !bit_of(valid, y)) continue;
            const unsigned long long bit = 1ULL << (y & 63);
            if (atomicOr((unsigned long long *)&seen[y >> 6], bit) & bit) continue;
            next[atomicAdd(nn, 1ull)] = y;
        }
    }
}

// the region's edges of this rank as records {id, out_info, in_info, mult | valid << 16}
__global__ void __launch_bounds__(kBlk) k_region_list(const uint64_t *reg, uint64_t n, const uint64_t *wpre, uint64_t id_lo,
                                                      const uint64_t *out_info, const uint64_t *in_info, const uint16_t *mult,
                                                      const uint64_t *valid, uint64_t *rec) {
    const uint64_t nw = (n + 63) / 64, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw * 64; i += stride) {
        const uint64_t w = i >> 6, word = reg[w];
        if (!((word >> (i & 63)) & 1)) continue;
        const uint64_t c = wpre[w] + __popcll(word & ((1ULL << (i & 63)) - 1));
        rec[4 * c] = id_lo + i;
        rec[4 * c + 1] = out_info[i];
        rec[4 * c + 2] = in_info[i];
        rec[4 * c + 3] = (uint64_t)mult[i] | ((uint64_t)bit_of(valid, i) << 16);
    }
}
__global__ void __launch_bounds__(kBlk) k_word_popc64(const uint64_t *bm, uint64_t nw, uint64_t *cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) cnt[w] = __popcll(bm[w]);
}

__device__ __forceinline__ uint64_t find_sorted(const uint64_t *a, uint64_t n, uint64_t x) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo < n && a[lo] == x ? lo : kNo;
}

// the compact replica: ids, multiplicities, adjacency words with compact first ids (a window
// outside the region points at the all-invalid null group after the last edge)
__global__ void __launch_bounds__(kBlk) k_region_build(const uint64_t *rec, uint64_t rn, uint64_t *gid, uint16_t *mult,
                                                       uint64_t *out_info, uint64_t *in_info) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < rn; c += stride) gid[c] = rec[4 * c];
}
__global__ void __launch_bounds__(kBlk) k_region_words(const uint64_t *rec, uint64_t rn, const uint64_t *gid, uint16_t *mult,
                                                       uint64_t *out_info, uint64_t *in_info, uint64_t *valid) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (rn + 63) / 64, wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += wstride) {
        const uint64_t c = w * 64 + lane;
        bool v = false;
        if (c < rn) {
            const uint64_t oi = rec[4 * c + 1], ii = rec[4 * c + 2], mv = rec[4 * c + 3];
            mult[c] = (uint16_t)(mv & 0xFFFF);
            v = (mv >> 16) & 1;
            const uint64_t om = oi >> kIdxBits;
            uint64_t olo = rn;
            if (om) {
                const uint64_t f = find_sorted(gid, rn, oi & kIdM);
                olo = f == kNo ? rn : f;
            }
            out_info[c] = olo | (om << kIdxBits);
            const uint64_t im = ii >> kIdxBits;
            uint64_t iw = 0;
            if (im) {
                const uint64_t f = find_sorted(gid, rn, ii & kIdM);
                iw = (f == kNo ? rn : f) | (im << kIdxBits);
            }
            in_info[c] = iw;
        }
        const unsigned long long m = __ballot(v);
        if (lane == 0) valid[w] = m;
    }
}

// ---------------------------------------------------------------- host drivers
struct ShardCf {
    mcaat_graph *g;
    mcaat_ctx *ctx;
    Comm &comm;
    Router rt;
    Owners o;
    hipStream_t st;
    uint64_t n, nwl;
    unsigned grid(uint64_t m, unsigned cap_per_cu = 16) const { return grid_for(m, kBlk, (unsigned)ctx->n_cu * cap_per_cu); }
    ShardCf(mcaat_graph *gr, Comm &c)
        : g(gr), ctx(gr->ctx), comm(c), rt(gr->ctx, c), o(owners_of(gr, c)), st(gr->ctx->stream), n(gr->D_local),
          nwl((gr->D_local + 63) / 64) {}

    uint64_t sum(uint64_t v) {
        uint64_t t = 0;
        for (uint64_t x : comm.allgather_one(v)) t += x;
        return t;
    }

    // BFS of `rounds` hops from the frontier (local indices, already seen and marked)
    void bfs(DevBuf<uint64_t> &front, uint64_t nf, uint64_t rounds, bool backward, const uint64_t *gs, uint64_t *reg,
             uint64_t *seen) {
        DevBuf<unsigned long long> c(2);
        for (uint64_t h = 0; h < rounds; ++h) {
            if (sum(nf) == 0) break;
            DevBuf<uint64_t> q(nf ? nf : 1);
            DevBuf<uint8_t> dest(nf ? nf : 1);
            HIP_OK(hipMemsetAsync(c.p, 0, 16, st));
            if (nf) {
                hipLaunchKernelGGL(k_bfs_req, dim3(grid(nf)), dim3(kBlk), 0, st, (const uint64_t *)front.p, nf,
                                   (const uint64_t *)g->out_info.p, (const uint64_t *)g->in_info.p, (int)backward, o, q.p,
                                   dest.p, c.p);
                LAUNCH_OK();
            }
            const uint64_t nq = nf ? read_u64(ctx, c.p) : 0;
            Routed r;
            rt.send(q.p, 1, dest.p, nq, r, false);
            // each received window adds at most 16 edges
            DevBuf<uint64_t> next(16 * r.n_in + 1);
            if (r.n_in) {
                hipLaunchKernelGGL(k_bfs_claim, dim3(grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r.in.p, r.n_in,
                                   g->id_lo, n, gs, (const uint64_t *)g->valid.p, reg, seen, next.p, c.p + 1);
                LAUNCH_OK();
            }
            nf = r.n_in ? read_u64(ctx, c.p + 1) : 0;
            front = std::move(next);
        }
    }

    // every rank: the compact replica of the groups marked in reg on all ranks
    void gather_region(const uint64_t *reg, mcaat_graph *rg, std::vector<uint64_t> &hgid) {
        DevBuf<uint64_t> pc(nwl + 1), wpre(nwl + 1);
        HIP_OK(hipMemsetAsync(pc.p + nwl, 0, 8, st));
        uint64_t mine = 0;
        if (nwl) {
            hipLaunchKernelGGL(k_word_popc64, dim3(grid(nwl)), dim3(kBlk), 0, st, reg, nwl, pc.p);
            LAUNCH_OK();
            size_t tmp = 0;
            HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, pc.p, wpre.p, (size_t)(nwl + 1), st));
            DevBuf<uint8_t> t(tmp);
            HIP_OK(hipcub::DeviceScan::ExclusiveSum(t.p, tmp, pc.p, wpre.p, (size_t)(nwl + 1), st));
            d2h(ctx, &mine, wpre.p + nwl, 8);
        }
        DevBuf<uint64_t> rec(4 * (mine ? mine : 1));
        if (mine) {
            hipLaunchKernelGGL(k_region_list, dim3(grid(nwl * 64)), dim3(kBlk), 0, st, reg, n, (const uint64_t *)wpre.p,
                               g->id_lo, (const uint64_t *)g->out_info.p, (const uint64_t *)g->in_info.p,
                               (const uint16_t *)g->mult.p, (const uint64_t *)g->valid.p, rec.p);
            LAUNCH_OK();
        }
        const std::vector<uint64_t> per = comm.allgather_one(mine);
        uint64_t rn = 0;
        std::vector<uint64_t> bytes(comm.world);
        for (int r = 0; r < comm.world; ++r) rn += per[r], bytes[r] = 32 * per[r];
        DevBuf<uint64_t> all(4 * (rn ? rn : 1));
        HIP_OK(hipStreamSynchronize(st));
        if (rn) comm.allgatherv_dev(rec.p, all.p, bytes.data());
        // rank order = ascending ids (every rank's list ascends): compact id = position
        const uint64_t D = rn + 16;  // + the null group
        rg->ctx = ctx;
        rg->k = g->k;
        rg->D = D;
        rg->gid.alloc(D);
        rg->mult.alloc(mcaat_graph::mult_entries(D));
        rg->out_info.alloc(D);
        rg->in_info.alloc(D);
        rg->valid.alloc(mcaat_graph::bitmap_words(D));
        HIP_OK(hipMemsetAsync(rg->mult.p, 0, rg->mult.bytes(), st));
        HIP_OK(hipMemsetAsync(rg->out_info.p, 0, rg->out_info.bytes(), st));
        HIP_OK(hipMemsetAsync(rg->in_info.p, 0, rg->in_info.bytes(), st));
        HIP_OK(hipMemsetAsync(rg->valid.p, 0, rg->valid.bytes(), st));
        HIP_OK(hipMemsetAsync(rg->gid.p, 0xFF, rg->gid.bytes(), st));
        if (rn) {
            hipLaunchKernelGGL(k_region_build, dim3(grid(rn)), dim3(kBlk), 0, st, (const uint64_t *)all.p, rn, rg->gid.p,
                               rg->mult.p, rg->out_info.p, rg->in_info.p);
            LAUNCH_OK();
            hipLaunchKernelGGL(k_region_words, dim3(grid(rn)), dim3(kBlk), 0, st, (const uint64_t *)all.p, rn,
                               (const uint64_t *)rg->gid.p, rg->mult.p, rg->out_info.p, rg->in_info.p, rg->valid.p);
            LAUNCH_OK();
        }
        rg->all_valid = false;
        hgid.resize(rn);
        if (rn) d2h(ctx, hgid.data(), rg->gid.p, 8 * rn);
    }
};

std::vector<uint64_t> to_compact(const std::vector<uint64_t> &hgid, const std::vector<uint64_t> &ids) {
    std::vector<uint64_t> c(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
        auto it = std::lower_bound(hgid.begin(), hgid.end(), ids[i]);
        if (it == hgid.end() || *it != ids[i]) throw Error(MCAAT_E_INVALID, "per-shard CycleFinder: a start is outside its region");
        c[i] = (uint64_t)(it - hgid.begin());
    }
    return c;
}

}  // namespace

// ---------------------------------------------------------------- sharded adjacency
void sdbg_finish_sharded(mcaat_ctx *ctx, Comm &comm, mcaat_graph *g) {
    hipStream_t st = ctx->stream;
    const int k = g->k;
    const uint64_t n = g->D_local;
    // local radix directory over the range's keys (~8 edges per prefix)
    uint64_t kmin = 0, kmax = 0;
    if (n) {
        d2h(ctx, &kmin, g->key.p, 8);
        d2h(ctx, &kmax, g->key.p + n - 1, 8);
    }
    int shift = 0;
    const uint64_t want = std::max<uint64_t>(1, n / 8);
    while (((kmax - kmin) >> shift) + 1 > want) ++shift;
    const uint64_t np = ((kmax - kmin) >> shift) + 1;
    g->dir.alloc(np + 1);
    g->dir_shift = shift;
    g->dir_base = kmin;
    g->dir_n = np;
    hipLaunchKernelGGL(k_sdir, dim3(grid_for(n + 1, kBlk, (unsigned)ctx->n_cu * 16)), dim3(kBlk), 0, st, g->key.p, n, kmin,
                       shift, np, g->dir.p);
    LAUNCH_OK();
    g->out_info.alloc(n ? n : 1);
    g->in_info.alloc(n ? n : 1);
    Router rt(ctx, comm);
    const Owners o = owners_of(g, comm);
    // chunks of edges: two queries each; every rank takes part in as many exchanges
    const uint64_t chunk = (uint64_t)std::max<int64_t>(1024, knob(ctx, "dist.adj_chunk", 1LL << 27));
    uint64_t n_chunks = (n + chunk - 1) / chunk;
    for (uint64_t x : comm.allgather_one(n_chunks)) n_chunks = std::max(n_chunks, x);
    KernelTimer kt(ctx, "adjacency", 32.0 * (double)n);
    for (uint64_t c = 0; c < n_chunks; ++c) {
        const uint64_t i0 = std::min(n, c * chunk), m = std::min(n, i0 + chunk) - i0;
        DevBuf<uint64_t> q(2 * m + 1);
        DevBuf<uint8_t> dest(2 * m + 1);
        if (m) {
            hipLaunchKernelGGL(k_adj_queries, dim3(grid_for(m, kBlk, (unsigned)ctx->n_cu * 16)), dim3(kBlk), 0, st, g->key.p,
                               i0, m, k, o, q.p, dest.p);
            LAUNCH_OK();
        }
        Routed r;
        rt.send(q.p, 1, dest.p, 2 * m, r, true);
        DevBuf<uint64_t> ans(r.n_in + 1), a2(2 * m + 1);
        if (r.n_in) {
            hipLaunchKernelGGL(k_adj_answer, dim3(grid_for(r.n_in, kBlk, (unsigned)ctx->n_cu * 16)), dim3(kBlk), 0, st,
                               (const uint64_t *)g->key.p, n, g->id_lo, (const uint64_t *)g->dir.p, kmin, shift, np,
                               (const uint64_t *)r.in.p, r.n_in, ans.p);
            LAUNCH_OK();
        }
        rt.reply(r, ans.p, 1, a2.p);
        if (m) {
            hipLaunchKernelGGL(k_adj_store, dim3(grid_for(m, kBlk, (unsigned)ctx->n_cu * 16)), dim3(kBlk), 0, st,
                               (const uint64_t *)a2.p, i0, m, g->out_info.p, g->in_info.p);
            LAUNCH_OK();
        }
    }
    kt.stop();
    g->valid.alloc(mcaat_graph::bitmap_words(n));
    HIP_OK(hipMemsetAsync(g->valid.p, 0, g->valid.bytes(), st));
    if (n) {
        hipLaunchKernelGGL(k_ones, dim3(grid_for((n + 63) / 64, kBlk)), dim3(kBlk), 0, st, g->valid.p, n);
        LAUNCH_OK();
    }
    g->all_valid = true;
    HIP_OK(hipStreamSynchronize(st));
    if (verbose())
        fprintf(stderr, "[mcaat] shard %d: adjacency of %llu edges, %llu exchanges, %llu queries\n", comm.rank,
                (unsigned long long)n, (unsigned long long)rt.rounds, (unsigned long long)rt.records);
}

// ---------------------------------------------------------------- per-shard CycleFinder
void cycle_finder_sharded(mcaat_graph *g, const mcaat_cf_params &p, mcaat_cycles *out, Comm &comm) {
    mcaat_ctx *ctx = g->ctx;
    hipStream_t st = ctx->stream;
    StageTimer timer(ctx);
    if (!g->all_valid)
        throw Error(MCAAT_E_INVALID, "per-shard CycleFinder needs the graph as built (every edge valid); unshard it first");
    g->all_valid = false;
    ShardCf s(g, comm);
    const uint64_t n = s.n, nwl = s.nwl, id_lo = g->id_lo;
    DevBuf<unsigned long long> cnt(8);
    HIP_OK(hipMemsetAsync(cnt.p, 0, 64, st));

    // 1-2. CollectTips (fresh graph) and InvalidateMultiplicityOneNodes: local
    DevBuf<uint64_t> post(nwl + 1), seed(nwl + 1);
    HIP_OK(hipMemsetAsync(post.p + nwl, 0, 8, st));
    HIP_OK(hipMemsetAsync(seed.p + nwl, 0, 8, st));
    if (n) {
        hipLaunchKernelGGL(k_sh_filter, dim3(s.grid(nwl * 64)), dim3(kBlk), 0, st, (const uint16_t *)g->mult.p,
                           (const uint64_t *)g->out_info.p, n, post.p, seed.p, cnt.p);
        LAUNCH_OK();
    }
    // filtered out-windows and the candidates' in-windows from their owners
    DevBuf<uint8_t> kind(n + 4), stt(n + 4);
    DevBuf<uint64_t> nx(n ? n : 1), own(n ? n : 1);
    HIP_OK(hipMemsetAsync(kind.p, 0, kind.bytes(), st));
    DevBuf<uint64_t> cand(n ? n : 1);
    HIP_OK(hipMemsetAsync(cnt.p + 5, 0, 8, st));
    // chunks of local edges per exchange (every rank runs as many): bounded transient memory
    const uint64_t chunk = (uint64_t)std::max<int64_t>(1024, knob(ctx, "dist.adj_chunk", 1LL << 27));
    uint64_t n_chunks = (n + chunk - 1) / chunk;
    for (uint64_t x : comm.allgather_one(n_chunks)) n_chunks = std::max(n_chunks, x);
    for (uint64_t c = 0; c < n_chunks; ++c) {
        const uint64_t a0 = std::min(n, c * chunk), a1 = std::min(n, a0 + chunk), m = a1 - a0;
        DevBuf<uint64_t> q(2 * m + 1), src(2 * m + 1);
        DevBuf<uint8_t> dest(2 * m + 1);
        HIP_OK(hipMemsetAsync(cnt.p + 4, 0, 8, st));
        if (m) {
            hipLaunchKernelGGL(k_win_req, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint64_t *)post.p,
                               (const uint16_t *)g->mult.p, (const uint64_t *)g->out_info.p, (const uint64_t *)g->in_info.p,
                               a0, a1, (uint64_t)p.threshold_multiplicity, s.o, q.p, dest.p, src.p, cnt.p + 4);
            LAUNCH_OK();
        }
        const uint64_t nq = m ? read_u64(ctx, cnt.p + 4) : 0;
        Routed r;
        s.rt.send(q.p, 1, dest.p, nq, r, true);
        DevBuf<uint64_t> ans(r.n_in + 1), a(nq + 1);
        if (r.n_in) {
            hipLaunchKernelGGL(k_win_ans, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)post.p, n, id_lo,
                               (const uint64_t *)r.in.p, r.n_in, ans.p);
            LAUNCH_OK();
        }
        s.rt.reply(r, ans.p, 1, a.p);
        if (nq) {
            hipLaunchKernelGGL(k_win_apply, dim3(s.grid(nq)), dim3(kBlk), 0, st, (const uint64_t *)src.p,
                               (const uint64_t *)a.p, nq, (const uint64_t *)g->out_info.p, (const uint64_t *)g->in_info.p,
                               id_lo, kind.p, nx.p, cand.p, cnt.p + 5);
            LAUNCH_OK();
        }
    }
    const uint64_t ncand = read_u64(ctx, cnt.p + 5);
    // predecessor flags, as messages to the successors' owners (after every window is in)
    for (uint64_t c = 0; c < n_chunks; ++c) {
        const uint64_t a0 = std::min(n, c * chunk), a1 = std::min(n, a0 + chunk), m = a1 - a0;
        DevBuf<uint64_t> q(4 * m + 1);
        DevBuf<uint8_t> dest(4 * m + 1);
        HIP_OK(hipMemsetAsync(cnt.p + 4, 0, 8, st));
        if (m) {
            hipLaunchKernelGGL(k_flag_msgs, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint64_t *)post.p,
                               (const uint64_t *)seed.p, (const uint8_t *)kind.p, (const uint64_t *)g->out_info.p, a0, a1,
                               s.o, q.p, dest.p, cnt.p + 4, cnt.p);
            LAUNCH_OK();
        }
        const uint64_t nq = m ? read_u64(ctx, cnt.p + 4) : 0;
        Routed r;
        s.rt.send(q.p, 1, dest.p, nq, r, false);
        if (r.n_in) {
            hipLaunchKernelGGL(k_flag_apply, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r.in.p, r.n_in,
                               id_lo, kind.p);
            LAUNCH_OK();
        }
    }
    unsigned long long hc[4];
    d2h(ctx, hc, cnt.p, 32);
    {
        const auto all = comm.allgather_vec(std::vector<uint64_t>{hc[0], hc[1], hc[2]});
        out->stats[0] = out->stats[1] = out->stats[3] = 0;
        for (int r = 0; r < comm.world; ++r)
            out->stats[0] += all[3 * r], out->stats[1] += all[3 * r + 1], out->stats[3] += all[3 * r + 2];
    }
    timer.mark("tips_filter");

    // 3. RecursiveReduction: rulers, walks, pointer jumping, branch resolution, removal
    const uint64_t rmask = (uint64_t)std::max<int64_t>(0, knob(ctx, "dist.ruler_mask", 15));
    DevBuf<uint64_t> rl(n ? n : 1), bl(n ? n : 1);
    HIP_OK(hipMemsetAsync(own.p, 0xFF, own.bytes(), st));
    HIP_OK(hipMemsetAsync(cnt.p + 4, 0, 16, st));
    if (n) {
        hipLaunchKernelGGL(k_prep, dim3(s.grid(n)), dim3(kBlk), 0, st, (const uint64_t *)post.p, (const uint64_t *)seed.p,
                           kind.p, stt.p, n, id_lo, rmask, rl.p, cnt.p + 4, bl.p, cnt.p + 5);
        LAUNCH_OK();
    }
    uint64_t nr = 0, nb = 0;
    {
        unsigned long long h2[2];
        d2h(ctx, h2, cnt.p + 4, 16);
        nr = h2[0];
        nb = h2[1];
    }
    uint64_t walk_rounds = 0;
    {
        DevBuf<uint64_t> w(4 * (nr ? nr : 1));
        if (nr) {
            hipLaunchKernelGGL(k_walk_init, dim3(s.grid(nr)), dim3(kBlk), 0, st, (const uint64_t *)rl.p, nr,
                               (const uint64_t *)nx.p, id_lo, w.p);
            LAUNCH_OK();
        }
        uint64_t m = nr;
        for (;; ++walk_rounds) {
            DevBuf<uint64_t> o4(4 * (m ? m : 1));
            DevBuf<uint8_t> dest(m ? m : 1);
            HIP_OK(hipMemsetAsync(cnt.p + 6, 0, 8, st));
            if (m) {
                hipLaunchKernelGGL(k_walk, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint64_t *)w.p, m,
                                   (const uint8_t *)kind.p, nx.p, own.p, s.o, o4.p, dest.p, cnt.p + 6);
                LAUNCH_OK();
            }
            const uint64_t mo = m ? read_u64(ctx, cnt.p + 6) : 0;
            Routed r;
            s.rt.send(o4.p, 4, dest.p, mo, r, false);
            if (!r.total) break;
            w = std::move(r.in);
            m = r.n_in;
        }
    }
    // pointer jumping over the rulers still pointing at a ruler
    uint64_t jump_rounds = 0;
    {
        DevBuf<uint64_t> al(nr ? nr : 1), al2(nr ? nr : 1);
        HIP_OK(hipMemsetAsync(cnt.p + 6, 0, 8, st));
        if (nr) {
            hipLaunchKernelGGL(k_active_rulers, dim3(s.grid(nr)), dim3(kBlk), 0, st, (const uint64_t *)rl.p, nr,
                               (const uint64_t *)nx.p, al.p, cnt.p + 6);
            LAUNCH_OK();
        }
        uint64_t na = nr ? read_u64(ctx, cnt.p + 6) : 0;
        const uint64_t total_rulers = s.sum(nr);
        int bound = 2;
        while ((1ULL << bound) < total_rulers + 1) ++bound;
        bound += 1;
        for (; jump_rounds < (uint64_t)bound; ++jump_rounds) {
            if (s.sum(na) == 0) break;
            DevBuf<uint64_t> q(na ? na : 1);
            DevBuf<uint8_t> dest(na ? na : 1);
            if (na) {
                hipLaunchKernelGGL(k_jump_req, dim3(s.grid(na)), dim3(kBlk), 0, st, (const uint64_t *)al.p, na,
                                   (const uint64_t *)nx.p, s.o, q.p, dest.p);
                LAUNCH_OK();
            }
            Routed r;
            s.rt.send(q.p, 1, dest.p, na, r, true);
            DevBuf<uint64_t> ans(r.n_in + 1), a(na + 1);
            if (r.n_in) {
                hipLaunchKernelGGL(k_jump_ans, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r.in.p, r.n_in,
                                   (const uint64_t *)nx.p, id_lo, ans.p);
                LAUNCH_OK();
            }
            s.rt.reply(r, ans.p, 1, a.p);
            HIP_OK(hipMemsetAsync(cnt.p + 6, 0, 8, st));
            if (na) {
                hipLaunchKernelGGL(k_jump_apply, dim3(s.grid(na)), dim3(kBlk), 0, st, (const uint64_t *)al.p, na,
                                   (const uint64_t *)a.p, nx.p, al2.p, cnt.p + 6);
                LAUNCH_OK();
            }
            na = na ? read_u64(ctx, cnt.p + 6) : 0;
            std::swap(al, al2);
        }
        // still pointing at a ruler after the bound: a unary cycle (or a chain into one) survives
        if (na) {
            hipLaunchKernelGGL(k_jump_cycle, dim3(s.grid(na)), dim3(kBlk), 0, st, (const uint64_t *)al.p, na, nx.p);
            LAUNCH_OK();
        }
    }
    // branch successors' references (two lookups: the successor, then a passing ruler's terminal)
    DevBuf<uint64_t> ref(4 * (nb ? nb : 1));  // per branch slot: its successor's reference, kPad unused
    if (nb) {
        hipLaunchKernelGGL(k_fill, dim3(s.grid(4 * nb)), dim3(kBlk), 0, st, ref.p, 4 * nb, kPad);
        LAUNCH_OK();
    }
    {
        DevBuf<uint64_t> q(4 * nb + 1), src(4 * nb + 1);
        DevBuf<uint8_t> dest(4 * nb + 1);
        HIP_OK(hipMemsetAsync(cnt.p + 6, 0, 8, st));
        if (nb) {
            hipLaunchKernelGGL(k_bref_req, dim3(s.grid(nb)), dim3(kBlk), 0, st, (const uint64_t *)bl.p, nb,
                               (const uint8_t *)kind.p, (const uint64_t *)g->out_info.p, s.o, q.p, dest.p, src.p, cnt.p + 6);
            LAUNCH_OK();
        }
        const uint64_t nq = nb ? read_u64(ctx, cnt.p + 6) : 0;
        Routed r;
        s.rt.send(q.p, 1, dest.p, nq, r, true);
        DevBuf<uint64_t> ans(r.n_in + 1), a(nq + 1);
        if (r.n_in) {
            hipLaunchKernelGGL(k_bref_ans, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r.in.p, r.n_in,
                               (const uint8_t *)kind.p, (const uint64_t *)nx.p, (const uint64_t *)own.p, id_lo, ans.p);
            LAUNCH_OK();
        }
        s.rt.reply(r, ans.p, 1, a.p);
        if (nq) {
            hipLaunchKernelGGL(k_scatter_ref, dim3(s.grid(nq)), dim3(kBlk), 0, st, (const uint64_t *)src.p,
                               (const uint64_t *)a.p, nq, ref.p);
            LAUNCH_OK();
        }
        // second step: a passing ruler's terminal
        HIP_OK(hipMemsetAsync(cnt.p + 6, 0, 8, st));
        if (nb) {
            hipLaunchKernelGGL(k_bref_req2, dim3(s.grid(4 * nb)), dim3(kBlk), 0, st, (const uint64_t *)ref.p, 4 * nb, s.o,
                               q.p, dest.p, src.p, cnt.p + 6);
            LAUNCH_OK();
        }
        const uint64_t nq2 = nb ? read_u64(ctx, cnt.p + 6) : 0;
        Routed r2;
        s.rt.send(q.p, 1, dest.p, nq2, r2, true);
        DevBuf<uint64_t> ans2(r2.n_in + 1), a2(nq2 + 1);
        if (r2.n_in) {
            hipLaunchKernelGGL(k_jump_ans, dim3(s.grid(r2.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r2.in.p, r2.n_in,
                               (const uint64_t *)nx.p, id_lo, ans2.p);
            LAUNCH_OK();
        }
        s.rt.reply(r2, ans2.p, 1, a2.p);
        if (nq2) {
            hipLaunchKernelGGL(k_scatter_ref, dim3(s.grid(nq2)), dim3(kBlk), 0, st, (const uint64_t *)src.p,
                               (const uint64_t *)a2.p, nq2, ref.p);
            LAUNCH_OK();
        }
    }
    // branch resolution rounds (until no branch changes on any rank)
    uint64_t res_rounds = 0;
    {
        DevBuf<uint64_t> q(4 * nb + 1), src(4 * nb + 1);
        DevBuf<uint8_t> dest(4 * nb + 1), slot_st(4 * nb + 4);
        for (;; ++res_rounds) {
            HIP_OK(hipMemsetAsync(cnt.p + 6, 0, 16, st));
            if (nb) {
                hipLaunchKernelGGL(k_res_req, dim3(s.grid(nb)), dim3(kBlk), 0, st, (const uint64_t *)bl.p,
                                   (const uint64_t *)ref.p, nb, stt.p, s.o, q.p, dest.p, src.p, cnt.p + 6, cnt.p + 7);
                LAUNCH_OK();
            }
            unsigned long long h2[2] = {0, 0};
            if (nb) d2h(ctx, h2, cnt.p + 6, 16);
            Routed r;
            s.rt.send(q.p, 1, dest.p, h2[0], r, true);
            DevBuf<uint64_t> ans(r.n_in + 1), a(h2[0] + 1);
            if (r.n_in) {
                hipLaunchKernelGGL(k_st_ans, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r.in.p, r.n_in,
                                   (const uint8_t *)stt.p, id_lo, ans.p);
                LAUNCH_OK();
            }
            s.rt.reply(r, ans.p, 1, a.p);
            // padding slots read as removed (they never keep a branch alive)
            if (nb) HIP_OK(hipMemsetAsync(slot_st.p, kStRem, 4 * nb, st));
            if (h2[0]) {
                hipLaunchKernelGGL(k_slot_st, dim3(s.grid(h2[0])), dim3(kBlk), 0, st, (const uint64_t *)src.p,
                                   (const uint64_t *)a.p, h2[0], slot_st.p);
                LAUNCH_OK();
            }
            if (nb) {
                hipLaunchKernelGGL(k_res_apply, dim3(s.grid(nb)), dim3(kBlk), 0, st, (const uint64_t *)bl.p, nb,
                                   (const uint8_t *)slot_st.p, stt.p, cnt.p + 7);
                LAUNCH_OK();
            }
            const uint64_t ch = nb ? read_u64(ctx, cnt.p + 7) : 0;
            if (s.sum(ch) == 0) break;
        }
    }
    // removal: resolved non-unary edges, rulers whose terminal went, and the chains they walked
    uint64_t n_rm_rulers = 0;
    {
        if (nwl) {
            hipLaunchKernelGGL(k_rm_nonunary, dim3(s.grid(nwl * 64)), dim3(kBlk), 0, st, (const uint64_t *)post.p,
                               (const uint8_t *)kind.p, (const uint8_t *)stt.p, n, g->valid.p);
            LAUNCH_OK();
        }
        DevBuf<uint64_t> q(nr + 1), src(nr + 1);
        DevBuf<uint8_t> dest(nr + 1);
        HIP_OK(hipMemsetAsync(cnt.p + 6, 0, 16, st));
        if (nr) {
            hipLaunchKernelGGL(k_term_req, dim3(s.grid(nr)), dim3(kBlk), 0, st, (const uint64_t *)rl.p, nr,
                               (const uint64_t *)nx.p, s.o, q.p, dest.p, src.p, cnt.p + 6);
            LAUNCH_OK();
        }
        const uint64_t nq = nr ? read_u64(ctx, cnt.p + 6) : 0;
        Routed r;
        s.rt.send(q.p, 1, dest.p, nq, r, true);
        DevBuf<uint64_t> ans(r.n_in + 1), a(nq + 1);
        if (r.n_in) {
            hipLaunchKernelGGL(k_st_ans, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r.in.p, r.n_in,
                               (const uint8_t *)stt.p, id_lo, ans.p);
            LAUNCH_OK();
        }
        s.rt.reply(r, ans.p, 1, a.p);
        DevBuf<uint64_t> rm(nq + 1);
        if (nq) {
            hipLaunchKernelGGL(k_rm_rulers, dim3(s.grid(nq)), dim3(kBlk), 0, st, (const uint64_t *)src.p,
                               (const uint64_t *)a.p, nq, id_lo, g->valid.p, rm.p, cnt.p + 7);
            LAUNCH_OK();
        }
        const uint64_t nrm = nq ? read_u64(ctx, cnt.p + 7) : 0;
        const std::vector<uint64_t> per = comm.allgather_one(nrm);
        std::vector<uint64_t> bytes(comm.world);
        for (int r2 = 0; r2 < comm.world; ++r2) n_rm_rulers += per[r2], bytes[r2] = 8 * per[r2];
        if (n_rm_rulers) {
            DevBuf<uint64_t> allrm(n_rm_rulers);
            HIP_OK(hipStreamSynchronize(st));
            comm.allgatherv_dev(rm.p, allrm.p, bytes.data());
            const uint64_t cap = next_pow2(2 * n_rm_rulers + 16);
            DevBuf<uint64_t> tab(cap);
            HIP_OK(hipMemsetAsync(tab.p, 0xFF, tab.bytes(), st));
            hipLaunchKernelGGL(k_set_build, dim3(s.grid(n_rm_rulers)), dim3(kBlk), 0, st, (const uint64_t *)allrm.p,
                               n_rm_rulers, tab.p, cap);
            LAUNCH_OK();
            if (nwl) {
                hipLaunchKernelGGL(k_rm_chains, dim3(s.grid(nwl * 64)), dim3(kBlk), 0, st, (const uint64_t *)post.p,
                                   (const uint8_t *)kind.p, (const uint64_t *)own.p, n, (const uint64_t *)tab.p, cap,
                                   g->valid.p);
                LAUNCH_OK();
            }
        }
        HIP_OK(hipStreamSynchronize(st));
    }
    if (verbose())
        fprintf(stderr,
                "[mcaat] shard %d peel: %llu rulers, %llu branches; walk %llu rounds, jumps %llu, resolution %llu; "
                "%llu removed rulers\n",
                comm.rank, (unsigned long long)nr, (unsigned long long)nb, (unsigned long long)walk_rounds,
                (unsigned long long)jump_rounds, (unsigned long long)res_rounds, (unsigned long long)n_rm_rulers);
    kind.release();
    stt.release();
    own.release();
    rl.release();
    bl.release();
    ref.release();
    seed.release();
    timer.mark("peel");

    // 4-5. valid count; the candidates still valid, ascending on every rank
    HIP_OK(hipMemsetAsync(cnt.p, 0, 16, st));
    if (nwl) {
        hipLaunchKernelGGL(k_popc, dim3(s.grid(nwl)), dim3(kBlk), 0, st, (const uint64_t *)g->valid.p, nwl, cnt.p);
        LAUNCH_OK();
    }
    out->stats[2] = s.sum(read_u64(ctx, cnt.p));
    std::vector<uint64_t> cand_mine;
    DevBuf<uint64_t> kept(ncand + 1);
    uint64_t nkept = 0;
    if (ncand) {
        hipLaunchKernelGGL(k_cand_keep, dim3(s.grid(ncand)), dim3(kBlk), 0, st, (const uint64_t *)cand.p, ncand,
                           (const uint64_t *)g->valid.p, id_lo, kept.p, cnt.p + 1);
        LAUNCH_OK();
        nkept = read_u64(ctx, cnt.p + 1);
        cand_mine.resize(nkept);
        if (nkept) d2h(ctx, cand_mine.data(), kept.p, 8 * nkept);
        std::sort(cand_mine.begin(), cand_mine.end());
    }
    cand.release();
    post.release();
    timer.mark("recount");

    // 6. search regions: groups of the (k-1)-suffix (whole nodes' out-edges and in-groups)
    DevBuf<uint64_t> gs(nwl + 1), reg(nwl + 1), seen(nwl + 1);
    HIP_OK(hipMemsetAsync(gs.p, 0, gs.bytes(), st));
    if (nwl) {
        hipLaunchKernelGGL(k_gstart, dim3(s.grid(nwl * 64)), dim3(kBlk), 0, st, (const uint64_t *)g->key.p, n, gs.p);
        LAUNCH_OK();
    }
    const uint64_t radius = (uint64_t)p.cycle_max_length + 1;
    auto forward_region = [&](const std::vector<uint64_t> &starts_mine) {
        HIP_OK(hipMemsetAsync(reg.p, 0, reg.bytes(), st));
        HIP_OK(hipMemsetAsync(seen.p, 0, seen.bytes(), st));
        const uint64_t m = starts_mine.size();
        DevBuf<uint64_t> ids(m + 1), front(m + 1);
        if (m) {
            h2d(ctx, ids.p, starts_mine.data(), 8 * m);
            hipLaunchKernelGGL(k_bfs_seed, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint64_t *)ids.p, m, id_lo, n,
                               (const uint64_t *)gs.p, reg.p, seen.p, front.p);
            LAUNCH_OK();
        }
        s.bfs(front, m, radius, false, gs.p, reg.p, seen.p);
    };
    // DepthLevelSearch region: valid edges within cycle_max_length + 1 hops of the candidates
    forward_region(cand_mine);
    mcaat_graph rg;
    std::vector<uint64_t> hgid;
    s.gather_region(reg.p, &rg, hgid);
    const std::vector<uint64_t> cand_all = [&] {
        std::vector<uint64_t> a = comm.allgather_vec(cand_mine);
        std::sort(a.begin(), a.end());
        return a;
    }();
    timer.mark("candidates");
    if (verbose())
        fprintf(stderr, "[mcaat] shard %d: %zu candidates, DLS region %llu edges\n", comm.rank, cand_all.size(),
                (unsigned long long)hgid.size());
    ctx->kstats["shard_dls_region_edges"].launches = hgid.size();
    std::vector<uint64_t> pass_c = cf_depth_level_search(&rg, to_compact(hgid, cand_all), p.cycle_max_length, &comm);
    // buckets by ceil(log2 mult) (cycle_finder.cpp:414), descending; ascending ids within
    std::map<int, std::vector<uint64_t>, std::greater<int>> chunks;
    if (!pass_c.empty()) {
        std::vector<uint16_t> hm(rg.D);
        d2h(ctx, hm.data(), rg.mult.p, 2 * rg.D);
        for (uint64_t c : pass_c) chunks[(int)std::ceil(std::log2(double(hm[c])))].push_back(hgid[c]);
    }
    std::vector<uint64_t> starts;
    for (auto &kv : chunks)
        for (uint64_t id : kv.second) {
            out->cand_ids.push_back(id);
            out->cand_bucket.push_back(kv.first);
            starts.push_back(id);
        }
    out->stats[4] = out->cand_ids.size();
    rg = mcaat_graph{};
    timer.mark("dls");

    // 7. FindCycle region: forward cycle_max_length + 1 hops from the starts, then backward as
    // many from every edge reached (the lock relaxation's reach)
    {
        std::vector<uint64_t> sm;
        for (uint64_t x : starts)
            if (x >= id_lo && x < id_lo + n) sm.push_back(x);
        std::sort(sm.begin(), sm.end());
        forward_region(sm);
        // the backward BFS starts from every edge the forward one reached
        DevBuf<uint64_t> pc(nwl + 1), wpre(nwl + 1);
        HIP_OK(hipMemsetAsync(pc.p + nwl, 0, 8, st));
        uint64_t nseen = 0;
        if (nwl) {
            hipLaunchKernelGGL(k_word_popc64, dim3(s.grid(nwl)), dim3(kBlk), 0, st, (const uint64_t *)seen.p, nwl, pc.p);
            LAUNCH_OK();
            size_t tmp = 0;
            HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, pc.p, wpre.p, (size_t)(nwl + 1), st));
            DevBuf<uint8_t> t(tmp);
            HIP_OK(hipcub::DeviceScan::ExclusiveSum(t.p, tmp, pc.p, wpre.p, (size_t)(nwl + 1), st));
            d2h(ctx, &nseen, wpre.p + nwl, 8);
        }
        DevBuf<uint64_t> front(nseen + 1);
        if (nseen) {
            // local indices of the seen edges, via the list kernel's id column
            DevBuf<uint64_t> rec(4 * nseen);
            hipLaunchKernelGGL(k_region_list, dim3(s.grid(nwl * 64)), dim3(kBlk), 0, st, (const uint64_t *)seen.p, n,
                               (const uint64_t *)wpre.p, (uint64_t)0, (const uint64_t *)g->out_info.p,
                               (const uint64_t *)g->in_info.p, (const uint16_t *)g->mult.p, (const uint64_t *)g->valid.p,
                               rec.p);
            LAUNCH_OK();
            std::vector<uint64_t> h(4 * nseen), li(nseen);
            d2h(ctx, h.data(), rec.p, 32 * nseen);
            for (uint64_t j = 0; j < nseen; ++j) li[j] = h[4 * j];
            h2d(ctx, front.p, li.data(), 8 * nseen);
        }
        s.bfs(front, nseen, radius, true, gs.p, reg.p, seen.p);
    }
    mcaat_graph fg;
    std::vector<uint64_t> fgid;
    s.gather_region(reg.p, &fg, fgid);
    reg.release();
    seen.release();
    gs.release();
    ctx->kstats["shard_fc_region_edges"].launches = fgid.size();
    if (verbose())
        fprintf(stderr, "[mcaat] shard %d: %zu FindCycle starts, region %llu edges; %llu exchanges, %llu records\n",
                comm.rank, starts.size(), (unsigned long long)fgid.size(), (unsigned long long)s.rt.rounds,
                (unsigned long long)s.rt.records);
    ctx->kstats["shard_exchanges"].launches = s.rt.rounds;
    mcaat_cycles local;
    cf_find_cycles(&fg, p, to_compact(fgid, starts), &local, &comm);
    for (size_t i = 0; i < local.starts.size(); ++i) {
        out->starts.push_back(fgid[local.starts[i]]);
        std::vector<uint64_t> fl(local.flat[i].size());
        for (size_t j = 0; j < fl.size(); ++j) fl[j] = fgid[local.flat[i][j]];
        out->flat.push_back(std::move(fl));
        out->offsets.push_back(std::move(local.offsets[i]));
    }
    out->stats[5] = local.stats[5];
    out->stats[6] = local.stats[6];
    out->stats[7] = local.stats[7];
    timer.mark("find_cycle");
    HIP_OK(hipStreamSynchronize(st));
    timer.finish();
}

// ---------------------------------------------------------------- unshard
__global__ void __launch_bounds__(kBlk) k_splice_bits(const uint64_t *loc, const uint64_t *loc_w0, const uint64_t *rank_lo, int N,
                                                      uint64_t D, uint64_t *out) {
    const uint64_t nw = (D + 63) / 64, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
        uint64_t v = 0;
        for (int b = 0; b < 64; ++b) {
            const uint64_t x = w * 64 + b;
            if (x >= D) break;
            int r = 0;
            while (r + 1 < N && rank_lo[r + 1] <= x) ++r;
            const uint64_t li = x - rank_lo[r];
            v |= ((loc[loc_w0[r] + (li >> 6)] >> (li & 63)) & 1) << b;
        }
        out[w] = v;
    }
}

void graph_unshard(mcaat_graph *g, Comm &comm) {
    if (!g->sharded) return;
    mcaat_ctx *ctx = g->ctx;
    hipStream_t st = ctx->stream;
    const int N = comm.world;
    const uint64_t D = g->D, n = g->D_local, nwl = (n + 63) / 64;
    std::vector<uint64_t> b8(N), b2(N), bw(N), w0(N + 1, 0);
    for (int r = 0; r < N; ++r) {
        const uint64_t nr = g->rank_lo[r + 1] - g->rank_lo[r];
        b8[r] = 8 * nr;
        b2[r] = 2 * nr;
        bw[r] = 8 * ((nr + 63) / 64);
        w0[r + 1] = w0[r] + (nr + 63) / 64;
    }
    DevBuf<uint64_t> key(D ? D : 1);
    DevBuf<uint16_t> mult(mcaat_graph::mult_entries(D));
    DevBuf<uint64_t> locv(w0[N] + 1);
    HIP_OK(hipStreamSynchronize(st));
    comm.allgatherv_dev(g->key.p, key.p, b8.data());
    comm.allgatherv_dev(g->mult.p, mult.p, b2.data());
    comm.allgatherv_dev(g->valid.p, locv.p, bw.data());
    (void)nwl;
    const bool all_valid = g->all_valid;
    g->sharded = false;
    g->key = std::move(key);
    g->mult = std::move(mult);
    g->out_info.release();
    g->in_info.release();
    g->dir.release();
    g->id_lo = 0;
    g->D_local = 0;
    sdbg_finish(ctx, g);  // the whole graph's directory and adjacency on every rank
    if (!all_valid) {
        DevBuf<uint64_t> dw0(N + 1), drl(N + 1);
        HIP_OK(hipMemcpyAsync(dw0.p, w0.data(), 8 * (N + 1), hipMemcpyHostToDevice, st));
        HIP_OK(hipMemcpyAsync(drl.p, g->rank_lo.data(), 8 * (N + 1), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_splice_bits, dim3(grid_for((D + 63) / 64, kBlk)), dim3(kBlk), 0, st, (const uint64_t *)locv.p,
                           (const uint64_t *)dw0.p, (const uint64_t *)drl.p, N, D, g->valid.p);
        LAUNCH_OK();
        g->all_valid = false;
        HIP_OK(hipStreamSynchronize(st));
    }
    g->rank_lo.clear();
    g->key_split.clear();
}

}  // namespace mcaat
