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
#include <chrono>
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
// (round 5, target-range windows) two or more filter-valid unary predecessors: the only edges
// two ruler walks can both reach, so the only ones a walk claims by compare-and-swap
constexpr uint8_t kMerge = 0x80;
constexpr uint8_t kStUnk = 0, kStRem = 1, kStSurv = 2;
constexpr uint64_t kPad = kNo - 1;  // an unused successor slot of a branch
// (round 5) the successor word of a unary edge carries the edge's own walk kind, so a walk step
// reads one scattered word instead of the kind byte and the word: kChain on every unary edge that
// is not a ruler (set with the successor, cleared on rulers by k_prep), kMergeW where several
// unary chains meet (walks claim it by compare-and-swap)
constexpr uint64_t kChain = 1ULL << 59, kMergeW = 1ULL << 58;
__device__ __forceinline__ bool is_chain(uint64_t v) { return v < kPad && (v & kChain) && !(v & (kRef | (1ULL << 61))); }

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
// Request / message slots of W 64-bit words, each with a destination rank (kNoDest: an empty
// slot), go to their ranks in one all-to-all. The grouping by destination is atomic-free and
// deterministic: the slots are cut into one contiguous range per block, every block counts its
// range's destinations with wave ballots, one small kernel turns the per-block counts into
// per-block send offsets, and the scatter ranks each slot among its block's slots of the same
// destination (ballot + mbcnt). The placement is stable (slot order within a destination), so the
// answers, which come back in the order the owner received the requests, are gathered into their
// slots by walking the same offsets again (no permutation array).
constexpr uint8_t kNoDest = 0xFF;
constexpr int kRBlocks = 1024;  // most blocks of a routing pass (the offsets kernel scans them in one block)

// the slots' destination bytes, eight per thread at a time (each byte compared to d with a
// zero-byte test): per-block counts per destination, no atomics
__device__ __forceinline__ uint32_t bytes_equal(uint64_t x, uint32_t d) {
    const uint64_t y = x ^ (0x0101010101010101ULL * d);
    return (uint32_t)__popcll(~(((y & 0x7F7F7F7F7F7F7F7FULL) + 0x7F7F7F7F7F7F7F7FULL) | y | 0x7F7F7F7F7F7F7F7FULL));
}
__global__ void __launch_bounds__(kBlk) k_route_count(const uint8_t *dest, uint64_t n, uint64_t per, int N, uint32_t *cnt) {
    __shared__ uint32_t h[64];
    for (int q = threadIdx.x; q < N; q += blockDim.x) h[q] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = min(n, b0 + per);  // b0 is a multiple of 8
    uint32_t c[64];
    for (int q = 0; q < N; ++q) c[q] = 0;
    for (uint64_t t = b0 + 8 * (uint64_t)threadIdx.x; t < b1; t += 8 * (uint64_t)kBlk) {
        uint64_t x;
        if (t + 8 <= b1) {
            x = *(const uint64_t *)(dest + t);
        } else {
            x = ~0ULL;  // kNoDest padding
            for (uint64_t i = t; i < b1; ++i) x = (x & ~(0xFFULL << (8 * (i - t)))) | ((uint64_t)dest[i] << (8 * (i - t)));
        }
        for (int q = 0; q < N; ++q) c[q] += bytes_equal(x, (uint32_t)q);
    }
    for (int q = 0; q < N; ++q) {
        uint32_t v = c[q];
        for (int o = 32; o; o >>= 1) v += __shfl_down(v, o);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(&h[q], v);
    }
    __syncthreads();
    for (int q = threadIdx.x; q < N; q += blockDim.x) cnt[(uint64_t)blockIdx.x * N + q] = h[q];
}

// base[b * N + d] = where block b's slots for destination d start in the send buffer
// (destinations back to back, blocks in order within one); tot[d] = all slots for d
__global__ void __launch_bounds__(1024) k_route_offsets(const uint32_t *cnt, int G, int N, uint64_t *base, uint64_t *tot) {
    __shared__ uint64_t sc[1024];
    __shared__ uint64_t run;
    if (threadIdx.x == 0) run = 0;
    __syncthreads();
    for (int d = 0; d < N; ++d) {
        const uint64_t v = (int)threadIdx.x < G ? cnt[(uint64_t)threadIdx.x * N + d] : 0;
        sc[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan
            const uint64_t x = threadIdx.x >= (unsigned)o ? sc[threadIdx.x - o] : 0;
            __syncthreads();
            sc[threadIdx.x] += x;
            __syncthreads();
        }
        if ((int)threadIdx.x < G) base[(uint64_t)threadIdx.x * N + d] = run + sc[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 0) {
            tot[d] = sc[1023];
            run += sc[1023];
        }
        __syncthreads();
    }
}

// kRT slots per thread per tile: fewer barriers per slot; a slot's send position depends only on
// the slots before it (stable within a destination), so the same walk also gathers the answers
// back in slot order (GATHER: out[slot] = back[position]) without a permutation array
constexpr int kRT = 8;
// self: this rank; its records are placed straight into the receive buffer (self_buf, from
// position self_pos0 of the send order) and its answers gathered from there, so the exchange
// copies nothing for them
template <bool GATHER>
__global__ void __launch_bounds__(kBlk) k_route_place(const uint64_t *rec, int W, const uint8_t *dest, uint64_t n,
                                                      uint64_t per, int N, const uint64_t *base, uint64_t *out,
                                                      int self, uint64_t *self_buf, uint64_t self_pos0) {
    __shared__ uint64_t run[64];
    __shared__ uint32_t tile_tot[64];
    __shared__ uint32_t wc[kRT * (kBlk / 64)][64];  // per (u, wave): counts, then exclusive prefixes
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = min(n, b0 + per);
    if (threadIdx.x < N) run[threadIdx.x] = base[(uint64_t)blockIdx.x * N + threadIdx.x];
    __syncthreads();
    for (uint64_t t = b0; t < b1; t += (uint64_t)kBlk * kRT) {
        int d[kRT];
        uint32_t rank[kRT];
#pragma unroll
        for (int u = 0; u < kRT; ++u) {
            const uint64_t i = t + (uint64_t)u * kBlk + threadIdx.x;
            d[u] = i < b1 ? dest[i] : kNoDest;
        }
#pragma unroll
        for (int u = 0; u < kRT; ++u) {
            uint32_t c = 0;
            rank[u] = 0;
            for (int q = 0; q < N; ++q) {
                const unsigned long long m = __ballot(d[u] == q);
                if (d[u] == q) rank[u] = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                if (lane == q) c = (uint32_t)__popcll(m);
            }
            wc[u * (kBlk / 64) + wave][lane] = c;
        }
        __syncthreads();
        // slot order is (u, wave, lane): exclusive prefix over (u, wave) per destination
        if (threadIdx.x < N) {
            uint32_t acc = 0;
            for (int k = 0; k < kRT * (kBlk / 64); ++k) {
                const uint32_t v = wc[k][threadIdx.x];
                wc[k][threadIdx.x] = acc;
                acc += v;
            }
            tile_tot[threadIdx.x] = acc;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kRT; ++u) {
            if (d[u] == kNoDest) continue;
            const uint64_t i = t + (uint64_t)u * kBlk + threadIdx.x;
            const uint64_t pos = run[d[u]] + wc[u * (kBlk / 64) + wave][d[u]] + rank[u];
            if (GATHER) {
                const uint64_t *src = d[u] == self ? self_buf + (pos - self_pos0) * W : rec + pos * W;
                for (int x = 0; x < W; ++x) out[i * W + x] = src[x];
            } else {
                uint64_t *dst = d[u] == self ? self_buf + (pos - self_pos0) * W : out + pos * W;
                for (int x = 0; x < W; ++x) dst[x] = rec[i * W + x];
            }
        }
        __syncthreads();
        if (threadIdx.x < N) run[threadIdx.x] += tile_tot[threadIdx.x];
        __syncthreads();
    }
}

__global__ void k_set_word(uint64_t *p, uint64_t v) { *p = v; }

struct Routed {
    int W = 1;
    uint64_t n = 0, sent = 0, n_in = 0, total = 0;  // slots, records sent, received, sent by all ranks
    std::vector<uint64_t> out_cnt, in_cnt;
    const uint8_t *dest = nullptr;  // the slots' destinations (reply: the caller keeps them alive)
    DevBuf<uint64_t> base;          // per (block, destination) send offsets (reply walks them again)
    uint64_t per = 0;
    int G = 0;
    std::vector<uint64_t> out_off, in_off;  // prefix sums of out_cnt / in_cnt
    DevBuf<uint64_t> in;            // received records, sources in rank order
};

struct Router {
    mcaat_ctx *ctx;
    Comm &comm;
    uint64_t rounds = 0, records = 0;  // collectives and records moved (diagnostics)
    // host time per part of a round (MCAAT_VERBOSE diagnostics): grouping kernels + count read,
    // count all-gather, placement + sync, all-to-all, reply
    double t_count = 0, t_gather = 0, t_place = 0, t_a2a = 0, t_reply = 0;
    static double now() {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    Router(mcaat_ctx *c, Comm &cm) : ctx(c), comm(cm) {}

    // n slots (rec: n x W words; dest[i] a rank or kNoDest). keep: a reply follows (dest must
    // stay valid until it). Records for this rank go straight to the receive buffer.
    // extra_sum: the sum over the ranks of `extra`, carried in the same count all-gather (a loop's
    // global condition without a collective of its own)
    void send(const uint64_t *rec, int W, const uint8_t *dest, uint64_t n, Routed &rt, bool keep,
              uint64_t extra = 0, uint64_t *extra_sum = nullptr) {
        hipStream_t st = ctx->stream;
        const int N = comm.world, R = comm.rank;
        rt.W = W;
        rt.n = n;
        rt.dest = dest;
        rt.out_cnt.assign(N, 0);
        rt.per = std::max<uint64_t>(kBlk * kRT, ((n + kRBlocks - 1) / kRBlocks + kBlk * kRT - 1) / (kBlk * kRT) * (kBlk * kRT));
        rt.G = n ? (int)((n + rt.per - 1) / rt.per) : 0;
        DevBuf<uint32_t> cnt((uint64_t)std::max(rt.G, 1) * N);
        rt.base.alloc((uint64_t)std::max(rt.G, 1) * N);
        const int NW = N + (extra_sum ? 1 : 0);
        DevBuf<uint64_t> tot(NW);
        if (extra_sum) {
            hipLaunchKernelGGL(k_set_word, dim3(1), dim3(1), 0, st, tot.p + N, extra);
            LAUNCH_OK();
        }
        double t0 = now();
        if (n) {
            hipLaunchKernelGGL(k_route_count, dim3(rt.G), dim3(kBlk), 0, st, dest, n, rt.per, N, cnt.p);
            LAUNCH_OK();
            hipLaunchKernelGGL(k_route_offsets, dim3(1), dim3(1024), 0, st, (const uint32_t *)cnt.p, rt.G, N, rt.base.p, tot.p);
            LAUNCH_OK();
        } else {
            HIP_OK(hipMemsetAsync(tot.p, 0, 8 * N, st));
        }
        double t1 = now();
        t_count += t1 - t0;
        // every rank's send counts straight from the device (one read of the gathered matrix)
        std::vector<uint64_t> mat;
        comm.allgather_dev_words(tot.p, NW, mat);
        if (extra_sum) {  // back to the N x N count matrix, the extra words summed
            std::vector<uint64_t> m2((uint64_t)N * N);
            *extra_sum = 0;
            for (int r = 0; r < N; ++r) {
                for (int q = 0; q < N; ++q) m2[(uint64_t)r * N + q] = mat[(uint64_t)r * NW + q];
                *extra_sum += mat[(uint64_t)r * NW + N];
            }
            mat.swap(m2);
        }
        for (int q = 0; q < N; ++q) rt.out_cnt[q] = mat[(uint64_t)R * N + q];
        rt.sent = 0;
        for (uint64_t x : rt.out_cnt) rt.sent += x;
        t0 = now();
        t_gather += t0 - t1;
        rt.in_cnt.assign(N, 0);
        rt.n_in = rt.total = 0;
        for (int s2 = 0; s2 < N; ++s2) {
            rt.in_cnt[s2] = mat[(uint64_t)s2 * N + R];
            rt.n_in += rt.in_cnt[s2];
            for (int d = 0; d < N; ++d) rt.total += mat[(uint64_t)s2 * N + d];
        }
        rt.out_off.assign(N + 1, 0);
        rt.in_off.assign(N + 1, 0);
        for (int q = 0; q < N; ++q) {
            rt.out_off[q + 1] = rt.out_off[q] + rt.out_cnt[q];
            rt.in_off[q + 1] = rt.in_off[q] + rt.in_cnt[q];
        }
        rt.in.alloc((rt.n_in ? rt.n_in : 1) * W);
        // the send buffer has a hole where this rank's own records would be (they go to rt.in)
        DevBuf<uint64_t> sendb((N > 1 && rt.sent ? rt.sent : 1) * W);
        if (rt.sent) {
            hipLaunchKernelGGL(k_route_place<false>, dim3(rt.G), dim3(kBlk), 0, st, rec, W, dest, n, rt.per, N,
                               (const uint64_t *)rt.base.p, sendb.p, R, rt.in.p + rt.in_off[R] * W, rt.out_off[R]);
            LAUNCH_OK();
        }
        if (!keep) rt.base.release();
        std::vector<uint64_t> sb(N), rb(N), so(N), ro(N);
        for (int q = 0; q < N; ++q) {
            sb[q] = 8ULL * W * rt.out_cnt[q], rb[q] = 8ULL * W * rt.in_cnt[q];
            so[q] = 8ULL * W * rt.out_off[q], ro[q] = 8ULL * W * rt.in_off[q];
        }
        sb[R] = rb[R] = 0;  // placed already
        // (the transports order the exchange after the placement on the context stream: RCCL
        // queues on it, the shared-memory transport synchronises it first)
        t1 = now();
        t_place += t1 - t0;
        if (N > 1) comm.alltoallv_dev(sendb.p, sb.data(), rt.in.p, rb.data(), so.data(), ro.data());
        t_a2a += now() - t1;
        ++rounds;
        records += rt.sent;
    }
    // answers (Wa words per received record, in received order) back to their slots: out[slot * Wa ..]
    // (slots without a request keep what out held); this rank's own answers are read in place
    void reply(Routed &rt, uint64_t *ans, int Wa, uint64_t *out) {
        const double t0 = now();
        struct Acc {
            double &t;
            double t0;
            ~Acc() { t += now() - t0; }
        } acc{t_reply, t0};
        hipStream_t st = ctx->stream;
        const int N = comm.world, R = comm.rank;
        DevBuf<uint64_t> back((N > 1 && rt.sent ? rt.sent : 1) * Wa);
        std::vector<uint64_t> sb(N), rb(N), so(N), ro(N);
        for (int q = 0; q < N; ++q) {
            sb[q] = 8ULL * Wa * rt.in_cnt[q], rb[q] = 8ULL * Wa * rt.out_cnt[q];
            so[q] = 8ULL * Wa * rt.in_off[q], ro[q] = 8ULL * Wa * rt.out_off[q];
        }
        sb[R] = rb[R] = 0;  // read in place
        if (N > 1) comm.alltoallv_dev(ans, sb.data(), back.p, rb.data(), so.data(), ro.data());
        if (rt.sent) {
            hipLaunchKernelGGL(k_route_place<true>, dim3(rt.G), dim3(kBlk), 0, st, (const uint64_t *)back.p, Wa, rt.dest,
                               rt.n, rt.per, N, (const uint64_t *)rt.base.p, out, R, ans + rt.in_off[R] * Wa,
                               rt.out_off[R]);
            LAUNCH_OK();
        }
        // (no synchronise: `out` is read by kernels or d2h on the same stream)
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

// ---- adjacency by key ranges (round 5, default; dist.adj_ranges=0 keeps the queries above) ----
// For each W the targets (W, s[1..k-1]) of a sorted run of sources lie in one key range
// (sdbg_build.hip k_adjacency_own), so rank r's sources target the global id ranges
// O_W(r) = [lb((W, key[rank_lo[r]] >> 4) << 2), the same for rank r + 1) (rank 0 from the W
// quarter's start, the last rank to its end), which tile [0, D) over (r, W), and every
// predecessor of an edge in O_W(r) is a source of rank r (groups do not straddle ranks). So
// rank r fetches the keys of its four ranges from their owners (contiguous slices, one
// all-to-all per W), computes out_info of its edges and in_info of its ranges exactly as one
// GPU does per run (LDS-staged, group-aligned runs), and returns the in_info slices to their
// owners: 16 B per edge over the links, against four 8-B words of queries and answers per edge.
__global__ void __launch_bounds__(kBlk) k_count_less(const uint64_t *key, uint64_t n, const uint64_t *qs, int nq,
                                                     uint64_t *out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq) return;
    const uint64_t q = qs[t];
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (key[mid] < q) lo = mid + 1;
        else hi = mid;
    }
    out[t] = lo;
}

struct TgtRanges {  // this rank's four target ranges O_W(r), fetched
    const uint64_t *key[4];  // their keys
    uint64_t *in[4];         // their in_info words, computed here
    uint64_t len[4];
    uint64_t g0[4];          // global id of the first
};

__device__ __forceinline__ uint64_t lb_arr(const uint64_t *a, uint64_t n, uint64_t q) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < q) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

constexpr int kRunT = 1024, kRunB = 2048, kRunMax = kRunB + 16, kRunCap = 3072;
// bounds[5 r] = local start of run r (group aligned), bounds[5 r + 1 + W] = its first owned
// position in range W; r = nruns: n and the range ends
__global__ void __launch_bounds__(kBlk) k_run_bounds(const uint64_t *key, uint64_t n, int k, TgtRanges T, uint64_t nruns,
                                                     uint64_t *bounds) {
    const uint64_t top = (uint64_t)1 << (2 * (k - 1));
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= nruns; r += stride) {
        uint64_t s = r * kRunB;
        if (r == nruns || s >= n) s = n;
        else if (s > 0) {
            const uint64_t g0 = key[s - 1] >> 4;
            while (s < n && (key[s] >> 4) == g0) ++s;
        }
        bounds[5 * r] = s;
        for (int W = 0; W < 4; ++W) {
            uint64_t b;
            if (r == 0) b = 0;
            else if (s >= n) b = T.len[W];
            else b = lb_arr(T.key[W], T.len[W], (((uint64_t)W * top) | (key[s] >> 4)) << 2);
            bounds[5 * r + 1 + W] = b;
        }
    }
}

__global__ void __launch_bounds__(kRunT) k_adj_ranges(const uint64_t *key, uint64_t id_lo, int k, TgtRanges T,
                                                      const uint64_t *bounds, uint64_t *out_info) {
    __shared__ uint64_t own[kRunMax];
    __shared__ uint64_t okey[kRunCap];
    __shared__ uint64_t ist[kRunCap];
    const uint64_t r = blockIdx.x;
    const uint64_t s0 = bounds[5 * r], s1 = bounds[5 * (r + 1)];
    uint64_t a[4];
    uint32_t len[4], off[4], tot = 0;
#pragma unroll
    for (int W = 0; W < 4; ++W) {
        a[W] = bounds[5 * r + 1 + W];
        len[W] = (uint32_t)(bounds[5 * (r + 1) + 1 + W] - a[W]);
        off[W] = tot;
        tot += len[W];
    }
    const uint32_t n = (uint32_t)(s1 - s0);
    const bool staged = tot <= (uint32_t)kRunCap;
    for (uint32_t j = threadIdx.x; j < n; j += kRunT) own[j] = key[s0 + j];
#pragma unroll
    for (int W = 0; W < 4; ++W)
        for (uint32_t i = threadIdx.x; i < len[W]; i += kRunT) {
            if (staged) {
                okey[off[W] + i] = T.key[W][a[W] + i];
                ist[off[W] + i] = 0;
            } else {
                T.in[W][a[W] + i] = 0;
            }
        }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < n; j += kRunT) {
        const uint64_t K = own[j];
        const uint32_t W = (uint32_t)(K & 3);
        const uint64_t Rt = ((uint64_t)W << (2 * (k - 1))) | (K >> 4), qk = Rt << 2;
        uint64_t lo;
        unsigned m = 0;
        if (staged) {
            const uint64_t *rk = okey + off[W];
            const uint32_t x = (uint32_t)lb_arr(rk, len[W], qk);
            lo = a[W] + x;
            for (uint32_t i = x; i < len[W] && (rk[i] >> 2) == Rt; ++i) m |= 1u << (rk[i] & 3);
        } else {
            lo = lb_arr(T.key[W], T.len[W], qk);
            for (uint64_t i = lo; i < T.len[W] && (T.key[W][i] >> 2) == Rt; ++i) m |= 1u << (T.key[W][i] & 3);
        }
        out_info[s0 + j] = (T.g0[W] + lo) | ((uint64_t)m << kIdxBits);
        if (!m) continue;
        const uint64_t gk = K >> 4;
        uint32_t gs = j;
        while (gs > 0 && (own[gs - 1] >> 4) == gk) --gs;
        unsigned pm = 0;
        int t = 0;
        for (uint32_t q = gs; q < n && (own[q] >> 4) == gk && t < 16; ++q, ++t)
            if ((own[q] & 3) == W) pm |= 1u << t;
        if ((uint32_t)(__ffs(pm) - 1) != j - gs) continue;  // another in-edge of the node writes
        const uint64_t v = (id_lo + s0 + gs) | ((uint64_t)pm << kIdxBits);
        const int deg = __popc(m);
        if (staged)
            for (int q = 0; q < deg; ++q) ist[off[W] + (uint32_t)(lo - a[W]) + q] = v;
        else
            for (int q = 0; q < deg; ++q) T.in[W][lo + q] = v;
    }
    if (!staged) return;
    __syncthreads();
#pragma unroll
    for (int W = 0; W < 4; ++W)
        for (uint32_t i = threadIdx.x; i < len[W]; i += kRunT) T.in[W][a[W] + i] = ist[off[W] + i];
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

// window requests, two slots per local edge of the chunk [a0, a1): slot 2j asks the 16
// filtered bits at its target node's first edge (a filter-valid edge with out-edges), slot 2j+1
// its predecessor group's (a filter-valid edge above the threshold: ChunkStartNodes' in-degree)
__global__ void __launch_bounds__(kBlk) k_win_req(const uint64_t *post, const uint16_t *mult, const uint64_t *out_info,
                                                  const uint64_t *in_info, uint64_t a0, uint64_t a1, uint64_t thr, Owners o,
                                                  uint64_t *q, uint8_t *dest) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a1 - a0; j += stride) {
        const uint64_t i = a0 + j;
        const bool pv = bit_of(post, i);
        const uint64_t oi = pv ? out_info[i] : 0;
        const uint64_t ii = pv && (uint64_t)mult[i] > thr ? in_info[i] : 0;
        q[2 * j] = oi & kIdM;
        dest[2 * j] = (oi >> kIdxBits) & 0xF ? (uint8_t)owner_of_id(o, oi & kIdM) : kNoDest;
        q[2 * j + 1] = ii & kIdM;
        dest[2 * j + 1] = (ii >> kIdxBits) ? (uint8_t)owner_of_id(o, ii & kIdM) : kNoDest;
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
__global__ void __launch_bounds__(kBlk) k_win_apply(const uint8_t *dest, const uint64_t *ans, uint64_t a0, uint64_t a1,
                                                    const uint64_t *out_info, const uint64_t *in_info, uint64_t id_lo,
                                                    uint8_t *kind, uint64_t *nx, uint64_t *cbits) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a1 - a0; j += stride) {
        const uint64_t i = a0 + j;
        if (dest[2 * j] != kNoDest) {
            const uint64_t oi = out_info[i];
            const int cnt = __popc((unsigned)(oi >> kIdxBits) & 0xF);
            const uint32_t pm = (uint32_t)ans[2 * j] & ((1u << cnt) - 1);
            kind[i] = (uint8_t)pm;  // the flag bits come later (k_flag_apply)
            if (__popc(pm) == 1) nx[i] = ((oi & kIdM) + (uint64_t)(__ffs(pm) - 1)) | kChain;
        }
        if (dest[2 * j + 1] != kNoDest) {
            const uint64_t ii = in_info[i], l = ii & kIdM, e = id_lo + i;
            const uint32_t in = (uint32_t)ans[2 * j + 1] & (uint32_t)((ii >> kIdxBits) & 0xFFFF);
            const bool self = e >= l && e - l < 16 && ((in >> (e - l)) & 1);
            if (__popc(in) >= 2 && !self)  // _IncomingNotEqualToCurrentNode, indegree >= 2
                atomicOr((unsigned long long *)&cbits[i >> 6], 1ULL << (i & 63));
        }
    }
}

// ---- the windows and flags by target ranges (round 5, default; dist.win_ranges=0: messages) ----
// The filtered out-window of an edge lies in its target range, so the owners' filter bits of the
// four ranges are pulled once (a byte per edge); what an edge tells its successors (unary /
// branch predecessor flags) and ChunkStartNodes' in-degree test of a node (decided by its
// predecessor group, which lives with the group's rank) are computed for the ranges' edges
// here and pushed to their owners as one byte per edge.
constexpr uint8_t kCandPre = 0x80, kMultiPre = 0x01;
__device__ __forceinline__ void or_byte(uint8_t *a, uint64_t i, uint32_t v) {
    atomicOr((unsigned int *)(a + (i & ~3ULL)), v << (8 * (i & 3)));
}  // pushed byte: the node's filter-valid in-degree test passed
struct TgtBytes {
    const uint8_t *pb[4];  // filter bits of the range's edges (pulled)
    uint8_t *tf[4];        // flag / candidate bytes for them (pushed)
    uint64_t g0[4];
    uint64_t len[4];
};

__global__ void __launch_bounds__(kBlk) k_post_bytes(const uint64_t *post, uint64_t n, uint8_t *pb) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) pb[i] = (uint8_t)bit_of(post, i);
}

// kind (filtered out-window) and the unary successor of every filter-valid edge
__global__ void __launch_bounds__(kBlk) k_out_win(const uint64_t *post, const uint64_t *key, const uint64_t *out_info,
                                                  uint64_t n, TgtBytes T, uint8_t *kind, uint64_t *nx) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (!bit_of(post, i)) continue;
        const uint64_t oi = out_info[i];
        const int cnt = __popc((unsigned)(oi >> kIdxBits) & 0xF);
        uint32_t pm = 0;
        if (cnt) {
            const int W = (int)(key[i] & 3);
            const uint8_t *b = T.pb[W] + ((oi & kIdM) - T.g0[W]);
            for (int q = 0; q < cnt; ++q) pm |= (uint32_t)b[q] << q;
            kind[i] = (uint8_t)pm;
        }
        // every filter-valid edge's word is written: a walk reads the word first
        nx[i] = __popc(pm) == 1 ? ((oi & kIdM) + (uint64_t)(__ffs(pm) - 1)) | kChain : kNo;
    }
}

// per local edge: post-filter tips that are not seeds (counts[2]); per group (its first edge) and
// W of the group: the W-edges share their target node, hence their filtered out-window pm, so the
// node's edges get, from this group alone (their only predecessor group), the predecessor flag of
// the filter-valid W-edges (unary or branch by popc(pm)) on the pm positions and ChunkStartNodes'
// in-degree test (at least two filter-valid predecessors, the node not one of them:
// _IncomingNotEqualToCurrentNode) — one plain byte store per target edge, no atomics
__global__ void __launch_bounds__(kBlk) k_push_bytes(const uint64_t *post, const uint64_t *seed, const uint64_t *key,
                                                     const uint64_t *out_info, const uint8_t *kind, uint64_t n,
                                                     uint64_t id_lo, TgtBytes T, unsigned long long *cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long tpf = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t K = key[i];
        if (bit_of(post, i) && (kind[i] & 0xF) == 0 && !bit_of(seed, i)) ++tpf;
        if (i > 0 && (key[i - 1] >> 4) == (K >> 4)) continue;  // not its group's first edge
        uint32_t inw[4] = {0, 0, 0, 0};
        uint64_t first[4] = {kNo, kNo, kNo, kNo}, valid_w[4] = {kNo, kNo, kNo, kNo};
        for (int t = 0; t < 16 && i + t < n; ++t) {
            const uint64_t x = key[i + t];
            if ((x >> 4) != (K >> 4)) break;
            const int W = (int)(x & 3);
            if (first[W] == kNo) first[W] = i + t;
            if (bit_of(post, i + t)) {
                inw[W] |= 1u << t;
                if (valid_w[W] == kNo) valid_w[W] = i + t;
            }
        }
        const uint64_t gs = id_lo + i;
        for (int W = 0; W < 4; ++W) {
            if (first[W] == kNo) continue;
            const uint64_t oi = out_info[first[W]];
            const int deg = __popc((unsigned)(oi >> kIdxBits) & 0xF);
            const uint64_t lo = oi & kIdM;
            const uint32_t pm = valid_w[W] != kNo ? kind[valid_w[W]] & 0xF : 0;
            const uint8_t flag = __popc(pm) == 1 ? kUpred : kBpred;
            const bool many = __popc(inw[W]) >= 2;
            for (int q = 0; q < deg; ++q) {
                const uint64_t t = lo + q;
                uint8_t b = (pm >> q) & 1 ? flag : 0;
                if (b == kUpred && __popc(inw[W]) >= 2) b |= kMultiPre;  // a merge of unary chains
                if (many && !(t >= gs && t - gs < 16 && ((inw[W] >> (t - gs)) & 1))) b |= kCandPre;
                if (b) T.tf[W][t - T.g0[W]] = b;
            }
        }
    }
    block_add(cnt + 2, tpf);
}

// the pushed bytes of the local edges: predecessor flags into kind, the in-degree test into the
// candidate bits (with the edge's own conditions: filter-valid, above the threshold)
__global__ void __launch_bounds__(kBlk) k_recv_bytes(const uint8_t *inb, const uint64_t *post, const uint16_t *mult,
                                                     uint64_t thr, uint64_t n, uint8_t *kind, uint64_t *nx, uint64_t *cbits) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (n + 63) / 64, wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += wstride) {
        const uint64_t i = w * 64 + lane;
        bool c = false;
        if (i < n) {
            const uint8_t b = inb[i];
            if (b & (kUpred | kBpred)) {
                const uint8_t k = kind[i];
                kind[i] = k | (b & (kUpred | kBpred)) | (b & kMultiPre ? kMerge : 0);
                if ((b & kMultiPre) && __popc(k & 0xF) == 1) nx[i] |= kMergeW;
            }
            c = (b & kCandPre) && bit_of(post, i) && (uint64_t)mult[i] > thr;
        }
        const unsigned long long m = __ballot(c);
        if (lane == 0) cbits[w] = m;
    }
}

// post-filter tips that are not seeds (counts[2]); predecessor flags as messages to the
// successors, four slots per local edge: id | 1 << 62 from a unary edge, id | 1 << 63 from a branch
__global__ void __launch_bounds__(kBlk) k_flag_msgs(const uint64_t *post, const uint64_t *seed, const uint8_t *kind,
                                                    const uint64_t *out_info, uint64_t a0, uint64_t a1, Owners o,
                                                    uint64_t *q, uint8_t *dest, unsigned long long *cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long tpf = 0;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a1 - a0; j += stride) {
        const uint64_t i = a0 + j;
        const bool pv = bit_of(post, i);
        const uint32_t pm = pv ? kind[i] & 0xF : 0;
        const int od = __popc(pm);
        if (pv && od == 0 && !bit_of(seed, i)) ++tpf;
        const uint64_t lo = pv ? out_info[i] & kIdM : 0;
        for (int b = 0; b < 4; ++b) {
            const uint64_t y = lo + b;
            q[4 * j + b] = y | (od == 1 ? (1ULL << 62) : (1ULL << 63));
            dest[4 * j + b] = (pm >> b) & 1 ? (uint8_t)owner_of_id(o, y) : kNoDest;
        }
    }
    block_add(cnt + 2, tpf);
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
                                               uint64_t *nx, uint64_t n, uint64_t id_lo, uint64_t rmask, uint64_t *rbits,
                                               uint64_t *bbits) {
    const int lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < ((n + 63) & ~63ULL); i0 += stride) {
        const uint64_t i = i0 + threadIdx.x;
        const bool pv = i < n && bit_of(post, i);
        const uint8_t k = pv ? kind[i] : 0;
        const int od = __popc(k & 0xF);
        const bool ruler = pv && od == 1 && (!(k & kUpred) || (mix64((id_lo + i) ^ 0x5eed) & rmask) == 0);
        const bool branch = pv && od >= 2;
        if (pv) {
            if (ruler) {
                kind[i] = k | kRuler;
                nx[i] &= kIdM;  // a ruler's word is its successor, then its jump
            }
            st[i] = od == 0 ? (bit_of(seed, i) ? kStRem : kStSurv) : kStUnk;
        }
        const unsigned long long rm = __ballot(ruler), bm = __ballot(branch);
        if (lane == 0) {
            rbits[i >> 6] = rm;
            bbits[i >> 6] = bm;
        }
    }
}

// the set bits of a local bitmap as a list of local indices (wpre: exclusive prefix of the words' popcounts)
__global__ void __launch_bounds__(kBlk) k_bits_list(const uint64_t *bm, uint64_t nw, const uint64_t *wpre, uint64_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw * 64; i += stride) {
        const uint64_t w = i >> 6, word = bm[w];
        if ((word >> (i & 63)) & 1) out[wpre[w] + __popcll(word & ((1ULL << (i & 63)) - 1))] = i;
    }
}

// a search region's ids: the position of each edge id in the region's ascending gid list (its
// compact id; ~0 when it is not in the region), and back (~0 for positions past the list);
// grid-stride (ShardCf::grid caps the grid)
__global__ void __launch_bounds__(kBlk) k_gid_find(const uint64_t *gid, uint64_t rn, const uint64_t *ids, uint64_t m,
                                                   uint64_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
        const uint64_t x = ids[i];
        uint64_t lo = 0, hi = rn;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (gid[mid] < x) lo = mid + 1;
            else hi = mid;
        }
        out[i] = (lo < rn && gid[lo] == x) ? lo : ~0ULL;
    }
}
__global__ void __launch_bounds__(kBlk) k_gid_of(const uint64_t *gid, uint64_t rn, const uint64_t *c, uint64_t m,
                                                 uint64_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride)
        out[i] = c[i] < rn ? gid[c[i]] : ~0ULL;
}
__global__ void __launch_bounds__(kBlk) k_mult_of(const uint16_t *mult, const uint64_t *c, uint64_t m, uint16_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) out[i] = mult[c[i]];
}

// walkers: {ruler, edge}; results: {ruler | 1 << 63, reached} (reached: a non-unary edge, kRef |
// a ruler, or kNo on a unary cycle). A walker claims each non-ruler unary edge it passes by
// swapping its successor word for kOwn | ruler (compare-and-swap: one claimer per edge); a
// walker that meets an edge claimed by another ruler r1 stops with kRef | r1 (both chains go on
// identically from there, so r1's terminal is its terminal), one that meets its own claim has
// gone round a unary cycle without a ruler (kNo: survives). The claims are also the chain
// edges' owners for the removal, so there is no owner array and merging chains walk once.
constexpr uint64_t kResult = 1ULL << 63;
constexpr uint64_t kOwn = 1ULL << 61;
__device__ __forceinline__ bool is_claim(uint64_t v) { return v < kPad && !(v & kRef) && (v & kOwn); }

__global__ void __launch_bounds__(kBlk) k_walk_init(const uint64_t *rl, uint64_t nr, const uint64_t *nx, uint64_t id_lo,
                                                    uint64_t *w) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nr; j += stride) {
        const uint64_t i = rl[j];
        w[2 * j] = id_lo + i;
        w[2 * j + 1] = nx[i];
    }
}

// one record of a walk round: a result lands in its ruler's jump word (nx of the ruler: a walk
// stops at a ruler before reading its word); a walker advances over this rank's edges and leaves
// for the owner of the next one, or ends with a result for its ruler's owner. Returns whether a
// record goes out (to rank `to`, as {r, x})
__device__ __forceinline__ bool walk_one(uint64_t &r, uint64_t &x, const uint8_t *kind, uint64_t *nx, const Owners &o,
                                         int merge_known, int &to) {
    if (r & kResult) {
        nx[(r & kIdM) - o.id_lo] = x;
        return false;
    }
    for (;;) {
        if (x < o.id_lo || x >= o.id_lo + o.n) {  // leaves for the owner of x
            to = owner_of_id(o, x);
            return true;
        }
        const uint64_t li = x - o.id_lo;
        uint64_t v = nx[li];
        bool done = true;
        if (is_chain(v)) {  // a unary edge, not a ruler, unclaimed
            const uint64_t own = kOwn | r;
            if (merge_known && !(v & kMergeW)) {
                nx[li] = own;  // one unary predecessor: no other walk comes here
                x = v & kIdM;
                done = false;
            } else {
                const uint64_t prev = atomicCAS((unsigned long long *)&nx[li], v, own);
                if (prev == v) {
                    x = v & kIdM;  // claimed: on to the successor
                    done = false;
                } else {
                    v = prev;  // another walk's claim
                }
            }
        }
        if (done) {
            uint64_t res;
            if (is_claim(v)) {
                res = (v & kIdM) == r ? kNo : (kRef | (v & kIdM));
            } else {
                const uint8_t k = kind[li];  // once per walk: where it ends
                res = __popc(k & 0xF) != 1 ? x : (kRef | x);  // a non-unary edge or a ruler
            }
            to = owner_of_id(o, r);
            r |= kResult;
            x = res;
            return true;
        }
    }
}

__global__ void __launch_bounds__(kBlk) k_walk(const uint64_t *in, uint64_t m, const uint8_t *kind, uint64_t *nx, Owners o,
                                               uint64_t *out, uint8_t *dest, int merge_known) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        uint64_t r = in[2 * j], x = in[2 * j + 1];
        int to = 0;
        const bool emit = walk_one(r, x, kind, nx, o, merge_known, to);
        out[2 * j] = r;  // one output slot per input record
        out[2 * j + 1] = x;
        dest[j] = emit ? (uint8_t)to : kNoDest;
    }
}

// (round 6) the walk's tail in fixed blocks (once every rank's records in flight fit one block):
// the records of every source block (blockIdx.y; this rank's own from self_in) walk, and what goes
// out lands in the destination's block of `send` or in self_out (word 0 of a block: its records)
__global__ void __launch_bounds__(kBlk) k_walk_fx(const uint64_t *recv, const uint64_t *self_in, int R, uint64_t P,
                                                  const uint8_t *kind, uint64_t *nx, Owners o, uint64_t *send,
                                                  uint64_t *self_out, int merge_known) {
    const int src = blockIdx.y;
    const uint64_t *blk = src == R ? self_in : recv + (uint64_t)src * (1 + 2 * P);
    const uint64_t m = blk[0];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < m; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        uint64_t r = 0, x = 0;
        int to = -1;
        if (j < m) {
            r = blk[1 + 2 * j];
            x = blk[2 + 2 * j];
            if (!walk_one(r, x, kind, nx, o, merge_known, to)) to = -1;
        }
        unsigned long long pend = __ballot(to >= 0);
        while (pend) {
            const int lead = __ffsll((long long)pend) - 1;
            const int dd = __shfl(to, lead);
            const unsigned long long mk = __ballot(to == dd);
            uint64_t *ob = dd == R ? self_out : send + (uint64_t)dd * (1 + 2 * P);
            uint64_t base = 0;
            if ((int)(threadIdx.x & 63) == lead) base = atomicAdd((unsigned long long *)ob, (unsigned long long)__popcll(mk));
            base = __shfl(base, lead);
            if (to == dd) {
                // (records never multiply: a block holds every record in flight when the tail began)
                const uint64_t at = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0));
                ob[1 + 2 * at] = r;
                ob[2 + 2 * at] = x;
            }
            pend &= ~mk;
        }
    }
}
// zero the counts of N blocks of `stride` words, and of one more block
__global__ void k_blk_zero(uint64_t *blocks, int N, uint64_t stride, uint64_t *one) {
    const int t = threadIdx.x;
    if (t < N) blocks[(uint64_t)t * stride] = 0;
    if (t == 0 && one) one[0] = 0;
}
// a routed round's received records (n of them) into the own block of the tail's first round
__global__ void __launch_bounds__(kBlk) k_walk_fx_seed(const uint64_t *in, uint64_t n, uint64_t *self_blk) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < 2 * n; j += stride) self_blk[1 + j] = in[j];
    if (blockIdx.x == 0 && threadIdx.x == 0) self_blk[0] = n;
}
// the records one round put out on this rank (every block's count), added into *tot
__global__ void k_walk_fx_count(const uint64_t *send, int N, int R, uint64_t P, const uint64_t *self_out,
                                unsigned long long *tot) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        unsigned long long t = self_out[0];
        for (int q = 0; q < N; ++q)
            if (q != R) t += send[(uint64_t)q * (1 + 2 * P)];
        *tot = t;
    }
}

// pointer jumping: requests of the rulers still pointing at a ruler
// (round 5) a target on this rank is answered here at once (kNoDest: the slot keeps it); the
// round stays Jacobi, as every rank's apply follows the round's exchange
__global__ void __launch_bounds__(kBlk) k_jump_req(const uint64_t *al, uint64_t na, const uint64_t *nx, Owners o, uint64_t *q,
                                                   uint8_t *dest) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < na; j += stride) {
        const uint64_t t = nx[al[j]] & kIdM;
        if (t >= o.id_lo && t < o.id_lo + o.n) {
            q[j] = nx[t - o.id_lo];
            dest[j] = kNoDest;
        } else {
            q[j] = t;
            dest[j] = (uint8_t)owner_of_id(o, t);
        }
    }
}
__global__ void __launch_bounds__(kBlk) k_jump_ans(const uint64_t *q, uint64_t m, const uint64_t *nx, uint64_t id_lo, uint64_t *ans) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) ans[j] = nx[q[j] - id_lo];
}
// the new jumps; keep[j]: ruler j still points at a ruler
__global__ void __launch_bounds__(kBlk) k_jump_apply(const uint64_t *al, uint64_t na, const uint64_t *a, uint64_t *nx,
                                                     uint8_t *keep) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < na; j += stride) {
        nx[al[j]] = a[j];
        keep[j] = a[j] != kNo && (a[j] & kRef);
    }
}
__global__ void __launch_bounds__(kBlk) k_jump_cycle(const uint64_t *al, uint64_t na, uint64_t *nx) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < na; j += stride) nx[al[j]] = kNo;
}
// the rulers whose jump still points at a ruler after the walks
__global__ void __launch_bounds__(kBlk) k_active_rulers(const uint64_t *rl, uint64_t nr, const uint64_t *nx, uint8_t *keep) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nr; j += stride)
        keep[j] = nx[rl[j]] != kNo && (nx[rl[j]] & kRef);
}

// the references of branch successors: request y, four slots per branch
__global__ void __launch_bounds__(kBlk) k_bref_req(const uint64_t *bl, uint64_t nb, const uint8_t *kind,
                                                   const uint64_t *out_info, Owners o, uint64_t *q, uint8_t *dest) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nb; j += stride) {
        const uint32_t pm = kind[bl[j]] & 0xF;
        const uint64_t lo = out_info[bl[j]] & kIdM;
        for (int b = 0; b < 4; ++b) {
            q[4 * j + b] = lo + b;
            dest[4 * j + b] = (pm >> b) & 1 ? (uint8_t)owner_of_id(o, lo + b) : kNoDest;
        }
    }
}
// a successor's reference: itself (non-unary), its ruler's terminal (a ruler), or kRef | the
// ruler whose walk passed it (kNo: none did — a ruler-less unary cycle)
__global__ void __launch_bounds__(kBlk) k_bref_ans(const uint64_t *q, uint64_t m, const uint8_t *kind, const uint64_t *nx,
                                                   uint64_t id_lo, uint64_t *ans) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        const uint64_t y = q[j], li = y - id_lo;
        const uint8_t k = kind[li];
        const uint64_t v = nx[li];
        if (__popc(k & 0xF) != 1) ans[j] = y;
        else if (k & kRuler) ans[j] = v;
        else ans[j] = is_claim(v) ? (kRef | (v & kIdM)) : kNo;  // unclaimed: a unary cycle without a ruler
    }
}
// second step for successors claimed by a ruler's walk: that ruler's terminal (slot per reference)
__global__ void __launch_bounds__(kBlk) k_bref_req2(const uint64_t *ref, uint64_t nslots, Owners o, uint64_t *q, uint8_t *dest) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nslots; j += stride) {
        const bool f = ref[j] < kPad && (ref[j] & kRef);
        q[j] = ref[j] & kIdM;
        dest[j] = f ? (uint8_t)owner_of_id(o, ref[j] & kIdM) : kNoDest;
    }
}

// branch resolution: a branch with a surviving reference (kNo: a unary cycle) survives at once;
// otherwise its references' states are requested
__global__ void __launch_bounds__(kBlk) k_res_req(const uint64_t *bl, const uint64_t *ref, uint64_t nb, uint8_t *st,
                                                  Owners o, uint64_t *q, uint8_t *dest, unsigned long long *changed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long ch = 0;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nb; j += stride) {
        bool unk = st[bl[j]] == kStUnk;
        if (unk) {
            for (int b = 0; b < 4; ++b)
                if (ref[4 * j + b] == kNo) unk = false;
            if (!unk) {
                st[bl[j]] = kStSurv;
                ++ch;
            }
        }
        for (int b = 0; b < 4; ++b) {
            const uint64_t t = ref[4 * j + b];
            q[4 * j + b] = t;
            dest[4 * j + b] = unk && t != kPad ? (uint8_t)owner_of_id(o, t) : kNoDest;
        }
    }
    block_add(changed, ch);
}
__global__ void __launch_bounds__(kBlk) k_st_ans(const uint64_t *q, uint64_t m, const uint8_t *st, uint64_t id_lo, uint64_t *ans) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) ans[j] = st[q[j] - id_lo];
}
// per branch slot: the state of its reference (a[slot], written by the answers; slots without a
// request read kStRem: padding never keeps a branch alive)
__global__ void __launch_bounds__(kBlk) k_res_apply(const uint64_t *bl, uint64_t nb, const uint64_t *a, const uint8_t *dest,
                                                    uint8_t *st, unsigned long long *changed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long ch = 0;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nb; j += stride) {
        if (st[bl[j]] != kStUnk) continue;
        bool all_rem = true, any_surv = false;
        for (int b = 0; b < 4; ++b) {
            const uint8_t sv = dest[4 * j + b] == kNoDest ? kStRem : (uint8_t)a[4 * j + b];
            if (sv == kStSurv) any_surv = true;
            if (sv != kStRem) all_rem = false;
        }
        if (any_surv) { st[bl[j]] = kStSurv; ++ch; }
        else if (all_rem) { st[bl[j]] = kStRem; ++ch; }
    }
    block_add(changed, ch);
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
// rulers: the state of their terminal (kNo: survive), one slot per ruler
__global__ void __launch_bounds__(kBlk) k_term_req(const uint64_t *rl, uint64_t nr, const uint64_t *nx, Owners o, uint64_t *q,
                                                   uint8_t *dest) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nr; j += stride) {
        const uint64_t t = nx[rl[j]];
        q[j] = t;
        dest[j] = t != kNo ? (uint8_t)owner_of_id(o, t) : kNoDest;
    }
}
// removed rulers (terminal resolved kRem): their own valid bit cleared, flagged for the list
__global__ void __launch_bounds__(kBlk) k_rm_rulers(const uint64_t *rl, uint64_t nr, const uint64_t *a, const uint8_t *dest,
                                                    uint64_t *valid, uint64_t id_lo, uint64_t *gid, uint8_t *flag) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nr; j += stride) {
        const bool r = dest[j] != kNoDest && a[j] == kStRem;
        if (r) atomicAnd((unsigned long long *)&valid[rl[j] >> 6], ~(1ULL << (rl[j] & 63)));
        gid[j] = id_lo + rl[j];
        flag[j] = r;
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
// non-ruler unary edges claimed by a removed ruler's walk
__global__ void __launch_bounds__(kBlk) k_rm_chains(const uint64_t *post, const uint8_t *kind, const uint64_t *nx, uint64_t n,
                                                    const uint64_t *tab, uint64_t cap, uint64_t *valid) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (n + 63) / 64, wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += wstride) {
        const uint64_t i = w * 64 + lane;
        bool rm = false;
        if (i < n && bit_of(post, i)) {
            const uint8_t k = kind[i];
            if (__popc(k & 0xF) == 1 && !(k & kRuler) && is_claim(nx[i])) {
                const uint64_t r = nx[i] & kIdM;
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

__global__ void __launch_bounds__(kBlk) k_and_words(uint64_t *a, const uint64_t *b, uint64_t nw) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) a[w] &= b[w];
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

__global__ void __launch_bounds__(kBlk) k_set_ids(const uint64_t *ids, uint64_t m, uint64_t *bm) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride)
        atomicOr((unsigned long long *)&bm[ids[j] >> 6], 1ULL << (ids[j] & 63));
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
                                                  uint8_t *dest) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nf; j += stride) {
        const uint64_t li = front[j];
        uint64_t lo, pos;
        if (backward) {
            const uint64_t ii = in_info[li];
            lo = ii & kIdM;
            pos = (ii >> kIdxBits) & 0xFFFF;
        } else {
            const uint64_t oi = out_info[li];
            lo = oi & kIdM;
            pos = (1ULL << __popc((unsigned)(oi >> kIdxBits) & 0xF)) - 1;
        }
        q[j] = lo | (pos << kIdxBits);
        dest[j] = pos ? (uint8_t)owner_of_id(o, lo) : kNoDest;
    }
}
// the owner: the window's group joins the region; its valid, unseen positions join the next frontier
__global__ void __launch_bounds__(kBlk) k_bfs_claim(const uint64_t *q, uint64_t m, uint64_t id_lo, uint64_t n, const uint64_t *gs,
                                                    const uint64_t *valid, uint64_t *reg, uint64_t *seen, uint64_t *next,
                                                    unsigned long long *nn) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < m; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        const uint64_t li = j < m ? (q[j] & kIdM) - id_lo : 0;
        const uint32_t pos = j < m ? (uint32_t)(q[j] >> kIdxBits) & 0xFFFF : 0;
        if (j < m) mark_group(gs, n, li, reg);
        for (int b = 0; b < 16; ++b) {
            const uint64_t y = li + b;
            bool f = ((pos >> b) & 1) && y < n && bit_of(valid, y);
            if (f) {
                const unsigned long long bit = 1ULL << (y & 63);
                f = !(atomicOr((unsigned long long *)&seen[y >> 6], bit) & bit);
            }
            unsigned long long mk;
            const uint64_t at = wave_reserve(f, nn, mk);
            if (f) next[at] = y;
        }
    }
}

// (round 6) The region BFS with its hops back to back on the device. A hop's requests go into
// fixed-capacity blocks, one per rank (word 0: the block's request count, then up to its capacity
// of requests; this rank's own block is separate and holds a whole frontier), exchanged by
// Comm::alltoall_fixed, which the RCCL transport leaves queued on the stream: no host round trip
// per hop (round 5's form took three: the count all-gather, the all-to-all, the next frontier's
// size). Frontier sizes stay in device memory (one counter per hop). A block or frontier that
// overflows its capacity sets a flag (with the count it needed); the host reads the flags once
// after the last hop, and if any rank overflowed every rank runs the BFS again with larger blocks.
struct BfsCaps {
    uint64_t P;   // requests per block to another rank
    uint64_t F;   // requests in the own block, edges per frontier
};
// flags: [0] a peer block overflowed, [1] the most requests one peer block needed,
// [2] the own block or a frontier overflowed, [3] the largest own block / frontier needed
__global__ void __launch_bounds__(kBlk) k_bfs_zero(uint64_t *send, int N, uint64_t P, uint64_t *self_blk) {
    const int t = threadIdx.x;
    if (t < N) send[(uint64_t)t * (1 + P)] = 0;
    if (t == 0) self_blk[0] = 0;
}
__global__ void __launch_bounds__(kBlk) k_bfs_req_dev(const uint64_t *front, const unsigned long long *nf_p,
                                                      const uint64_t *out_info, const uint64_t *in_info, int backward,
                                                      Owners o, uint64_t *send, BfsCaps c, uint64_t *self_blk,
                                                      unsigned long long *flags) {
    const uint64_t nf = min((uint64_t)*nf_p, c.F), stride = (uint64_t)gridDim.x * blockDim.x;  // (past F: flagged)
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < nf; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        uint64_t rec = 0;
        int d = -1;
        if (j < nf) {
            const uint64_t li = front[j];
            uint64_t lo, pos;
            if (backward) {
                const uint64_t ii = in_info[li];
                lo = ii & kIdM;
                pos = (ii >> kIdxBits) & 0xFFFF;
            } else {
                const uint64_t oi = out_info[li];
                lo = oi & kIdM;
                pos = (1ULL << __popc((unsigned)(oi >> kIdxBits) & 0xF)) - 1;
            }
            rec = lo | (pos << kIdxBits);
            if (pos) d = owner_of_id(o, lo);
        }
        // one count atomic per destination present in the wave
        unsigned long long pend = __ballot(d >= 0);
        while (pend) {
            const int lead = __ffsll((long long)pend) - 1;
            const int dd = __shfl(d, lead);
            const unsigned long long m = __ballot(d == dd);
            const bool self = dd == o.R;
            uint64_t *blk = self ? self_blk : send + (uint64_t)dd * (1 + c.P);
            const uint64_t cap = self ? c.F : c.P;
            uint64_t base = 0;
            if ((int)(threadIdx.x & 63) == lead) base = atomicAdd((unsigned long long *)blk, (unsigned long long)__popcll(m));
            base = __shfl(base, lead);
            if (d == dd) {
                const uint64_t at = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                if (at < cap) blk[1 + at] = rec;
                if (at + 1 == base + __popcll(m) && base + __popcll(m) > cap) {  // the wave's last slot
                    atomicOr(&flags[self ? 2 : 0], 1ull);
                    atomicMax(&flags[self ? 3 : 1], (unsigned long long)(base + __popcll(m)));
                }
            }
            pend &= ~m;
        }
    }
}
// (round 6) fixed-block request / reply (branch resolution): slot j's request q[j] goes to rank
// dest[j] (kNoDest: none) into that rank's block (word 0: count; this rank's own requests into
// its own block, which holds every slot), its position kept in pos[j]; the answers come back in
// the same positions
__global__ void __launch_bounds__(kBlk) k_fx_post(const uint64_t *q, const uint8_t *dest, uint64_t m, int R,
                                                  uint64_t *send, uint64_t P, uint64_t *self_blk, uint32_t *pos) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < m; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        const int d = j < m && dest[j] != kNoDest ? (int)dest[j] : -1;
        unsigned long long pend = __ballot(d >= 0);
        while (pend) {
            const int lead = __ffsll((long long)pend) - 1;
            const int dd = __shfl(d, lead);
            const unsigned long long mk = __ballot(d == dd);
            uint64_t *blk = dd == R ? self_blk : send + (uint64_t)dd * (1 + P);
            uint64_t base = 0;
            if ((int)(threadIdx.x & 63) == lead) base = atomicAdd((unsigned long long *)blk, (unsigned long long)__popcll(mk));
            base = __shfl(base, lead);
            if (d == dd) {
                const uint64_t at = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0));
                blk[1 + at] = q[j];  // (P holds every slot of the largest rank: no overflow)
                pos[j] = (uint32_t)at;
            }
            pend &= ~mk;
        }
    }
}
// the owner: each received request's state (as k_st_ans) into the reply block at its position
__global__ void __launch_bounds__(kBlk) k_fx_st_ans(const uint64_t *recv, const uint64_t *self_blk, int R, uint64_t P,
                                                    const uint8_t *st, uint64_t id_lo, uint64_t *rsend, uint64_t *rself) {
    const int src = blockIdx.y;
    const uint64_t *blk = src == R ? self_blk : recv + (uint64_t)src * (1 + P);
    uint64_t *out = src == R ? rself : rsend + (uint64_t)src * (1 + P);
    const uint64_t m = blk[0];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) out[1 + j] = st[blk[1 + j] - id_lo];
}
// the requester: slot j's answer from its destination's reply block
__global__ void __launch_bounds__(kBlk) k_fx_gather(const uint8_t *dest, const uint32_t *pos, uint64_t m, int R,
                                                    const uint64_t *rrecv, uint64_t P, const uint64_t *rself, uint64_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        if (dest[j] == kNoDest) continue;
        const int d = dest[j];
        out[j] = d == R ? rself[1 + pos[j]] : rrecv[(uint64_t)d * (1 + P) + 1 + pos[j]];
    }
}

// the owner side of a hop, over every rank's block (blockIdx.y: the source rank); as k_bfs_claim
__global__ void __launch_bounds__(kBlk) k_bfs_claim_dev(const uint64_t *recv, const uint64_t *self_blk, int R, BfsCaps c,
                                                        uint64_t id_lo, uint64_t n, const uint64_t *gs,
                                                        const uint64_t *valid, uint64_t *reg, uint64_t *seen,
                                                        uint64_t *next, unsigned long long *nn,
                                                        unsigned long long *flags) {
    const int src = blockIdx.y;
    const uint64_t *blk = src == R ? self_blk : recv + (uint64_t)src * (1 + c.P);
    const uint64_t m = min(blk[0], src == R ? c.F : c.P);
    const uint64_t *q = blk + 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = (uint64_t)blockIdx.x * blockDim.x; j0 < m; j0 += stride) {
        const uint64_t j = j0 + threadIdx.x;
        const uint64_t li = j < m ? (q[j] & kIdM) - id_lo : 0;
        const uint32_t pos = j < m ? (uint32_t)(q[j] >> kIdxBits) & 0xFFFF : 0;
        if (j < m) mark_group(gs, n, li, reg);
        for (int b = 0; b < 16; ++b) {
            const uint64_t y = li + b;
            bool f = ((pos >> b) & 1) && y < n && bit_of(valid, y);
            if (f) {
                const unsigned long long bit = 1ULL << (y & 63);
                f = !(atomicOr((unsigned long long *)&seen[y >> 6], bit) & bit);
            }
            unsigned long long mk;
            const uint64_t at = wave_reserve(f, nn, mk);
            if (f) {
                if (at < c.F) next[at] = y;
                else {
                    atomicOr(&flags[2], 1ull);
                    atomicMax(&flags[3], (unsigned long long)(at + 1));
                }
            }
        }
    }
}

// a BFS hop on a region replica (compact ids, every rank alike): the valid successors not seen yet
__global__ void __launch_bounds__(kBlk) k_cbfs(GraphView g, const uint64_t *front, uint64_t nf, uint64_t *seen, uint64_t *next,
                                               unsigned long long *nn) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nf; j += stride) {
        uint64_t out[4];
        const int od = dev_outgoing(g, front[j], out);
        for (int b = 0; b < od; ++b) {
            const uint64_t x = out[b], bit = 1ULL << (x & 63);
            if (!(atomicOr((unsigned long long *)&seen[x >> 6], bit) & bit)) next[atomicAdd(nn, 1ull)] = x;
        }
    }
}

// (round 6) the same hop with the frontier size read on the device: the hops run back to back
// with no host round trip between them (the frontier buffers hold every edge of the replica, and
// each edge joins a frontier at most once)
__global__ void __launch_bounds__(kBlk) k_cbfs_dev(GraphView g, const uint64_t *front, const unsigned long long *nf_p,
                                                   uint64_t *seen, uint64_t *next, unsigned long long *nn) {
    const uint64_t nf = *nf_p, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nf; j += stride) {
        uint64_t out[4];
        const int od = dev_outgoing(g, front[j], out);
        for (int b = 0; b < od; ++b) {
            const uint64_t x = out[b], bit = 1ULL << (x & 63);
            if (!(atomicOr((unsigned long long *)&seen[x >> 6], bit) & bit)) next[atomicAdd(nn, 1ull)] = x;
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

    // the set bits of a local bitmap (nwl words) as local indices, ascending
    // (nw: the bitmap's words, default this rank's)
    uint64_t list_bits(const uint64_t *bm, DevBuf<uint64_t> &out, uint64_t nw = ~0ULL) {
        if (nw == ~0ULL) nw = nwl;
        DevBuf<uint64_t> pc(nw + 1), wpre(nw + 1);
        HIP_OK(hipMemsetAsync(pc.p + nw, 0, 8, st));
        uint64_t cnt = 0;
        if (nw) {
            hipLaunchKernelGGL(k_word_popc64, dim3(grid(nw)), dim3(kBlk), 0, st, bm, nw, pc.p);
            LAUNCH_OK();
            size_t tmp = 0;
            HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, pc.p, wpre.p, (size_t)(nw + 1), st));
            DevBuf<uint8_t> t(tmp);
            HIP_OK(hipcub::DeviceScan::ExclusiveSum(t.p, tmp, pc.p, wpre.p, (size_t)(nw + 1), st));
            d2h(ctx, &cnt, wpre.p + nw, 8);
        }
        out.alloc(cnt ? cnt : 1);
        if (cnt) {
            hipLaunchKernelGGL(k_bits_list, dim3(grid(nw * 64)), dim3(kBlk), 0, st, bm, nw, (const uint64_t *)wpre.p, out.p);
            LAUNCH_OK();
        }
        return cnt;
    }

    // (round 6) a search region's id translations on the device, where its gid list stays (its
    // 8 B per edge were read back whole before: C3 at one rank, 20 ms for the DLS region's 5.5 M
    // ids and 16 ms of host binary searches for the candidates)
    // edge ids -> compact ids of region rg (rn edges); every id must lie in the region
    std::vector<uint64_t> to_compact(const mcaat_graph &rg, uint64_t rn, const std::vector<uint64_t> &ids) {
        const uint64_t m = ids.size();
        std::vector<uint64_t> c(m);
        if (!m) return c;
        DevBuf<uint64_t> d(m), o(m);
        h2d(ctx, d.p, ids.data(), 8 * m);
        hipLaunchKernelGGL(k_gid_find, dim3(grid(m)), dim3(kBlk), 0, st, (const uint64_t *)rg.gid.p, rn,
                           (const uint64_t *)d.p, m, o.p);
        LAUNCH_OK();
        d2h(ctx, c.data(), o.p, 8 * m);
        for (uint64_t x : c)
            if (x == ~0ULL) throw Error(MCAAT_E_INVALID, "per-shard CycleFinder: a start is outside its region");
        return c;
    }
    // compact ids (device list of m) -> edge ids (~0 past the region's edges)
    std::vector<uint64_t> to_global(const mcaat_graph &rg, uint64_t rn, const uint64_t *c, uint64_t m) {
        std::vector<uint64_t> g(m);
        if (!m) return g;
        DevBuf<uint64_t> o(m);
        hipLaunchKernelGGL(k_gid_of, dim3(grid(m)), dim3(kBlk), 0, st, (const uint64_t *)rg.gid.p, rn, c, m, o.p);
        LAUNCH_OK();
        d2h(ctx, g.data(), o.p, 8 * m);
        return g;
    }
    std::vector<uint64_t> to_global(const mcaat_graph &rg, uint64_t rn, const std::vector<uint64_t> &c) {
        if (c.empty()) return {};
        DevBuf<uint64_t> d(c.size());
        h2d(ctx, d.p, c.data(), 8 * c.size());
        return to_global(rg, rn, d.p, c.size());
    }

    // in[j] where flags[j] != 0, in order (hipcub select); returns the count
    uint64_t select(const uint64_t *in, const uint8_t *flags, uint64_t m, uint64_t *out) {
        DevBuf<unsigned long long> num(1);
        size_t tmp = 0;
        HIP_OK(hipcub::DeviceSelect::Flagged(nullptr, tmp, in, flags, out, num.p, (size_t)m, st));
        DevBuf<uint8_t> t(tmp ? tmp : 1);
        HIP_OK(hipcub::DeviceSelect::Flagged(t.p, tmp, in, flags, out, num.p, (size_t)m, st));
        return read_u64(ctx, num.p);
    }

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
            DevBuf<uint64_t> q(nf ? nf : 1);
            DevBuf<uint8_t> dest(nf ? nf : 1);
            HIP_OK(hipMemsetAsync(c.p, 0, 16, st));
            if (nf) {
                hipLaunchKernelGGL(k_bfs_req, dim3(grid(nf)), dim3(kBlk), 0, st, (const uint64_t *)front.p, nf,
                                   (const uint64_t *)g->out_info.p, (const uint64_t *)g->in_info.p, (int)backward, o, q.p,
                                   dest.p);
                LAUNCH_OK();
            }
            Routed r;
            rt.send(q.p, 1, dest.p, nf, r, false);
            if (!r.total) break;  // every rank's frontier was empty (the routing's count exchange says so)
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

    // (round 6) the BFS from this rank's edges `ids` (global ids), hops back to back on the device
    // (see k_bfs_req_dev); reg and seen are cleared and seeded here, and cleared again for a run
    // with larger blocks after an overflow on any rank
    void bfs_dev(const std::vector<uint64_t> &ids, uint64_t rounds, bool backward, const uint64_t *gs, uint64_t *reg,
                 uint64_t *seen) {
        const int N = comm.world, R = comm.rank;
        const uint64_t m = ids.size();
        DevBuf<uint64_t> dids(m + 1);
        if (m) h2d(ctx, dids.p, ids.data(), 8 * m);
        BfsCaps c;
        // (C3 at 8 ranks needs up to 2^15 requests a block: 2^16 is 512 KB a peer and hop)
        c.P = (uint64_t)std::max<int64_t>(64, knob(ctx, "dist.bfs_block", 1 << 16));
        if (!knob_set(ctx, "dist.bfs_block")) c.P = std::max(c.P, ctx->bfs_block[backward]);
        // a frontier or the own block: the whole local graph in the end (each edge joins one
        // frontier at most once), a sixteenth of it (and the seeds) first
        c.F = std::min<uint64_t>(n + 1, std::max<uint64_t>({m + 1, n / 16 + 1, 1u << 20}));
        if (knob_set(ctx, "dist.bfs_frontier")) c.F = std::max<uint64_t>(m + 1, (uint64_t)knob(ctx, "dist.bfs_frontier", 1));
        for (int attempt = 0;; ++attempt) {
            HIP_OK(hipMemsetAsync(reg, 0, 8 * (nwl + 1), st));
            HIP_OK(hipMemsetAsync(seen, 0, 8 * (nwl + 1), st));
            DevBuf<uint64_t> fr[2];
            fr[0].alloc(c.F);
            fr[1].alloc(c.F);
            DevBuf<uint64_t> send((uint64_t)N * (1 + c.P)), recv((uint64_t)N * (1 + c.P)), self_blk(1 + c.F);
            DevBuf<unsigned long long> cnt(rounds + 1), flags(4);
            HIP_OK(hipMemsetAsync(cnt.p, 0, cnt.bytes(), st));
            HIP_OK(hipMemsetAsync(flags.p, 0, flags.bytes(), st));
            if (m) {
                hipLaunchKernelGGL(k_bfs_seed, dim3(grid(m)), dim3(kBlk), 0, st, (const uint64_t *)dids.p, m, g->id_lo, n, gs,
                                   reg, seen, fr[0].p);
                LAUNCH_OK();
                h2d(ctx, cnt.p, &m, 8);
            }
            const unsigned gq = grid(std::min<uint64_t>(c.F, 1u << 22));
            const unsigned gc = grid(std::min<uint64_t>(std::max(c.F, c.P), 1u << 22)) / (unsigned)N + 1;
            for (uint64_t h = 0; h < rounds; ++h) {
                hipLaunchKernelGGL(k_bfs_zero, dim3(1), dim3(kBlk), 0, st, send.p, N, c.P, self_blk.p);
                LAUNCH_OK();
                hipLaunchKernelGGL(k_bfs_req_dev, dim3(gq), dim3(kBlk), 0, st, (const uint64_t *)fr[h & 1].p,
                                   (const unsigned long long *)(cnt.p + h), (const uint64_t *)g->out_info.p,
                                   (const uint64_t *)g->in_info.p, (int)backward, o, send.p, c, self_blk.p, flags.p);
                LAUNCH_OK();
                comm.alltoall_fixed(send.p, 8 * (1 + c.P), recv.p);
                hipLaunchKernelGGL(k_bfs_claim_dev, dim3(gc, (unsigned)N), dim3(kBlk), 0, st, (const uint64_t *)recv.p,
                                   (const uint64_t *)self_blk.p, R, c, g->id_lo, n, gs, (const uint64_t *)g->valid.p, reg,
                                   seen, fr[(h + 1) & 1].p, cnt.p + h + 1, flags.p);
                LAUNCH_OK();
            }
            unsigned long long fl[4];
            d2h(ctx, fl, flags.p, 32);
            // every rank takes the same decision (the exchanges are collective)
            const auto all = comm.allgather_vec(std::vector<uint64_t>{fl[0] | fl[2], fl[1], fl[3]});
            bool again = false;
            uint64_t needP = 0, needF = 0;
            for (int r = 0; r < N; ++r) {
                again |= all[3 * r] != 0;
                needP = std::max<uint64_t>(needP, all[3 * r + 1]);
                needF = std::max<uint64_t>(needF, all[3 * r + 2]);
            }
            if (!again) {
                ctx->bfs_block[backward] = c.P;
                break;
            }
            if (attempt >= 8) throw Error(MCAAT_E_CAPACITY, "per-shard region BFS: blocks still overflow");
            // a hop after an overflowed one saw a partial frontier: twice what was counted, at least
            c.P = std::max(c.P, next_pow2(2 * needP));
            c.F = std::min<uint64_t>(n + 1, std::max(c.F, 2 * needF));
            if (needF > c.F) c.F = n + 1;
            if (verbose())
                fprintf(stderr, "[mcaat] shard %d: region BFS again with %llu-request blocks, %llu-edge frontiers\n", R,
                        (unsigned long long)c.P, (unsigned long long)c.F);
        }
    }

    // every rank: the compact replica of the groups marked in reg on all ranks
    // returns the region's edge count (rg->gid: their ascending ids, kept on the device)
    uint64_t gather_region(const uint64_t *reg, mcaat_graph *rg) {
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
        verbose_mark(ctx, "region.list");
        const std::vector<uint64_t> per = comm.allgather_one(mine);
        uint64_t rn = 0;
        std::vector<uint64_t> bytes(comm.world);
        for (int r = 0; r < comm.world; ++r) rn += per[r], bytes[r] = 32 * per[r];
        DevBuf<uint64_t> all(4 * (rn ? rn : 1));
        HIP_OK(hipStreamSynchronize(st));
        if (rn) comm.allgatherv_dev(rec.p, all.p, bytes.data());
        verbose_mark(ctx, "region.gather");
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
        verbose_mark(ctx, "region.build");
        return rn;
    }
};

}  // namespace

// ---------------------------------------------------------------- sharded adjacency
namespace {
void finish_valid(mcaat_ctx *ctx, mcaat_graph *g) {
    const uint64_t n = g->D_local;
    g->valid.alloc(mcaat_graph::bitmap_words(n));
    HIP_OK(hipMemsetAsync(g->valid.p, 0, g->valid.bytes(), ctx->stream));
    if (n) {
        hipLaunchKernelGGL(k_ones, dim3(grid_for((n + 63) / 64, kBlk)), dim3(kBlk), 0, ctx->stream, g->valid.p, n);
        LAUNCH_OK();
    }
    g->all_valid = true;
    HIP_OK(hipStreamSynchronize(ctx->stream));
}

// O_W(r) for every rank: O[W * (N + 1) + r] (kept in g->tgt_lo)
std::vector<uint64_t> target_ranges(mcaat_ctx *ctx, Comm &comm, const mcaat_graph *g) {
    hipStream_t st = ctx->stream;
    const int k = g->k, N = comm.world;
    const uint64_t n = g->D_local, D = g->D;
    // every rank's first key (empty ranks: the next rank's, or none)
    uint64_t fk = ~0ULL;
    if (n) d2h(ctx, &fk, g->key.p, 8);
    const std::vector<uint64_t> first = comm.allgather_one(fk);
    const uint64_t top = (uint64_t)1 << (2 * (k - 1));
    // queries q[W][r], r = 0..N: the start of O_W(r); the global lower bound = sum over ranks of
    // their local count below q (q past the key space: D)
    std::vector<uint64_t> qs(4 * (N + 1));
    for (int W = 0; W < 4; ++W)
        for (int r = 0; r <= N; ++r) {
            uint64_t f = ~0ULL;
            for (int x = r; x < N && f == ~0ULL; ++x) f = first[x];
            uint64_t t;
            if (r == 0) t = (uint64_t)W * top;
            else if (r == N || f == ~0ULL) t = (uint64_t)(W + 1) * top;
            else t = ((uint64_t)W * top) | (f >> 4);
            qs[W * (N + 1) + r] = t << 2;
        }
    std::vector<uint64_t> cl(qs.size(), 0);
    if (n) {
        DevBuf<uint64_t> dq(qs.size()), dc(qs.size());
        h2d(ctx, dq.p, qs.data(), 8 * qs.size());
        hipLaunchKernelGGL(k_count_less, dim3(grid_for(qs.size(), kBlk)), dim3(kBlk), 0, st, (const uint64_t *)g->key.p, n,
                           (const uint64_t *)dq.p, (int)qs.size(), dc.p);
        LAUNCH_OK();
        d2h(ctx, cl.data(), dc.p, 8 * cl.size());
    }
    const std::vector<uint64_t> all = comm.allgather_vec(cl);
    std::vector<uint64_t> O(qs.size(), 0);  // O[W * (N + 1) + r]
    for (size_t i = 0; i < qs.size(); ++i) {
        if (qs[i] >> (2 * (k + 1))) {
            O[i] = D;
            continue;
        }
        for (int x = 0; x < N; ++x) O[i] += all[x * qs.size() + i];
    }
    return O;
}

// contiguous-range exchanges over the target ranges: pull = the values of O_W(R)'s edges from
// their owners; push = values computed here for O_W(R)'s edges to their owners
struct RangeX {
    Comm &comm;
    int N, R;
    const std::vector<uint64_t> &lo;  // rank_lo
    const std::vector<uint64_t> &O;
    uint64_t a(int W, int r) const { return O[W * (N + 1) + r]; }
    uint64_t len(int W) const { return a(W, R + 1) - a(W, R); }
    // es-byte elements: local[n] -> out[len(W)]
    void pull(const void *local, size_t es, int W, void *out) const {
        std::vector<uint64_t> sb(N), so(N), rb(N), ro(N);
        for (int q = 0; q < N; ++q) {
            // to q: my elements inside O_W(q); from q: q's elements inside O_W(R)
            const uint64_t s0 = std::max(a(W, q), lo[R]), s1 = std::min(a(W, q + 1), lo[R + 1]);
            sb[q] = s1 > s0 ? es * (s1 - s0) : 0;
            so[q] = s1 > s0 ? es * (s0 - lo[R]) : 0;
            const uint64_t r0 = std::max(a(W, R), lo[q]), r1 = std::min(a(W, R + 1), lo[q + 1]);
            rb[q] = r1 > r0 ? es * (r1 - r0) : 0;
            ro[q] = r1 > r0 ? es * (r0 - a(W, R)) : 0;
        }
        comm.alltoallv_dev(local, sb.data(), out, rb.data(), so.data(), ro.data());
    }
    // in[len(W)] -> local[n]
    void push(const void *in, size_t es, int W, void *local) const {
        std::vector<uint64_t> sb(N), so(N), rb(N), ro(N);
        for (int q = 0; q < N; ++q) {
            const uint64_t s0 = std::max(a(W, R), lo[q]), s1 = std::min(a(W, R + 1), lo[q + 1]);
            sb[q] = s1 > s0 ? es * (s1 - s0) : 0;
            so[q] = s1 > s0 ? es * (s0 - a(W, R)) : 0;
            const uint64_t r0 = std::max(a(W, q), lo[R]), r1 = std::min(a(W, q + 1), lo[R + 1]);
            rb[q] = r1 > r0 ? es * (r1 - r0) : 0;
            ro[q] = r1 > r0 ? es * (r0 - lo[R]) : 0;
        }
        comm.alltoallv_dev(in, sb.data(), local, rb.data(), so.data(), ro.data());
    }
};

// out_info / in_info of the rank's edges through its four target ranges (k_adj_ranges above)
void adjacency_by_ranges(mcaat_ctx *ctx, Comm &comm, mcaat_graph *g) {
    hipStream_t st = ctx->stream;
    const int k = g->k, R = comm.rank;
    const uint64_t n = g->D_local, id_lo = g->id_lo;
    KernelTimer kt(ctx, "adjacency", 32.0 * (double)n);
    g->tgt_lo = target_ranges(ctx, comm, g);
    const RangeX X{comm, comm.world, R, g->rank_lo, g->tgt_lo};
    // fetch the keys of O_W(R) from their owners, one all-to-all per W
    DevBuf<uint64_t> tk[4], ti[4];
    TgtRanges T{};
    for (int W = 0; W < 4; ++W) {
        const uint64_t a = X.a(W, R), b = X.a(W, R + 1);
        tk[W].alloc(b - a + 1);
        ti[W].alloc(b - a + 1);
        X.pull(g->key.p, 8, W, tk[W].p);
        T.key[W] = tk[W].p;
        T.in[W] = ti[W].p;
        T.len[W] = b - a;
        T.g0[W] = a;
    }
    // runs of the own edges, then out_info and the ranges' in_info
    const uint64_t nruns = (n + kRunB - 1) / kRunB;
    if (nruns) {
        DevBuf<uint64_t> bounds(5 * (nruns + 1));
        hipLaunchKernelGGL(k_run_bounds, dim3(grid_for(nruns + 1, kBlk)), dim3(kBlk), 0, st, (const uint64_t *)g->key.p, n, k,
                           T, nruns, bounds.p);
        LAUNCH_OK();
        hipLaunchKernelGGL(k_adj_ranges, dim3((unsigned)nruns), dim3(kRunT), 0, st, (const uint64_t *)g->key.p, id_lo, k, T,
                           (const uint64_t *)bounds.p, g->out_info.p);
        LAUNCH_OK();
    } else {
        for (int W = 0; W < 4; ++W)  // no sources: the ranges (empty or not) have no predecessors here
            if (T.len[W]) HIP_OK(hipMemsetAsync(ti[W].p, 0, 8 * T.len[W], st));
    }
    for (int W = 0; W < 4; ++W) tk[W].release();
    // the in_info slices back to their owners
    for (int W = 0; W < 4; ++W) X.push(ti[W].p, 8, W, g->in_info.p);
    kt.stop();
    if (verbose())
        fprintf(stderr, "[mcaat] shard %d: adjacency of %llu edges by key ranges (%llu + %llu + %llu + %llu target keys)\n",
                R, (unsigned long long)n, (unsigned long long)T.len[0], (unsigned long long)T.len[1],
                (unsigned long long)T.len[2], (unsigned long long)T.len[3]);
}
}  // namespace

void sdbg_finish_sharded(mcaat_ctx *ctx, Comm &comm, mcaat_graph *g) {
    hipStream_t st = ctx->stream;
    const int k = g->k;
    const uint64_t n = g->D_local;
    // local radix directory over the range's keys (dist.dir_edges edges per prefix, default 2)
    uint64_t kmin = 0, kmax = 0;
    if (n) {
        d2h(ctx, &kmin, g->key.p, 8);
        d2h(ctx, &kmax, g->key.p + n - 1, 8);
    }
    int shift = 0;
    const uint64_t want = std::max<uint64_t>(1, n / (uint64_t)std::max<int64_t>(1, knob(ctx, "dist.dir_edges", 2)));
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
    if (knob(ctx, "dist.adj_ranges", 1)) {
        adjacency_by_ranges(ctx, comm, g);
        finish_valid(ctx, g);
        return;
    }
    Router rt(ctx, comm);
    const Owners o = owners_of(g, comm);
    // chunks of edges: two queries each; every rank takes part in as many exchanges
    const uint64_t chunk = (uint64_t)std::max<int64_t>(1024, knob(ctx, "dist.adj_chunk", 1LL << 26));
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
    finish_valid(ctx, g);
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
    // collectives per stage (kstats "xr_<stage>".launches): the bulk-synchronous rounds that bound
    // this path at N ranks (DESIGN.md §7's model)
    uint64_t xr_last = comm.n_coll, xq_last = comm.n_queued;
    auto xr = [&](const char *stage) {
        ctx->kstats[std::string("xr_") + stage].launches += comm.n_coll - xr_last;
        ctx->kstats[std::string("xq_") + stage].launches += comm.n_queued - xq_last;  // of them queued
        xr_last = comm.n_coll;
        xq_last = comm.n_queued;
    };
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
    DevBuf<uint64_t> nx(n ? n : 1);
    HIP_OK(hipMemsetAsync(kind.p, 0, kind.bytes(), st));
    DevBuf<uint64_t> cbits(nwl + 1);  // ChunkStartNodes' filter, one bit per local edge
    HIP_OK(hipMemsetAsync(cbits.p, 0, cbits.bytes(), st));
    // chunks of local edges per exchange (every rank runs as many): bounded transient memory
    const uint64_t chunk = (uint64_t)std::max<int64_t>(1024, knob(ctx, "dist.adj_chunk", 1LL << 26));
    uint64_t n_chunks = (n + chunk - 1) / chunk;
    for (uint64_t x : comm.allgather_one(n_chunks)) n_chunks = std::max(n_chunks, x);
    const bool win_ranges = knob(ctx, "dist.win_ranges", 1) != 0;  // (also: merge points known, kMerge)
    if (win_ranges) {
        n_chunks = 0;  // (the message form below is skipped)
        if (g->tgt_lo.empty()) g->tgt_lo = target_ranges(ctx, comm, g);
        const RangeX X{comm, comm.world, comm.rank, g->rank_lo, g->tgt_lo};
        TgtBytes T{};
        DevBuf<uint8_t> tpb[4], tf[4];
        {
            DevBuf<uint8_t> pb(n + 1);
            if (n) {
                hipLaunchKernelGGL(k_post_bytes, dim3(s.grid(n)), dim3(kBlk), 0, st, (const uint64_t *)post.p, n, pb.p);
                LAUNCH_OK();
            }
            for (int W = 0; W < 4; ++W) {
                const uint64_t len = X.len(W);
                tpb[W].alloc(len + 8);
                tf[W].alloc(len + 8);
                HIP_OK(hipMemsetAsync(tf[W].p, 0, tf[W].bytes(), st));
                X.pull(pb.p, 1, W, tpb[W].p);
                T.pb[W] = tpb[W].p;
                T.tf[W] = tf[W].p;
                T.g0[W] = X.a(W, comm.rank);
                T.len[W] = len;
            }
        }
        if (n) {
            hipLaunchKernelGGL(k_out_win, dim3(s.grid(n)), dim3(kBlk), 0, st, (const uint64_t *)post.p,
                               (const uint64_t *)g->key.p, (const uint64_t *)g->out_info.p, n, T, kind.p, nx.p);
            LAUNCH_OK();
            hipLaunchKernelGGL(k_push_bytes, dim3(s.grid(n)), dim3(kBlk), 0, st, (const uint64_t *)post.p,
                               (const uint64_t *)seed.p, (const uint64_t *)g->key.p, (const uint64_t *)g->out_info.p,
                               (const uint8_t *)kind.p, n, id_lo, T, cnt.p);
            LAUNCH_OK();
        }
        for (int W = 0; W < 4; ++W) tpb[W].release();
        DevBuf<uint8_t> inb(n + 1);
        HIP_OK(hipMemsetAsync(inb.p, 0, inb.bytes(), st));
        for (int W = 0; W < 4; ++W) X.push(tf[W].p, 1, W, inb.p);
        if (n) {
            hipLaunchKernelGGL(k_recv_bytes, dim3(s.grid(nwl * 64)), dim3(kBlk), 0, st, (const uint8_t *)inb.p,
                               (const uint64_t *)post.p, (const uint16_t *)g->mult.p, (uint64_t)p.threshold_multiplicity,
                               n, kind.p, nx.p, cbits.p);
            LAUNCH_OK();
        }
    }
    if (n_chunks) HIP_OK(hipMemsetAsync(nx.p, 0xFF, nx.bytes(), st));  // kNo: no successor word
    for (uint64_t c = 0; c < n_chunks; ++c) {
        const uint64_t a0 = std::min(n, c * chunk), a1 = std::min(n, a0 + chunk), m = a1 - a0;
        DevBuf<uint64_t> q(2 * m + 1);
        DevBuf<uint8_t> dest(2 * m + 1);
        if (m) {
            hipLaunchKernelGGL(k_win_req, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint64_t *)post.p,
                               (const uint16_t *)g->mult.p, (const uint64_t *)g->out_info.p, (const uint64_t *)g->in_info.p,
                               a0, a1, (uint64_t)p.threshold_multiplicity, s.o, q.p, dest.p);
            LAUNCH_OK();
        }
        Routed r;
        s.rt.send(q.p, 1, dest.p, 2 * m, r, true);
        DevBuf<uint64_t> ans(r.n_in + 1);
        if (r.n_in) {
            hipLaunchKernelGGL(k_win_ans, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)post.p, n, id_lo,
                               (const uint64_t *)r.in.p, r.n_in, ans.p);
            LAUNCH_OK();
        }
        s.rt.reply(r, ans.p, 1, q.p);  // the answers land in their request slots
        if (m) {
            hipLaunchKernelGGL(k_win_apply, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint8_t *)dest.p,
                               (const uint64_t *)q.p, a0, a1, (const uint64_t *)g->out_info.p, (const uint64_t *)g->in_info.p,
                               id_lo, kind.p, nx.p, cbits.p);
            LAUNCH_OK();
        }
    }
    // predecessor flags, as messages to the successors' owners (after every window is in)
    for (uint64_t c = 0; c < n_chunks; ++c) {
        const uint64_t a0 = std::min(n, c * chunk), a1 = std::min(n, a0 + chunk), m = a1 - a0;
        DevBuf<uint64_t> q(4 * m + 1);
        DevBuf<uint8_t> dest(4 * m + 1);
        if (m) {
            hipLaunchKernelGGL(k_flag_msgs, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint64_t *)post.p,
                               (const uint64_t *)seed.p, (const uint8_t *)kind.p, (const uint64_t *)g->out_info.p, a0, a1,
                               s.o, q.p, dest.p, cnt.p);
            LAUNCH_OK();
        }
        Routed r;
        s.rt.send(q.p, 1, dest.p, 4 * m, r, false);
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
    xr("tips_filter");

    // 3. RecursiveReduction: rulers, walks, pointer jumping, branch resolution, removal
    // ruler density: a walk's rounds are the rank crossings of the longest walk (≈ (N-1)/N x its
    // length), so more ranks take denser rulers (C3, two shm ranks: 1 in 4 / 8 / 16 / 64 unary
    // edges -> 35 / 77 / 135 / 489 walk rounds, 1.13 / 0.60 / 0.36 / 0.20 G records)
    const uint64_t rmask = (uint64_t)std::max<int64_t>(0, knob(ctx, "dist.ruler_mask", comm.world > 2 ? 3 : 15));
    DevBuf<uint64_t> rl, bl;
    uint64_t nr = 0, nb = 0;
    {
        DevBuf<uint64_t> rbits(nwl + 1), bbits(nwl + 1);
        if (n) {
            hipLaunchKernelGGL(k_prep, dim3(s.grid(nwl * 64)), dim3(kBlk), 0, st, (const uint64_t *)post.p,
                               (const uint64_t *)seed.p, kind.p, stt.p, nx.p, n, id_lo, rmask, rbits.p, bbits.p);
            LAUNCH_OK();
        }
        nr = s.list_bits(rbits.p, rl);
        nb = s.list_bits(bbits.p, bl);
    }
    verbose_mark(ctx, "shard_cf.peel_prep");
    uint64_t walk_rounds = 0;
    // (round 6) the walk's tail in fixed blocks of dist.walk_block records (default 2^15; 0: every
    // round routed, round 5's form)
    const uint64_t walkP = (uint64_t)std::max<int64_t>(0, knob(ctx, "dist.walk_block", 1 << 15));
    const bool walk_fixed = walkP > 0;
    {
        DevBuf<uint64_t> w(2 * (nr ? nr : 1));
        if (nr) {
            hipLaunchKernelGGL(k_walk_init, dim3(s.grid(nr)), dim3(kBlk), 0, st, (const uint64_t *)rl.p, nr,
                               (const uint64_t *)nx.p, id_lo, w.p);
            LAUNCH_OK();
        }
        uint64_t m = nr;
        for (;; ++walk_rounds) {
            DevBuf<uint64_t> o2(2 * (m ? m : 1));
            DevBuf<uint8_t> dest(m ? m : 1);
            if (m) {
                hipLaunchKernelGGL(k_walk, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint64_t *)w.p, m,
                                   (const uint8_t *)kind.p, nx.p, s.o, o2.p, dest.p, (int)win_ranges);
                LAUNCH_OK();
            }
            Routed r;
            s.rt.send(o2.p, 2, dest.p, m, r, false);
            if (!r.total) break;
            w = std::move(r.in);
            m = r.n_in;
            // (round 6) the tail: once every rank's records in flight fit one block (they never
            // multiply), the rounds run in fixed blocks back to back on the device, one queued
            // all-to-all each, checked once per batch (an empty round changes nothing)
            if (walk_fixed && r.total <= walkP) {
                const int N = comm.world, R = comm.rank;
                const uint64_t P = walkP, bs = 1 + 2 * P;
                DevBuf<uint64_t> send((uint64_t)N * bs), recv((uint64_t)N * bs), sb[2];
                sb[0].alloc(bs);
                sb[1].alloc(bs);
                DevBuf<unsigned long long> tot(1);
                hipLaunchKernelGGL(k_blk_zero, dim3(1), dim3(kBlk), 0, st, recv.p, N, bs, (uint64_t *)nullptr);
                LAUNCH_OK();
                hipLaunchKernelGGL(k_walk_fx_seed, dim3(s.grid(2 * m + 1)), dim3(kBlk), 0, st, (const uint64_t *)w.p, m,
                                   sb[0].p);
                LAUNCH_OK();
                const unsigned gy = s.grid(P) / (unsigned)N + 1;
                const int K = (int)std::max<int64_t>(1, knob(ctx, "dist.walk_batch", 8));
                int t = 0;
                for (bool done = false; !done;) {
                    for (int b = 0; b < K; ++b, ++t, ++walk_rounds) {
                        hipLaunchKernelGGL(k_blk_zero, dim3(1), dim3(kBlk), 0, st, send.p, N, bs, sb[(t + 1) & 1].p);
                        LAUNCH_OK();
                        hipLaunchKernelGGL(k_walk_fx, dim3(gy, (unsigned)N), dim3(kBlk), 0, st, (const uint64_t *)recv.p,
                                           (const uint64_t *)sb[t & 1].p, R, P, (const uint8_t *)kind.p, nx.p, s.o, send.p,
                                           sb[(t + 1) & 1].p, (int)win_ranges);
                        LAUNCH_OK();
                        comm.alltoall_fixed(send.p, 8 * bs, recv.p);
                    }
                    hipLaunchKernelGGL(k_walk_fx_count, dim3(1), dim3(64), 0, st, (const uint64_t *)send.p, N, R, P,
                                       (const uint64_t *)sb[t & 1].p, tot.p);
                    LAUNCH_OK();
                    done = s.sum(read_u64(ctx, tot.p)) == 0;  // the batch's last round put nothing out
                }
                break;
            }
        }
    }
    verbose_mark(ctx, "shard_cf.peel_walk");
    // pointer jumping over the rulers still pointing at a ruler
    uint64_t jump_rounds = 0;
    {
        DevBuf<uint64_t> al;
        DevBuf<uint8_t> keep(nr + 1);
        uint64_t na = 0;
        if (nr) {
            hipLaunchKernelGGL(k_active_rulers, dim3(s.grid(nr)), dim3(kBlk), 0, st, (const uint64_t *)rl.p, nr,
                               (const uint64_t *)nx.p, keep.p);
            LAUNCH_OK();
            al.alloc(nr);
            na = s.select(rl.p, keep.p, nr, al.p);
        }
        const uint64_t total_rulers = s.sum(nr);
        int bound = 2;
        while ((1ULL << bound) < total_rulers + 1) ++bound;
        bound += 1;
        for (; jump_rounds < (uint64_t)bound; ++jump_rounds) {
            DevBuf<uint64_t> q(na ? na : 1);
            DevBuf<uint8_t> dest(na ? na : 1);
            if (na) {
                hipLaunchKernelGGL(k_jump_req, dim3(s.grid(na)), dim3(kBlk), 0, st, (const uint64_t *)al.p, na,
                                   (const uint64_t *)nx.p, s.o, q.p, dest.p);
                LAUNCH_OK();
            }
            Routed r;
            uint64_t active_all = 0;  // every rank's active rulers (round 5: a sum of its own first)
            s.rt.send(q.p, 1, dest.p, na, r, true, na, &active_all);
            if (active_all == 0) break;  // (the round carried nothing on any rank)
            DevBuf<uint64_t> ans(r.n_in + 1);
            if (r.n_in) {
                hipLaunchKernelGGL(k_jump_ans, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r.in.p, r.n_in,
                                   (const uint64_t *)nx.p, id_lo, ans.p);
                LAUNCH_OK();
            }
            s.rt.reply(r, ans.p, 1, q.p);
            if (na) {
                hipLaunchKernelGGL(k_jump_apply, dim3(s.grid(na)), dim3(kBlk), 0, st, (const uint64_t *)al.p, na,
                                   (const uint64_t *)q.p, nx.p, keep.p);
                LAUNCH_OK();
                DevBuf<uint64_t> al2(na);
                na = s.select(al.p, keep.p, na, al2.p);
                al = std::move(al2);
            }
        }
        // still pointing at a ruler after the bound: a unary cycle (or a chain into one) survives
        if (na) {
            hipLaunchKernelGGL(k_jump_cycle, dim3(s.grid(na)), dim3(kBlk), 0, st, (const uint64_t *)al.p, na, nx.p);
            LAUNCH_OK();
        }
    }
    verbose_mark(ctx, "shard_cf.peel_jumps");
    // branch successors' references (two lookups: the successor, then a claiming ruler's terminal)
    DevBuf<uint64_t> ref(4 * (nb ? nb : 1));  // per branch slot: its successor's reference, kPad unused
    if (nb) {
        hipLaunchKernelGGL(k_fill, dim3(s.grid(4 * nb)), dim3(kBlk), 0, st, ref.p, 4 * nb, kPad);
        LAUNCH_OK();
    }
    {
        DevBuf<uint64_t> q(4 * nb + 1);
        DevBuf<uint8_t> dest(4 * nb + 1);
        if (nb) {
            hipLaunchKernelGGL(k_bref_req, dim3(s.grid(nb)), dim3(kBlk), 0, st, (const uint64_t *)bl.p, nb,
                               (const uint8_t *)kind.p, (const uint64_t *)g->out_info.p, s.o, q.p, dest.p);
            LAUNCH_OK();
        }
        Routed r;
        s.rt.send(q.p, 1, dest.p, 4 * nb, r, true);
        DevBuf<uint64_t> ans(r.n_in + 1);
        if (r.n_in) {
            hipLaunchKernelGGL(k_bref_ans, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r.in.p, r.n_in,
                               (const uint8_t *)kind.p, (const uint64_t *)nx.p, id_lo, ans.p);
            LAUNCH_OK();
        }
        s.rt.reply(r, ans.p, 1, ref.p);  // slots without a successor keep kPad
        // second step: a claiming ruler's terminal replaces kRef | ruler
        if (nb) {
            hipLaunchKernelGGL(k_bref_req2, dim3(s.grid(4 * nb)), dim3(kBlk), 0, st, (const uint64_t *)ref.p, 4 * nb, s.o,
                               q.p, dest.p);
            LAUNCH_OK();
        }
        Routed r2;
        s.rt.send(q.p, 1, dest.p, 4 * nb, r2, true);
        DevBuf<uint64_t> ans2(r2.n_in + 1);
        if (r2.n_in) {
            hipLaunchKernelGGL(k_jump_ans, dim3(s.grid(r2.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r2.in.p, r2.n_in,
                               (const uint64_t *)nx.p, id_lo, ans2.p);
            LAUNCH_OK();
        }
        s.rt.reply(r2, ans2.p, 1, ref.p);
    }
    verbose_mark(ctx, "shard_cf.peel_bref");
    // branch resolution rounds (until no branch changes on any rank)
    uint64_t res_rounds = 0;
    // (round 6) in fixed blocks, the rounds back to back on the device in batches (a round after
    // one without a change changes nothing, so the batch's last round decides): one queued
    // all-to-all each way per round and one host wait per batch, against a routed exchange, a
    // reply and a sum (three host waits) per round. Blocks hold every slot of the rank with the
    // most branches; above dist.res_block_mb (64 MB of blocks) the routed rounds stay.
    const uint64_t nb_most = [&] {
        uint64_t x = 0;
        for (uint64_t v : comm.allgather_one(nb)) x = std::max(x, v);
        return x;
    }();
    const uint64_t resP = 4 * nb_most;
    const bool res_fixed = knob(ctx, "dist.res_fixed", 1) != 0 &&
                           8 * (uint64_t)comm.world * (1 + resP) <= ((uint64_t)std::max<int64_t>(1, knob(ctx, "dist.res_block_mb", 64)) << 20);
    if (res_fixed) {
        const int N = comm.world, R = comm.rank;
        const uint64_t m = 4 * nb, P = resP;
        DevBuf<uint64_t> q(m + 1), a(m + 1);
        DevBuf<uint8_t> dest(m + 1);
        DevBuf<uint32_t> pos(m + 1);
        DevBuf<uint64_t> send((uint64_t)N * (1 + P)), recv((uint64_t)N * (1 + P)), self_blk(1 + m);
        DevBuf<uint64_t> rsend((uint64_t)N * (1 + P)), rrecv((uint64_t)N * (1 + P)), rself(1 + m);
        const int K = (int)std::max<int64_t>(1, knob(ctx, "dist.res_batch", 8));
        for (bool done = false; !done;) {
            for (int b = 0; b < K; ++b, ++res_rounds) {
                HIP_OK(hipMemsetAsync(cnt.p + 7, 0, 8, st));
                hipLaunchKernelGGL(k_bfs_zero, dim3(1), dim3(kBlk), 0, st, send.p, N, P, self_blk.p);
                LAUNCH_OK();
                if (nb) {
                    hipLaunchKernelGGL(k_res_req, dim3(s.grid(nb)), dim3(kBlk), 0, st, (const uint64_t *)bl.p,
                                       (const uint64_t *)ref.p, nb, stt.p, s.o, q.p, dest.p, cnt.p + 7);
                    LAUNCH_OK();
                    hipLaunchKernelGGL(k_fx_post, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint64_t *)q.p,
                                       (const uint8_t *)dest.p, m, R, send.p, P, self_blk.p, pos.p);
                    LAUNCH_OK();
                }
                comm.alltoall_fixed(send.p, 8 * (1 + P), recv.p);
                hipLaunchKernelGGL(k_fx_st_ans, dim3(s.grid(std::max<uint64_t>(m, 1)) / (unsigned)N + 1, (unsigned)N),
                                   dim3(kBlk), 0, st, (const uint64_t *)recv.p, (const uint64_t *)self_blk.p, R, P,
                                   (const uint8_t *)stt.p, id_lo, rsend.p, rself.p);
                LAUNCH_OK();
                comm.alltoall_fixed(rsend.p, 8 * (1 + P), rrecv.p);
                if (nb) {
                    hipLaunchKernelGGL(k_fx_gather, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint8_t *)dest.p,
                                       (const uint32_t *)pos.p, m, R, (const uint64_t *)rrecv.p, P,
                                       (const uint64_t *)rself.p, a.p);
                    LAUNCH_OK();
                    hipLaunchKernelGGL(k_res_apply, dim3(s.grid(nb)), dim3(kBlk), 0, st, (const uint64_t *)bl.p, nb,
                                       (const uint64_t *)a.p, (const uint8_t *)dest.p, stt.p, cnt.p + 7);
                    LAUNCH_OK();
                }
            }
            const uint64_t ch = read_u64(ctx, cnt.p + 7);  // the batch's last round
            done = s.sum(ch) == 0;
        }
    } else {
        DevBuf<uint64_t> q(4 * nb + 1);
        DevBuf<uint8_t> dest(4 * nb + 1);
        for (;; ++res_rounds) {
            HIP_OK(hipMemsetAsync(cnt.p + 7, 0, 8, st));
            if (nb) {
                hipLaunchKernelGGL(k_res_req, dim3(s.grid(nb)), dim3(kBlk), 0, st, (const uint64_t *)bl.p,
                                   (const uint64_t *)ref.p, nb, stt.p, s.o, q.p, dest.p, cnt.p + 7);
                LAUNCH_OK();
            }
            Routed r;
            s.rt.send(q.p, 1, dest.p, 4 * nb, r, true);
            DevBuf<uint64_t> ans(r.n_in + 1);
            if (r.n_in) {
                hipLaunchKernelGGL(k_st_ans, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r.in.p, r.n_in,
                                   (const uint8_t *)stt.p, id_lo, ans.p);
                LAUNCH_OK();
            }
            s.rt.reply(r, ans.p, 1, q.p);
            if (nb) {
                hipLaunchKernelGGL(k_res_apply, dim3(s.grid(nb)), dim3(kBlk), 0, st, (const uint64_t *)bl.p, nb,
                                   (const uint64_t *)q.p, (const uint8_t *)dest.p, stt.p, cnt.p + 7);
                LAUNCH_OK();
            }
            const uint64_t ch = nb ? read_u64(ctx, cnt.p + 7) : 0;
            if (s.sum(ch) == 0) break;
        }
    }
    verbose_mark(ctx, "shard_cf.peel_resolution");
    // removal: resolved non-unary edges, rulers whose terminal went, and the chains they claimed
    uint64_t n_rm_rulers = 0;
    {
        if (nwl) {
            hipLaunchKernelGGL(k_rm_nonunary, dim3(s.grid(nwl * 64)), dim3(kBlk), 0, st, (const uint64_t *)post.p,
                               (const uint8_t *)kind.p, (const uint8_t *)stt.p, n, g->valid.p);
            LAUNCH_OK();
        }
        DevBuf<uint64_t> q(nr + 1);
        DevBuf<uint8_t> dest(nr + 1);
        if (nr) {
            hipLaunchKernelGGL(k_term_req, dim3(s.grid(nr)), dim3(kBlk), 0, st, (const uint64_t *)rl.p, nr,
                               (const uint64_t *)nx.p, s.o, q.p, dest.p);
            LAUNCH_OK();
        }
        Routed r;
        s.rt.send(q.p, 1, dest.p, nr, r, true);
        DevBuf<uint64_t> ans(r.n_in + 1);
        if (r.n_in) {
            hipLaunchKernelGGL(k_st_ans, dim3(s.grid(r.n_in)), dim3(kBlk), 0, st, (const uint64_t *)r.in.p, r.n_in,
                               (const uint8_t *)stt.p, id_lo, ans.p);
            LAUNCH_OK();
        }
        s.rt.reply(r, ans.p, 1, q.p);
        DevBuf<uint64_t> rm(nr + 1), gidr(nr + 1);
        DevBuf<uint8_t> flag(nr + 1);
        uint64_t nrm = 0;
        if (nr) {
            hipLaunchKernelGGL(k_rm_rulers, dim3(s.grid(nr)), dim3(kBlk), 0, st, (const uint64_t *)rl.p, nr,
                               (const uint64_t *)q.p, (const uint8_t *)dest.p, g->valid.p, id_lo, gidr.p, flag.p);
            LAUNCH_OK();
            nrm = s.select(gidr.p, flag.p, nr, rm.p);
        }
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
                                   (const uint8_t *)kind.p, (const uint64_t *)nx.p, n, (const uint64_t *)tab.p, cap,
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
    verbose_mark(ctx, "shard_cf.peel_removal");
    kind.release();
    stt.release();
    nx.release();
    rl.release();
    bl.release();
    ref.release();
    seed.release();
    timer.mark("peel");
    xr("peel");

    // 4-5. valid count; the candidates still valid, ascending on every rank
    HIP_OK(hipMemsetAsync(cnt.p, 0, 16, st));
    if (nwl) {
        hipLaunchKernelGGL(k_popc, dim3(s.grid(nwl)), dim3(kBlk), 0, st, (const uint64_t *)g->valid.p, nwl, cnt.p);
        LAUNCH_OK();
    }
    out->stats[2] = s.sum(read_u64(ctx, cnt.p));
    std::vector<uint64_t> cand_mine;  // the candidates still valid, ascending ids
    {
        if (nwl) {
            hipLaunchKernelGGL(k_and_words, dim3(s.grid(nwl)), dim3(kBlk), 0, st, cbits.p, (const uint64_t *)g->valid.p, nwl);
            LAUNCH_OK();
        }
        DevBuf<uint64_t> cl;
        const uint64_t nk = s.list_bits(cbits.p, cl);
        cand_mine.resize(nk);
        if (nk) d2h(ctx, cand_mine.data(), cl.p, 8 * nk);
        for (auto &x : cand_mine) x += id_lo;
    }
    cbits.release();
    post.release();
    timer.mark("recount");
    xr("recount");

    // 6. search regions: groups of the (k-1)-suffix (whole nodes' out-edges and in-groups)
    DevBuf<uint64_t> gs(nwl + 1), reg(nwl + 1), seen(nwl + 1);
    HIP_OK(hipMemsetAsync(gs.p, 0, gs.bytes(), st));
    if (nwl) {
        hipLaunchKernelGGL(k_gstart, dim3(s.grid(nwl * 64)), dim3(kBlk), 0, st, (const uint64_t *)g->key.p, n, gs.p);
        LAUNCH_OK();
    }
    const uint64_t radius = (uint64_t)p.cycle_max_length + 1;
    // (round 6) the region BFS hops run back to back on the device (ShardCf::bfs_dev);
    // dist.bfs_sync=1: round 5's form, one routed exchange with host waits per hop
    const bool bfs_sync = knob(ctx, "dist.bfs_sync", 0) != 0;
    auto forward_region = [&](const std::vector<uint64_t> &starts_mine) {
        if (!bfs_sync) {
            s.bfs_dev(starts_mine, radius, false, gs.p, reg.p, seen.p);
            return;
        }
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
    verbose_mark(ctx, "shard_cf.dls_region_bfs");
    mcaat_graph rg;
    const uint64_t rn = s.gather_region(reg.p, &rg);
    const std::vector<uint64_t> cand_all = [&] {
        std::vector<uint64_t> a = comm.allgather_vec(cand_mine);
        std::sort(a.begin(), a.end());
        return a;
    }();
    timer.mark("candidates");
    xr("candidates");
    if (verbose())
        fprintf(stderr, "[mcaat] shard %d: %zu candidates, DLS region %llu edges\n", comm.rank, cand_all.size(),
                (unsigned long long)rn);
    ctx->kstats["shard_dls_region_edges"].launches = rn;
    verbose_mark(ctx, "shard_cf.dls_begin");
    const std::vector<uint64_t> cand_c = s.to_compact(rg, rn, cand_all);
    verbose_mark(ctx, "shard_cf.dls_compact_ids");
    std::vector<uint64_t> pass_c = cf_depth_level_search(&rg, cand_c, p.cycle_max_length, &comm);
    verbose_mark(ctx, "shard_cf.dls_search");
    // buckets by ceil(log2 mult) (cycle_finder.cpp:414), descending; ascending ids within
    std::map<int, std::vector<uint64_t>, std::greater<int>> chunks;
    if (!pass_c.empty()) {
        const uint64_t m = pass_c.size();
        DevBuf<uint64_t> dc(m);
        DevBuf<uint16_t> dm(m);
        h2d(ctx, dc.p, pass_c.data(), 8 * m);
        hipLaunchKernelGGL(k_mult_of, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint16_t *)rg.mult.p,
                           (const uint64_t *)dc.p, m, dm.p);
        LAUNCH_OK();
        std::vector<uint16_t> hm(m);
        d2h(ctx, hm.data(), dm.p, 2 * m);
        const std::vector<uint64_t> ids = s.to_global(rg, rn, dc.p, m);
        for (uint64_t i = 0; i < m; ++i) chunks[(int)std::ceil(std::log2(double(hm[i])))].push_back(ids[i]);
    }
    std::vector<uint64_t> starts;
    for (auto &kv : chunks)
        for (uint64_t id : kv.second) {
            out->cand_ids.push_back(id);
            out->cand_bucket.push_back(kv.first);
            starts.push_back(id);
        }
    out->stats[4] = out->cand_ids.size();
    verbose_mark(ctx, "shard_cf.dls_buckets");
    // FindCycle's forward reach (cycle_max_length + 1 hops from the starts) lies inside the
    // DepthLevelSearch region (the starts are candidates): found on the replica, no exchange
    std::vector<uint64_t> fwd;  // its edge ids, ascending
    {
        const std::vector<uint64_t> sc = s.to_compact(rg, rn, starts);
        const uint64_t nwr = mcaat_graph::bitmap_words(rg.D);
        DevBuf<uint64_t> rseen(nwr);
        HIP_OK(hipMemsetAsync(rseen.p, 0, rseen.bytes(), st));
        const uint64_t nf = sc.size();
        if (nf && knob(ctx, "dist.bfs_sync", 0) == 0) {
            // (round 6) the hops back to back on the device: ping-pong frontiers of the replica's
            // size, per-hop counts in device memory (one host wait after the last hop instead of
            // one per hop: C3 at one rank, the DLS stage's 78 waits)
            DevBuf<uint64_t> fr[2];
            fr[0].alloc(rg.D + 1);
            fr[1].alloc(rg.D + 1);
            DevBuf<unsigned long long> cnt(radius + 1);
            HIP_OK(hipMemsetAsync(cnt.p, 0, cnt.bytes(), st));
            h2d(ctx, fr[0].p, sc.data(), 8 * nf);
            h2d(ctx, cnt.p, &nf, 8);
            hipLaunchKernelGGL(k_set_ids, dim3(s.grid(nf)), dim3(kBlk), 0, st, (const uint64_t *)fr[0].p, nf, rseen.p);
            LAUNCH_OK();
            const unsigned gcap = s.grid(rg.D);
            for (uint64_t h = 0; h < radius; ++h) {
                hipLaunchKernelGGL(k_cbfs_dev, dim3(gcap), dim3(kBlk), 0, st, rg.view(), (const uint64_t *)fr[h & 1].p,
                                   (const unsigned long long *)(cnt.p + h), rseen.p, fr[(h + 1) & 1].p, cnt.p + h + 1);
                LAUNCH_OK();
            }
            HIP_OK(hipStreamSynchronize(st));
        } else if (nf) {  // dist.bfs_sync=1: round 5's form, the frontier size read after every hop
            DevBuf<uint64_t> front(nf + 1);
            DevBuf<unsigned long long> nn(1);
            uint64_t m = nf;
            h2d(ctx, front.p, sc.data(), 8 * nf);
            hipLaunchKernelGGL(k_set_ids, dim3(s.grid(nf)), dim3(kBlk), 0, st, (const uint64_t *)front.p, nf, rseen.p);
            LAUNCH_OK();
            for (uint64_t h = 0; h < radius && m; ++h) {
                DevBuf<uint64_t> next(4 * m);
                HIP_OK(hipMemsetAsync(nn.p, 0, 8, st));
                hipLaunchKernelGGL(k_cbfs, dim3(s.grid(m)), dim3(kBlk), 0, st, rg.view(), (const uint64_t *)front.p, m,
                                   rseen.p, next.p, nn.p);
                LAUNCH_OK();
                m = read_u64(ctx, nn.p);
                front = std::move(next);
            }
        }
        // the reached compact ids, ascending, as edge ids (ascending too); the null group's
        // positions past the region's edges come last and are dropped
        DevBuf<uint64_t> rl;
        const uint64_t nl = s.list_bits(rseen.p, rl, nwr);
        fwd = s.to_global(rg, rn, rl.p, nl);
        while (!fwd.empty() && fwd.back() == ~0ULL) fwd.pop_back();
    }
    verbose_mark(ctx, "shard_cf.fc_reach");
    rg = mcaat_graph{};
    timer.mark("dls");
    xr("dls");

    // 7. FindCycle region: the forward reach found on the DepthLevelSearch replica above, then
    // cycle_max_length + 1 hops backward from every edge of it (the lock relaxation's reach)
    {
        // this rank's edges of the forward reach: their groups, and the sources of the backward BFS
        const auto a = std::lower_bound(fwd.begin(), fwd.end(), id_lo), b = std::lower_bound(fwd.begin(), fwd.end(), id_lo + n);
        const std::vector<uint64_t> sm(a, b);
        if (!bfs_sync) s.bfs_dev(sm, radius, true, gs.p, reg.p, seen.p);
        else {
        HIP_OK(hipMemsetAsync(reg.p, 0, reg.bytes(), st));
        HIP_OK(hipMemsetAsync(seen.p, 0, seen.bytes(), st));
        const uint64_t m = sm.size();
        DevBuf<uint64_t> ids(m + 1), front(m + 1);
        if (m) {
            h2d(ctx, ids.p, sm.data(), 8 * m);
            hipLaunchKernelGGL(k_bfs_seed, dim3(s.grid(m)), dim3(kBlk), 0, st, (const uint64_t *)ids.p, m, id_lo, n,
                               (const uint64_t *)gs.p, reg.p, seen.p, front.p);
            LAUNCH_OK();
        }
        s.bfs(front, m, radius, true, gs.p, reg.p, seen.p);
        }
    }
    mcaat_graph fg;
    const uint64_t fn = s.gather_region(reg.p, &fg);
    reg.release();
    seen.release();
    gs.release();
    ctx->kstats["shard_fc_region_edges"].launches = fn;
    if (verbose())
        fprintf(stderr, "[mcaat] shard %d: %zu FindCycle starts, region %llu edges; %llu exchanges, %llu records\n",
                comm.rank, starts.size(), (unsigned long long)fn, (unsigned long long)s.rt.rounds,
                (unsigned long long)s.rt.records);
    ctx->kstats["shard_exchanges"].launches = s.rt.rounds;
    if (verbose())
        fprintf(stderr, "[mcaat] shard %d: routing host ms: grouping %.1f, count all-gather %.1f, placement %.1f, "
                        "all-to-all %.1f, replies %.1f\n",
                comm.rank, s.rt.t_count, s.rt.t_gather, s.rt.t_place, s.rt.t_a2a, s.rt.t_reply);
    mcaat_cycles local;
    cf_find_cycles(&fg, p, s.to_compact(fg, fn, starts), &local, &comm);
    {
        // the results' compact ids back to edge ids in one translation: the starts, then every flat list
        std::vector<uint64_t> all(local.starts);
        for (const auto &fl : local.flat) all.insert(all.end(), fl.begin(), fl.end());
        const std::vector<uint64_t> g_all = s.to_global(fg, fn, all);
        size_t at = local.starts.size();
        for (size_t i = 0; i < local.starts.size(); ++i) {
            out->starts.push_back(g_all[i]);
            out->flat.emplace_back(g_all.begin() + at, g_all.begin() + at + local.flat[i].size());
            at += local.flat[i].size();
            out->offsets.push_back(std::move(local.offsets[i]));
        }
    }
    out->stats[5] = local.stats[5];
    out->stats[6] = local.stats[6];
    out->stats[7] = local.stats[7];
    timer.mark("find_cycle");
    xr("find_cycle");
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

void preload_shard_cf() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, (const void *)k_route_count);
}

}  // namespace mcaat
