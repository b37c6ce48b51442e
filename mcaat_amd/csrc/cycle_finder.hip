// cycle_finder.hip — CycleFinder (reference cycle_finder.cpp:131-492) on gfx950.
//
// Stages:
//   1. CollectTips (:346-357)                -> wave-ballot bitmap scan
//   2. InvalidateMultiplicityOneNodes (:372) -> wave-ballot bitmap AND
//   3. RecursiveReduction (:359-371)          -> parallel peel fixpoint: unary chains are
//      resolved by ruler walks + pointer jumping (list ranking), branch nodes by a short
//      iteration. Same result as the recursion (monotone least fixpoint).
//   4. valid count / tips again (:443-452)   -> popcount scans
//   5. ChunkStartNodes (:387-427)            -> filter kernel + one DLS thread per candidate
//   6. bucket loop of FindCycle (:468-487)   -> speculative FindCycle, one thread per start
//      against a `visited` snapshot, committed on the host in the reference's threads=1
//      order; a start whose search read a node that an earlier commit marked visited is
//      re-run (its footprint is its lock table).
// The libstdc++ unordered_set iteration order of FindCycle's neighbour frames is emulated
// exactly (13 buckets, identity hash; DESIGN.md "FindCycle frame order").
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <map>
#include <unordered_set>

#include "comm.h"

namespace mcaat {

namespace {

constexpr int kBlock = 256;
constexpr uint64_t kNone = ~0ULL;
constexpr uint8_t kUnk = 0, kRem = 1, kSurv = 2;

// ------------------------------- peel --------------------------------------
// kind[e]: low 6 bits the valid out-degree (0..4; 0x3F invalid edge), 0x80 when e is a
// ruler, 0x40 when e is a successor of a branch node (only those nodes' owners are ever
// read, so a walk stores no other owner: the walk is one random read per step).
// nxk[e] (unary e): its sole successor in bits 0..55 and the successor's kind in 56..63, so a
// ruler walk pays one dependent load per step.
constexpr uint8_t kInvalid = 0x3F, kRulerBit = 0x80, kBranchSucc = 0x40;
constexpr uint64_t kNodeMask = (1ULL << 56) - 1;
__device__ __forceinline__ int kind_od(uint8_t k) { return k & 0x3F; }
__device__ __forceinline__ bool kind_chain(uint8_t k) { return (k & 0xBF) == 1; }  // unary, not a ruler

// Per-ruler words live in arrays indexed by the ruler's position in the ruler list, so the
// only D-sized arrays are the flag words (4 B), nxk (8 B) and owner (4 B): 16 B per edge
// (the graph itself is 26 B per edge; C5's ~4e9-edge graph must fit beside it).
// jump[i]: kRRef | index of the next ruler (kRSuper when that ruler is a super ruler), or the
// terminal node id (a non-unary node), or kNone (a ruler-less unary cycle)
constexpr uint64_t kRRef = 1ULL << 62, kRSuper = 1ULL << 61, kRIdx = (1ULL << 40) - 1;
constexpr uint32_t kNoOwner = 0xFFFFFFFFu;

// a node's four flag bytes share one word (nf[4e + field]), so a walk or a successor check
// touches one line per node instead of one per byte array
enum : int { kFKind = 0, kFUpred = 1, kFBpred = 2, kFSt = 3 };
struct PeelArrays {
    uint8_t *nf;      // per node: kind; upred (1: some unary node points here); bpred (1: some
                      // branch node, out-degree >= 2, points here); st (kUnk / kRem / kSurv,
                      // non-unary nodes)
    __device__ __forceinline__ uint8_t &kind(uint64_t e) const { return nf[4 * e + kFKind]; }
    __device__ __forceinline__ uint8_t &upred(uint64_t e) const { return nf[4 * e + kFUpred]; }
    __device__ __forceinline__ uint8_t &bpred(uint64_t e) const { return nf[4 * e + kFBpred]; }
    __device__ __forceinline__ uint8_t &st(uint64_t e) const { return nf[4 * e + kFSt]; }
    __device__ __forceinline__ uchar4 flags(uint64_t e) const { return *(const uchar4 *)(nf + 4 * e); }
    uint64_t *nxk;    // successor | successor kind << 56 (unary nodes)
    uint32_t *owner;  // rulers: their own list index; non-ruler branch successors: the list index
                      // of the ruler whose walk passed them (kNoOwner: none); others unused
    uint64_t *jump;   // per ruler (list index), see kRRef; after k_peel_final: terminal or kNone
    uint32_t *sowner; // per ruler: the super ruler whose walk over rulers passed it (itself for a
                      // super ruler, kNoOwner: none)
    const uint64_t *seed;  // tips bitmap collected before the multiplicity filter
    // Round 4: the per-edge arrays above hold only the edges valid after the multiplicity filter,
    // at their rank among them (cidx): post is that filter's bitmap as the peel starts (the peel
    // clears bits in the graph's own copy, never in this one), wpre[w] the set bits of its words
    // before w. Null wpre: the arrays are indexed by edge id (every edge has a slot).
    const uint64_t *post;
    const uint32_t *wpre;
    uint64_t nw;
    __device__ __forceinline__ uint64_t cidx(uint64_t e) const {
        if (!wpre) return e;
        const uint64_t w = e >> 6;
        return (uint64_t)wpre[w] + (uint64_t)__popcll(post[w] & ((1ull << (e & 63)) - 1));
    }
    // the edge id of slot c (wpre non-null; only on the removal path: the removed edges)
    __device__ __forceinline__ uint64_t gid(uint64_t c) const {
        if (!wpre) return c;
        uint64_t lo = 0, hi = nw;  // last word w with wpre[w] <= c holds slot c
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if ((uint64_t)wpre[mid] <= c) lo = mid;
            else hi = mid;
        }
        uint64_t x = post[lo];
        for (uint32_t r = (uint32_t)(c - wpre[lo]); r; --r) x &= x - 1;
        return lo * 64 + (uint64_t)__builtin_ctzll(x);
    }
};

// ------------------------------- scans -------------------------------------
// one wave per 64-edge bitmap word, kScanU words per iteration with all their loads in flight
// together: the out-edges of e are the consecutive ids [lo, lo + cnt), so its valid out-degree
// is a popcount of at most two bitmap words (no per-successor loads); the in-edges of e are the
// positions of a 16-bit mask inside the group starting at in_lo, so the valid in-degree and the
// self-loop test of the candidate filter are two bitmap words as well
// (knob cf.scan_u). More words per wave means fewer waves: C3 recount with 1 / 2 / 4 / 8 words
// 5.5 / 5.7 / 8.3 / 18.0 ms (79 VGPRs at 2, 141 at 4, 256 at 8), the occupancy matters more
// (round 6) default 1: the tips / filter pass C3 14.3 -> 13.8 ms, C5 50.1 -> 46.0 (4: 61.2);
// cf.scan_u=2 keeps round 3's two words
constexpr int kScanUDefault = 1;

// A wave's appends to a global id list, staged in LDS and published 64 at a time with one
// cursor atomic (at C5 the candidates and the peel's branch nodes occur in most waves, and an
// atomic per wave on one counter serialised tens of millions of them). `buf` is this wave's
// 128-entry LDS slice; `n` is wave-uniform. Entries past `cap` are counted, not written (the
// caller re-runs with the counted size).
struct WaveList {
    uint64_t *buf;
    uint64_t *out;
    unsigned long long *cursor;
    uint64_t cap;
    uint32_t n = 0;
    __device__ __forceinline__ void wave_fence() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __device__ __forceinline__ void publish(uint32_t count) {  // the first `count` (<= 64)
        const int lane = threadIdx.x & 63;
        wave_fence();
        unsigned long long at = 0;
        if (lane == 0) at = atomicAdd(cursor, (unsigned long long)count);
        at = __shfl(at, 0);
        const uint64_t v = buf[lane], keep = buf[64 + lane];
        if ((uint32_t)lane < count && at + lane < cap) out[at + lane] = v;
        wave_fence();
        if (count == 64) buf[lane] = keep;  // the rest moves to the front
        n -= count;
        wave_fence();
    }
    __device__ __forceinline__ void push(bool f, uint64_t v) {
        const unsigned long long m = __ballot(f);
        if (!m) return;
        const int lane = threadIdx.x & 63;
        if (f) buf[n + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] = v;
        n += (uint32_t)__popcll(m);
        if (n >= 64) publish(64);
        (void)lane;
    }
    __device__ __forceinline__ void finish() {
        if (n) publish(n);
    }
};

// InvalidateMultiplicityOneNodes (round 4: a pass of its own, ahead of CollectTips): post[w]
// (indexed from w_lo) = the valid bits of word w whose edge has multiplicity > 1, and counts[1]
// += every mult <= 1 edge (the reference counts valid or not). The tips pass then reads the
// filtered bitmap where it needs post-filter validity (one window per neighbour set instead of
// the neighbours' multiplicities), and its popcounts give the peel's compact slots.
// the valid bits of word w of a graph whose every edge is valid (mcaat_graph::all_valid)
__device__ __forceinline__ uint64_t word_ones(uint64_t w, uint64_t D) {
    const uint64_t e0 = w * 64;
    return e0 + 64 <= D ? ~0ull : e0 < D ? (~0ull >> (64 - (D - e0))) : 0ull;
}

template <int kScanU>
__global__ void __launch_bounds__(kBlock) k_post_filter(GraphView g, uint64_t w_lo, uint64_t w_hi, uint64_t *post,
                                                        unsigned long long *counts, bool fresh) {
    const int lane = threadIdx.x & 63;
    const uint64_t wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    unsigned long long low_n = 0;
    for (uint64_t wb = w_lo + (((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6); wb < w_hi; wb += kScanU * wstride) {
        uint64_t sv[kScanU];
        uint32_t mu[kScanU];
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const uint64_t w = wb + u * wstride, e = w * 64 + lane;
            sv[u] = w < w_hi ? (fresh ? word_ones(w, g.D) : g.valid[w]) : 0;
            mu[u] = e < g.D && w < w_hi ? g.mult[e] : 0xFFFFu;
        }
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const uint64_t w = wb + u * wstride;
            const unsigned long long lowm = __ballot(mu[u] <= 1);
            if (lane == 0 && w < w_hi) {
                post[w - w_lo] = sv[u] & ~lowm;
                low_n += __popcll(lowm);
            }
        }
    }
    block_add(counts + 1, low_n);
}

// set bits per word (the exclusive scan of these is PeelArrays::wpre)
__global__ void __launch_bounds__(kBlock) k_word_pop(const uint64_t *bm, uint64_t nw, uint32_t *cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) cnt[w] = __popcll(bm[w]);
}

// CollectTips from the valid bits before the filter (every successor window is read from
// `valid`, which this pass does not write), counts[0] tips, into tip_bm (indexed from w_lo).
// `post` is the whole filtered bitmap (k_post_filter; all ranks' words).
// With pa.nf (the list-ranking peel's arrays, nf zeroed) the pass also does the peel's first
// D-wide pass (k_peel_init) from the same loads: an edge's filtered valid out-degree is one
// window of post over its successors (consecutive ids), so kinds, unary successors and the
// predecessor flags come out here instead of from a second streaming pass over out_info and
// the filtered bitmap; with pa.wpre they go to the edges' compact slots (PeelArrays::cidx).
// words [w_lo, w_hi) (a rank's share; all of them on one GPU)
// With a candidate list (cand != nullptr) the pass also does the recount's work on the
// post-filter graph (round 3): counts[2] post-filter tips that are not seeds (every one of them
// survives the peel, and no surviving edge becomes a tip: the reduction removes every valid edge
// whose successors it all removed), and ChunkStartNodes' filter on post-filter validity
// (valid, mult > thr, at least two valid in-edges, not its own in-edge) into cand (counts[3]
// counts them all). A removed edge had no valid successor, so the peel changes no surviving
// edge's valid in-edges: the final candidates are these, still valid after the peel.
// (round 5) fresh and pull are template parameters: the default form (fresh, no pull) then keeps
// none of the other forms' registers (C3: 105 VGPRs, four waves per SIMD, in one kernel for all)
template <int kScanU, bool kFresh, bool kPull>
// fresh: every edge is valid before the filter (mcaat_graph::all_valid), so an edge is a tip
// iff it has no out-edges at all, and no window of the unfiltered bitmap is read
// pull (round 4, with the peel's arrays): an edge writes its own predecessor flags instead of
// each predecessor setting a byte at its successors' slots. All predecessors of y share y's
// source node, so their filtered out-degree is the number of filter-valid siblings of y (the
// out-edges of that node: consecutive ids, and with any predecessor present exactly the ids
// around y whose in_info word equals y's), and y has one iff its in-edge window holds a
// filter-valid edge. One 4-byte store per edge, no scattered byte stores and no clearing pass.
__global__ void __launch_bounds__(kBlock) k_tips_filter(GraphView g, uint64_t w_lo, uint64_t w_hi, uint64_t *tip_bm,
                                                        const uint64_t *post, unsigned long long *counts, PeelArrays pa,
                                                        uint64_t thr, uint64_t *cand, uint64_t cap) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (g.D + 63) / 64;
    const uint64_t wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const bool peel = pa.nf != nullptr, fold = cand != nullptr;
    constexpr bool fresh = kFresh;
    const bool pull = kPull && peel;
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    __shared__ uint64_t cbuf[kBlock / 64][128];
    WaveList cl{cbuf[threadIdx.x >> 6], cand, counts + 3, cap};
    unsigned long long acc = 0, tips_pf = 0;
    for (uint64_t wb = w_lo + (((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6); wb < w_hi; wb += kScanU * wstride) {
        uint64_t sv[kScanU], pv[kScanU], oi[kScanU], xb[kScanU];
        WordPair a[kScanU], a2[kScanU];
        uint32_t mu[kScanU];
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const uint64_t w = wb + u * wstride, e = w * 64 + lane;
            sv[u] = w < w_hi ? (fresh ? word_ones(w, g.D) : g.valid[w]) : 0;
            pv[u] = w < w_hi ? post[w] : 0;
            oi[u] = e < g.D && w < w_hi ? g.out_info[e] : 0;
            mu[u] = e < g.D && w < w_hi && fold ? g.mult[e] : 0;
            // pull: lanes 0..2 and 61..63 hold the in_info words of the 3 ids on either side of
            // the word (0 unless filter-valid), for their neighbours' sibling counts
            xb[u] = 0;
            if (pull && w < w_hi && (lane < 3 || lane > 60)) {
                const int64_t y = lane < 3 ? (int64_t)(w * 64) - 3 + lane : (int64_t)(w * 64) + 64 + (lane - 61);
                if (y >= 0 && (uint64_t)y < g.D) {  // both loads issued together
                    const uint64_t x = g.in_info[y], pw = post[(uint64_t)y >> 6];
                    xb[u] = ((pw >> (y & 63)) & 1) ? x : 0;
                }
            }
        }
        uint64_t ii[kScanU];
        WordPair b[kScanU];
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const uint64_t w = wb + u * wstride, e = w * 64 + lane;
            // the candidate filter's in-edge window, for post-filter valid edges above thr
            const bool cv = e < g.D && w < w_hi && ((pv[u] >> lane) & 1) && (pull || (fold && (uint64_t)mu[u] > thr));
            ii[u] = cv ? g.in_info[e] : 0;
        }
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const uint64_t lo = oi[u] & kIdxMask;
            if (!fresh) a[u] = word_pair(g.valid, lo, nw);
            if (peel || fold) a2[u] = word_pair(post, lo, nw);
            if (fold || pull) b[u] = word_pair(post, ii[u] & kIdxMask, nw);
        }
        // pull: filter-valid siblings of each edge (equal in_info words within 3 ids); the ids
        // outside the wave's word come from the neighbouring words, read only by the lanes at
        // its ends that need them
        uint32_t sib[kScanU];
        if (pull) {
#pragma unroll
            for (int u = 0; u < kScanU; ++u) {
                const uint64_t w = wb + u * wstride, e = w * 64 + lane;
                const uint64_t my = ii[u];
                uint32_t c = 0;
#pragma unroll
                for (int d = -3; d <= 3; ++d) {
                    if (!d) continue;
                    const int nl = lane + d;
                    // every lane shuffles (uniform): the neighbour's word from its lane, or from the
                    // lane holding that id outside the word (xb, loaded with the scan's other loads)
                    const uint64_t x = __shfl(my, nl & 63);
                    const uint64_t xo = __shfl(xb[u], nl < 0 ? nl + 3 : (nl - 64 + 61) & 63);
                    c += (nl >= 0 && nl < 64 ? x : xo) == my;
                }
                (void)e;
                sib[u] = c + 1;  // and the edge itself
            }
        }
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const uint64_t w = wb + u * wstride, e = w * 64 + lane;
            const uint64_t lo = oi[u] & kIdxMask;
            const uint32_t cnt = __popc((unsigned)(oi[u] >> kIdxBits) & 0xF);
            const uint32_t pre = fresh ? ((1u << cnt) - 1) : bits16(a[u].a, a[u].b, lo) & ((1u << cnt) - 1);
            const bool t = ((sv[u] >> lane) & 1) && pre == 0;
            const unsigned long long m = __ballot(t);
            if (lane == 0 && w < w_hi) {
                tip_bm[w - w_lo] = m;
                acc += __popcll(m);
            }
            const bool vpf = e < g.D && w < w_hi && ((pv[u] >> lane) & 1);  // valid after the filter
            const unsigned pfo = (peel || fold) ? bits16(a2[u].a, a2[u].b, lo) & ((1u << cnt) - 1) : 0;  // successors valid after it
            if (fold) {
                // a post-filter tip that is not a seed (t: a pre-filter tip, i.e. a seed)
                const unsigned long long tpm = __ballot(vpf && pfo == 0 && !t);
                if (lane == 0) tips_pf += __popcll(tpm);
                bool c = false;
                if (vpf && (uint64_t)mu[u] > thr) {
                    const uint64_t l = ii[u] & kIdxMask;
                    const unsigned in = bits16(b[u].a, b[u].b, l) & (uint32_t)((ii[u] >> kIdxBits) & 0xFFFF);  // post-filter valid in-edges
                    const bool self = e >= l && e - l < 16 && ((in >> (e - l)) & 1);
                    c = __popc(in) >= 2 && !self;
                }
                cl.push(c, e);
            }
            // (an edge invalid after the filter gets no kind byte: prep reads the filtered bitmap
            // first, and every other pass reaches only valid edges)
            if (peel && e < g.D && w < w_hi) {
                if (vpf) {
                    const uint64_t ce = pa.wpre ? (uint64_t)pa.wpre[w] + __popcll(pv[u] & lt) : e;
                    // compact slot of successor lo + i: its word is lo's or the next one
                    auto cs = [&](int i) -> uint64_t {
                        const uint64_t y = lo + i;
                        if (!pa.wpre) return y;
                        const uint64_t wy = y >> 6;
                        const uint64_t pw = wy == this_word(lo, nw) ? a2[u].a : a2[u].b;
                        return (uint64_t)pa.wpre[wy] + __popcll(pw & ((1ull << (y & 63)) - 1));
                    };
                    int od = 0, i1 = -1;
                    for (int i = (int)cnt - 1; i >= 0; --i)  // descending ids, as dev_outgoing
                        if ((pfo >> i) & 1) {
                            ++od;
                            i1 = i;
                        }
                    if (pull) {
                        const uint64_t l = ii[u] & kIdxMask;
                        const bool haspred = (bits16(b[u].a, b[u].b, l) & (uint32_t)((ii[u] >> kIdxBits) & 0xFFFF)) != 0;
                        const uint32_t up = haspred && sib[u] == 1, bp = haspred && sib[u] >= 2;
                        *(uint32_t *)(pa.nf + 4 * ce) = (uint32_t)od | (up << (8 * kFUpred)) | (bp << (8 * kFBpred));
                        if (od == 1) pa.nxk[ce] = cs(i1);
                    } else {
                        pa.kind(ce) = (uint8_t)od;
                        if (od == 1) {
                            const uint64_t cy = cs(i1);
                            pa.nxk[ce] = cy;
                            pa.upred(cy) = 1;
                        } else {
                            for (int i = (int)cnt - 1; i >= 0; --i)
                                if ((pfo >> i) & 1) pa.bpred(cs(i)) = 1;
                        }
                    }
                }
            }
        }
    }
    if (fold) cl.finish();
    block_add(counts, acc);
    block_add(counts + 2, tips_pf);
}

// popcount of bitmap words [w_lo, w_hi)
__global__ void __launch_bounds__(kBlock) k_popcount(const uint64_t *bm, uint64_t w_lo, uint64_t w_hi,
                                                     unsigned long long *out) {
    unsigned long long c = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = w_lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < w_hi; w += stride) c += __popcll(bm[w]);
    block_add(out, c);
}

// the candidates still valid (flags for select_flagged)
__global__ void __launch_bounds__(kBlock) k_still_valid(const uint64_t *bm, const uint64_t *ids, uint64_t n, uint8_t *f) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) f[i] = bit_get(bm, ids[i]);
}

// the recount after the reduction (valid edges, tips) and ChunkStartNodes' candidate filter in
// one pass: counts[0] valid, counts[1] tips (whole graph), candidates only in [lo, hi) (a rank's
// share), appended to list while they fit in cap (counts[2] counts them all)
// the words covering ids [lo, hi) (a rank's share; all of them on one GPU): counts over those
// words (summed over the ranks), candidates among ids [lo, hi)
template <int kScanU>
__global__ void __launch_bounds__(kBlock) k_recount_candidates(GraphView g, uint64_t thr, uint64_t lo, uint64_t hi,
                                                               uint64_t w_lo, uint64_t w_hi, uint64_t *list,
                                                               uint64_t cap, unsigned long long *counts) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (g.D + 63) / 64;
    const uint64_t wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    unsigned long long nvalid = 0, ntips = 0;
    __shared__ uint64_t wbuf[kBlock / 64][128];
    WaveList wl{wbuf[threadIdx.x >> 6], list, counts + 2, cap};
    for (uint64_t wb = w_lo + (((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6); wb < w_hi; wb += kScanU * wstride) {
        uint64_t sv[kScanU], oi[kScanU], ii[kScanU];
        WordPair a[kScanU], b[kScanU];
        uint32_t mu[kScanU];
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const uint64_t w = wb + u * wstride, e = w * 64 + lane;
            const bool in = e < g.D && w < w_hi;
            sv[u] = w < w_hi ? g.valid[w] : 0;
            oi[u] = in ? g.out_info[e] : 0;
            const bool cr = in && e >= lo && e < hi && ((sv[u] >> lane) & 1);
            ii[u] = cr ? g.in_info[e] : 0;
            mu[u] = cr ? g.mult[e] : 0;
        }
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            a[u] = word_pair(g.valid, oi[u] & kIdxMask, nw);
            b[u] = word_pair(g.valid, ii[u] & kIdxMask, nw);
        }
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const uint64_t w = wb + u * wstride, e = w * 64 + lane;
            const bool v = (sv[u] >> lane) & 1;
            const uint32_t cnt = __popc((unsigned)(oi[u] >> kIdxBits) & 0xF);
            const bool t = v && (bits16(a[u].a, a[u].b, oi[u] & kIdxMask) & ((1u << cnt) - 1)) == 0;
            const unsigned long long tm = __ballot(t);
            if (lane == 0 && w < w_hi) {
                ntips += __popcll(tm);
                nvalid += __popcll(sv[u]);
            }
            const uint64_t l = ii[u] & kIdxMask;
            const uint32_t in = bits16(b[u].a, b[u].b, l) & (uint32_t)((ii[u] >> kIdxBits) & 0xFFFF);  // valid in-edges
            // _IncomingNotEqualToCurrentNode: e must not be one of its own in-edges
            const bool self = e >= l && e - l < 16 && ((in >> (e - l)) & 1);
            const bool c = v && e >= lo && e < hi && (uint64_t)mu[u] > thr && __popc(in) >= 2 && !self;
            wl.push(c, e);
        }
    }
    wl.finish();
    block_add(counts, nvalid);
    block_add(counts + 1, ntips);
}



// super rulers: chain heads and 1 in 64 of the other rulers (a ruler reached from another
// ruler has a unary predecessor, so for it the hash alone decides)
constexpr uint64_t kSuperMask = 63;
__device__ __forceinline__ bool peel_super_hash(uint64_t r) { return (mix64(r ^ 0xbeefULL) & kSuperMask) == 0; }

// pass 1 (D-wide): out-degree, the unary successor, unary- and branch-predecessor flags
// (g.valid: the filtered bitmap, equal to pa.post when the arrays are compact)
__global__ void __launch_bounds__(kBlock) k_peel_init(GraphView g, PeelArrays pa) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < g.D; e += stride) {
        if (!bit_get(g.valid, e)) continue;  // no kind byte: prep reads the bitmap first
        uint64_t out[4];
        const int n = dev_outgoing(g, e, out);
        const uint64_t ce = pa.cidx(e);
        pa.kind(ce) = (uint8_t)n;
        if (n == 1) {
            const uint64_t cy = pa.cidx(out[0]);
            pa.nxk[ce] = cy;
            pa.upred(cy) = 1;
        } else {
            for (int j = 0; j < n; ++j) pa.bpred(pa.cidx(out[j])) = 1;
        }
    }
}

// pass 2 (D-wide): final kind bytes (ruler, branch-successor), each unary node's successor
// packed with the successor's final kind (computed here from its flags, so the walk pays
// one dependent load per step), non-unary states; rulers (unary chain heads plus 1 in
// ruler_mask + 1 others) compacted into list with one cursor atomic per 4096-edge tile,
// branch nodes and removed seeds into blist
constexpr int kTileJ = 16;  // 64-edge words per wave per tile
// (list / blist hold cap / bcap entries; the cursors count past them, and the driver then
// runs the pass again with larger lists: it is idempotent)
template <int kPB>
__global__ void __launch_bounds__(kBlock) k_peel_prep(uint64_t D, PeelArrays pa, uint64_t ruler_mask, uint64_t *list,
                                                      uint64_t cap, unsigned long long *cursor, uint64_t *blist,
                                                      uint64_t bcap, unsigned long long *bcursor) {
    __shared__ uint32_t wcnt[kBlock / 64];
    __shared__ unsigned long long tbase;
    __shared__ uint64_t bbuf[kBlock / 64][128];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    WaveList bl{bbuf[wave], blist, bcursor, bcap};
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t tile = (uint64_t)kBlock * kTileJ;
    for (uint64_t t0 = (uint64_t)blockIdx.x * tile; t0 < D; t0 += (uint64_t)gridDim.x * tile) {
        unsigned long long m[kTileJ];
        uint32_t c = 0;
        // kPB edges per thread at a time: their own bytes and successors are loaded first (all
        // in flight together), then their successors' flags, then everything is written
        static_assert(kTileJ % kPB == 0, "whole batches per tile");
#pragma unroll
        for (int h = 0; h < kTileJ; h += kPB) {
            uint8_t od[kPB], bp[kPB], up[kPB], oy[kPB], by[kPB], uy[kPB];
            uint64_t y[kPB];
            uint64_t ce[kPB];
#pragma unroll
            for (int q = 0; q < kPB; ++q) {
                const uint64_t e = t0 + (uint64_t)(h + q) * kBlock + threadIdx.x;
                // a wave's 64 edges are one word of the filtered bitmap: edges without a valid
                // bit have no slot (compact arrays) or an invalid kind
                const uint64_t pw = e < D ? pa.post[e >> 6] : 0;
                const bool valid = (pw >> (e & 63)) & 1;
                ce[q] = pa.wpre && valid ? (uint64_t)pa.wpre[e >> 6] + __popcll(pw & lt) : e;
                // other lanes may already have set their own kind bits: the low 6 are the degree
                const uchar4 f = valid ? pa.flags(ce[q]) : make_uchar4(kInvalid, 0, 0, 0);
                od[q] = (uint8_t)(f.x & 0x3F);
                up[q] = f.y;
                bp[q] = f.z;
            }
#pragma unroll
            for (int q = 0; q < kPB; ++q)
                y[q] = od[q] == 1 ? (pa.nxk[ce[q]] & kNodeMask) : 0;  // masked: prep may run again
#pragma unroll
            for (int q = 0; q < kPB; ++q) {
                oy[q] = by[q] = uy[q] = 0;
                if (od[q] == 1) {
                    const uchar4 f = pa.flags(y[q]);
                    oy[q] = f.x & 0x3F;
                    uy[q] = f.y;
                    by[q] = f.z;
                }
            }
#pragma unroll
            for (int q = 0; q < kPB; ++q) {
                const int j = h + q;
                const uint64_t e = t0 + (uint64_t)j * kBlock + threadIdx.x;
                const uint64_t cq = ce[q];
                bool r = false, br = false;
                if (od[q] != kInvalid) {
                    uint8_t k = od[q] | (bp[q] ? kBranchSucc : 0);
                    if (od[q] == 1) {
                        // the ruler hash is of the slot (compact or id): the same on every rank
                        r = up[q] == 0 || (mix64(cq ^ 0x5eed) & ruler_mask) == 0;
                        if (r) k |= kRulerBit;
                        // owners: rulers get their list index below; of the others only branch
                        // successors' are ever read (peel_res)
                        if (!r && bp[q]) pa.owner[cq] = kNoOwner;
                        uint8_t ky = oy[q] | (by[q] ? kBranchSucc : 0);
                        if (oy[q] == 1 && (uy[q] == 0 || (mix64(y[q] ^ 0x5eed) & ruler_mask) == 0)) ky |= kRulerBit;
                        pa.nxk[cq] = y[q] | ((uint64_t)ky << 56);
                    } else if (od[q] == 0) {
                        const bool rm = bit_get(pa.seed, e);
                        pa.st(cq) = rm ? kRem : kSurv;
                        br = rm;
                    } else {
                        pa.st(cq) = kUnk;
                        br = true;
                    }
                    pa.kind(cq) = k;
                }
                m[j] = __ballot(r);
                c += __popcll(m[j]);
                bl.push(br, e);
            }
        }
        if (lane == 0) wcnt[wave] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (int w = 0; w < kBlock / 64; ++w) {
                const uint32_t x = wcnt[w];
                wcnt[w] = t;
                t += x;
            }
            tbase = t ? atomicAdd(cursor, (unsigned long long)t) : 0;
        }
        __syncthreads();
        uint64_t off = tbase + wcnt[wave];
#pragma unroll
        for (int j = 0; j < kTileJ; ++j) {
            if ((m[j] >> lane) & 1) {
                const uint64_t i = off + __popcll(m[j] & lt), e = t0 + (uint64_t)j * kBlock + threadIdx.x;
                if (i < cap) {
                    const uint64_t c = pa.cidx(e);  // rulers are listed by slot
                    list[i] = c;
                    pa.owner[c] = (uint32_t)i;
                }
            }
            off += __popcll(m[j]);
        }
        __syncthreads();
    }
    bl.finish();
}

// each ruler walks its chain to the next ruler or non-unary node (Brent cycle check) and
// records what it reached in jump (a ruler by its list index, read from its owner word)
__global__ void __launch_bounds__(kBlock) k_peel_walk(PeelArrays pa, const uint64_t *list, uint64_t nr) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += stride) {
        const uint64_t r = list[i];
        uint64_t w = pa.nxk[r], tort = r;
        uint64_t power = 1, lam = 1;
        uint64_t res = kNone;
        for (;;) {
            const uint64_t y = w & kNodeMask;
            const uint8_t ky = (uint8_t)(w >> 56);
            if (!kind_chain(ky)) {
                if (kind_od(ky) == 1)  // a ruler, reached from a unary node: super by the hash alone
                    res = kRRef | (peel_super_hash(y) ? kRSuper : 0) | (uint64_t)pa.owner[y];
                else
                    res = y;
                break;
            }
            if (y == tort) { res = kNone; break; }  // ruler-less unary cycle reached
            if (ky & kBranchSucc) pa.owner[y] = (uint32_t)i;
            if (power == lam) { tort = y; power <<= 1; lam = 0; }
            w = pa.nxk[y];
            ++lam;
        }
        pa.jump[i] = res;
    }
}

// list ranking one level up: each super ruler walks the rulers of its chain (one jump load per
// ruler) to the next super ruler or terminal, marking itself as their owner, and is listed
__global__ void __launch_bounds__(kBlock) k_peel_super(PeelArrays pa, const uint64_t *list, uint64_t nr,
                                                       uint32_t *slist, unsigned long long *scursor) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < nr; i0 += stride) {
        const uint64_t i = i0 + threadIdx.x;
        bool sup = false;
        if (i < nr) {
            const uint64_t r = list[i];
            sup = pa.upred(r) == 0 || peel_super_hash(r);
        }
        const unsigned long long m = __ballot(sup);
        if (m) {
            unsigned long long off = 0;
            if (lane == 0) off = atomicAdd(scursor, (unsigned long long)__popcll(m));
            off = __shfl(off, 0);
            if (sup) slist[off + __popcll(m & lt)] = (uint32_t)i;
        }
        if (!sup) continue;
        pa.sowner[i] = (uint32_t)i;
        uint64_t w = pa.jump[i], tort = i, power = 1, lam = 1;
        for (;;) {
            if (w == kNone || !(w & kRRef) || (w & kRSuper)) break;  // cycle, terminal or super ruler
            const uint64_t x = w & kRIdx;
            if (x == tort) { w = kNone; break; }  // a cycle of rulers without a super ruler
            pa.sowner[x] = (uint32_t)i;
            if (power == lam) { tort = x; power <<= 1; lam = 0; }
            w = pa.jump[x];
            ++lam;
        }
        // a super ruler's jump is only read by its own walks from here on (walks stop at it)
        pa.jump[i] = w;
    }
}

// one pointer-jumping round over the super rulers; *changed is raised when some super ruler
// still pointed at a ruler (a round that changes nothing proves every jump final)
__global__ void __launch_bounds__(kBlock) k_peel_jump(PeelArrays pa, const uint32_t *slist, uint64_t ns, int *changed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    bool ch = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += stride) {
        const uint32_t s = slist[i];
        const uint64_t j = pa.jump[s];
        if (j != kNone && (j & kRRef)) {
            const uint64_t t = pa.jump[j & kRIdx];
            if (t != j) {
                pa.jump[s] = t;
                ch = true;
            }
        }
    }
    if (__ballot(ch) && (threadIdx.x & 63) == 0) *changed = 1;
}

// every ruler's terminal: a super ruler's own jump, another ruler's through its super owner
// (kNone: on a cycle); only non-super entries are written, only super entries read
__global__ void __launch_bounds__(kBlock) k_peel_final(PeelArrays pa, uint64_t nr) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += stride) {
        const uint32_t o = pa.sowner[i];
        if (o == (uint32_t)i) continue;
        pa.jump[i] = o == kNoOwner ? kNone : pa.jump[o];
    }
}

__device__ __forceinline__ uint8_t peel_res(const PeelArrays &pa, uint64_t y) {
    const uchar4 f = pa.flags(y);
    const uint8_t k = f.x;
    if (kind_od(k) != 1) return f.w;
    const uint32_t o = pa.owner[y];
    if (o == kNoOwner) return kSurv;  // unary node on a ruler-less cycle
    const uint64_t t = pa.jump[o];
    if (t == kNone || (t & kRRef)) return kSurv;
    const uchar4 ft = pa.flags(t);
    if (kind_od(ft.x) == 1) return kSurv;  // chain ends in a unary cycle
    return ft.w;
}

__global__ void __launch_bounds__(kBlock) k_peel_branch(GraphView g, PeelArrays pa, const uint64_t *blist,
                                                        uint64_t nb, int *changed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += stride) {
        const uint64_t b = blist[i], cb = pa.cidx(b);  // blist: edge ids
        if (pa.st(cb) != kUnk) continue;
        uint64_t out[4];
        const int n = dev_outgoing(g, b, out);
        bool all_rem = true, any_surv = false;
        for (int j = 0; j < n; ++j) {
            const uint8_t r = peel_res(pa, pa.cidx(out[j]));
            if (r == kSurv) any_surv = true;
            if (r != kRem) all_rem = false;
        }
        if (any_surv) { pa.st(cb) = kSurv; *changed = 1; }
        else if (all_rem) { pa.st(cb) = kRem; *changed = 1; }
    }
}

__device__ __forceinline__ void clear_valid(GraphView &g, uint64_t e) {
    atomicAnd((unsigned long long *)&g.valid[e >> 6], ~(1ull << (e & 63)));
}

// removal: listed non-unary nodes resolved kRem, and the chain segments of rulers whose
// terminal was removed (each segment re-walked; only removed ones are visited)
__global__ void __launch_bounds__(kBlock) k_peel_apply_list(GraphView g, PeelArrays pa, const uint64_t *blist,
                                                            uint64_t nb) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += stride)
        if (pa.st(pa.cidx(blist[i])) == kRem) clear_valid(g, blist[i]);
}

__global__ void __launch_bounds__(kBlock) k_peel_apply_rulers(GraphView g, PeelArrays pa, const uint64_t *list,
                                                              uint64_t nr) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += stride) {
        const uint64_t r = list[i];  // slots; their edge ids by pa.gid (removed edges only)
        if (peel_res(pa, r) != kRem) continue;  // a removed chain ends at a non-unary node: no cycle
        clear_valid(g, pa.gid(r));
        for (uint64_t w = pa.nxk[r]; kind_chain((uint8_t)(w >> 56)); w = pa.nxk[w & kNodeMask])
            clear_valid(g, pa.gid(w & kNodeMask));
    }
}

// ---- counter-driven peel (Kahn-style) ----
// rem[e] = number of valid successors of a valid edge. Removing a child decrements each valid
// parent; the thread whose decrement reaches zero owns that parent, removes it and keeps
// walking, so every parent is removed exactly when its last valid child is (the reference's
// recursion fixpoint) and chains are walked without a kernel per level.
__global__ void __launch_bounds__(kBlock) k_kahn_init(GraphView g, const uint64_t *seed, uint32_t *rem, uint64_t *out,
                                                      unsigned long long *cursor) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (g.D + 63) / 64;
    const uint64_t wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += wstride) {
        const uint64_t e = w * 64 + lane;
        bool f = false;
        if (e < g.D) {
            uint32_t od = 0;
            if (bit_get(g.valid, e)) od = (uint32_t)dev_outdeg(g, e);
            rem[e] = od;
            f = od == 0 && ((seed[w] & g.valid[w]) >> lane) & 1;
        }
        const unsigned long long m = __ballot(f);
        unsigned long long off = 0;
        if (lane == 0 && m) off = atomicAdd(cursor, (unsigned long long)__popcll(m));
        off = __shfl(off, 0);
        if (f) out[off + __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))))] = e;
    }
}

__global__ void __launch_bounds__(kBlock) k_kahn_walk(GraphView g, uint32_t *rem, const uint64_t *f, uint64_t n,
                                                      uint64_t *next, unsigned long long *cursor, uint32_t budget,
                                                      uint64_t *pend, unsigned long long *pend_n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t t = f[i];
        for (uint32_t step = 0;; ++step) {
            if (step == budget) {  // long chain: leave t (counter already zero, still valid) pending
                pend[atomicAdd(pend_n, 1ull)] = t;
                break;
            }
            // parents are read before t is invalidated (valid-only in-edges of t)
            uint64_t in[4];
            const int ni = dev_incoming(g, t, in);
            atomicAnd((unsigned long long *)&g.valid[t >> 6], ~(1ull << (t & 63)));
            uint64_t cont = kNone;
            for (int j = 0; j < ni; ++j) {
                if (atomicSub(&rem[in[j]], 1u) != 1u) continue;
                if (cont == kNone) cont = in[j];
                else next[atomicAdd(cursor, 1ull)] = in[j];
            }
            if (cont == kNone) break;
            t = cont;
        }
    }
}

__global__ void __launch_bounds__(kBlock) k_ids_to_bits(const uint64_t *ids, uint64_t n, uint64_t *bm) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        atomicOr((unsigned long long *)&bm[ids[i] >> 6], 1ull << (ids[i] & 63));
}

// ------------------------------ DLS ------------------------------------------
// DepthLevelSearch(v, v, limit) (cycle_finder.cpp:248-343), one thread per candidate.
// res: 1 found, 0 not found, -1 scratch overflow (re-run with larger caps)
__device__ __forceinline__ bool set_insert(uint64_t *tab, uint32_t cap, uint64_t x, uint32_t &size, bool &over) {
    uint32_t s = (uint32_t)(mix64(x) & (cap - 1));
    for (;;) {
        const uint64_t c = tab[s];
        if (c == x) return false;
        if (c == kNone) {
            if (size + 1 > cap / 4 * 3) { over = true; return false; }
            tab[s] = x;
            ++size;
            return true;
        }
        s = (s + 1) & (cap - 1);
    }
}
__device__ __forceinline__ bool set_contains(const uint64_t *tab, uint32_t cap, uint64_t x) {
    uint32_t s = (uint32_t)(mix64(x) & (cap - 1));
    for (;;) {
        const uint64_t c = tab[s];
        if (c == x) return true;
        if (c == kNone) return false;
        s = (s + 1) & (cap - 1);
    }
}

__global__ void __launch_bounds__(kBlock) k_dls(GraphView g, const uint64_t *cand, uint64_t n, int limit,
                                                uint64_t *stack_all, uint32_t cs, uint64_t *vis_all, uint32_t cv,
                                                int8_t *res, int lpw) {
    // lpw searches per wave (divergent searches serialise each other's branches); the whole
    // wave first clears their visited sets, then lanes >= lpw leave
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64 * lpw;
    {
        const uint64_t nw_s = w0 < n ? (n - w0 < (uint64_t)lpw ? n - w0 : (uint64_t)lpw) : 0;
        uint64_t *v0 = vis_all + w0 * cv;
        for (uint64_t j = threadIdx.x & 63; j < nw_s * cv; j += 64) v0[j] = kNone;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    if ((int)(threadIdx.x & 63) >= lpw) return;
    const uint64_t i = w0 + (threadIdx.x & 63);
    if (i >= n) return;
    uint64_t *stk = stack_all + i * cs;
    uint64_t *vis = vis_all + i * cv;
    const uint64_t start = cand[i];
    uint32_t sp = 0, vsize = 0;
    bool over = false;
    stk[sp++] = start << 8;  // (node << 8) | depth
    int8_t found = 0;
    while (sp > 0) {
        const uint64_t top = stk[--sp];
        const uint64_t v = top >> 8;
        const int depth = (int)(top & 0xFF);
        if (!bit_get(g.valid, v)) continue;
        uint64_t nb[4];
        const int od = dev_outgoing(g, v, nb);
        if (od == 0) continue;  // EdgeOutdegreeZero
        if (depth >= limit) continue;
        for (int j = 0; j < od; ++j) {
            const uint64_t x = nb[j];
            const bool nv = !set_contains(vis, cv, x);
            const bool sr = (x == start && depth > 0);
            if (nv || sr) {
                set_insert(vis, cv, x, vsize, over);
                if (sp >= cs) over = true;
                if (over) break;
                stk[sp++] = (x << 8) | (uint64_t)(depth + 1);
            }
        }
        if (over) break;
        if (v == start && depth > 1) { found = 1; break; }
    }
    res[i] = over ? -1 : found;
}

// (round 4) The same search with scratch per lane instead of per candidate: lane q of the
// launch takes candidates q, q + L, q + 2L, ... (L lanes in all), so a wave's time is the sum of
// its lanes' searches, not the longest search of one batch, and every candidate gets the large
// scratch. The visited table is not cleared between searches: an entry carries its search's
// generation in bits 56..63 (node ids are below 2^56), and entries of other generations read
// as empty; the table is cleared when the 8-bit generation wraps.
__device__ __forceinline__ bool gset_insert(uint64_t *tab, uint32_t cap, uint64_t x, uint64_t gen, uint32_t &size,
                                            bool &over) {
    const uint64_t tx = (gen << 56) | x;
    uint32_t s = (uint32_t)(mix64(x) & (cap - 1));
    for (;;) {
        const uint64_t c = tab[s];
        if (c == tx) return false;
        if ((c >> 56) != gen) {
            if (size + 1 > cap / 4 * 3) { over = true; return false; }
            tab[s] = tx;
            ++size;
            return true;
        }
        s = (s + 1) & (cap - 1);
    }
}
__device__ __forceinline__ bool gset_contains(const uint64_t *tab, uint32_t cap, uint64_t x, uint64_t gen) {
    const uint64_t tx = (gen << 56) | x;
    uint32_t s = (uint32_t)(mix64(x) & (cap - 1));
    for (;;) {
        const uint64_t c = tab[s];
        if (c == tx) return true;
        if ((c >> 56) != gen) return false;
        s = (s + 1) & (cap - 1);
    }
}

// vis_all zeroed by the caller (generation 0 = empty); lpw active lanes per wave
__global__ void __launch_bounds__(kBlock) k_dls_lanes(GraphView g, const uint64_t *cand, uint64_t n, int limit,
                                                      uint64_t *stack_all, uint32_t cs, uint64_t *vis_all, uint32_t cv,
                                                      int8_t *res, int lpw, uint64_t n_lanes) {
    const int lane = threadIdx.x & 63;
    if (lane >= lpw) return;
    const uint64_t q = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64 * lpw + lane;
    if (q >= n_lanes) return;
    uint64_t *stk = stack_all + q * cs;
    uint64_t *vis = vis_all + q * cv;
    uint64_t gen = 0;
    for (uint64_t i = q; i < n; i += n_lanes) {
        if (++gen == 256) {
            for (uint32_t j = 0; j < cv; ++j) vis[j] = 0;
            gen = 1;
        }
        const uint64_t start = cand[i];
        uint32_t sp = 0, vsize = 0;
        bool over = false;
        stk[sp++] = start << 8;  // (node << 8) | depth
        int8_t found = 0;
        while (sp > 0) {
            const uint64_t top = stk[--sp];
            const uint64_t v = top >> 8;
            const int depth = (int)(top & 0xFF);
            if (!bit_get(g.valid, v)) continue;
            uint64_t nb[4];
            const int od = dev_outgoing(g, v, nb);
            if (od == 0) continue;  // EdgeOutdegreeZero
            if (depth >= limit) continue;
            for (int j = 0; j < od; ++j) {
                const uint64_t x = nb[j];
                const bool nv = !gset_contains(vis, cv, x, gen);
                const bool sr = (x == start && depth > 0);
                if (nv || sr) {
                    gset_insert(vis, cv, x, gen, vsize, over);
                    if (sp >= cs) over = true;
                    if (over) break;
                    stk[sp++] = (x << 8) | (uint64_t)(depth + 1);
                }
            }
            if (over) break;
            if (v == start && depth > 1) { found = 1; break; }
        }
        res[i] = over ? -1 : found;
    }
}

// (round 5) The same search with its visited set and stack in LDS (cf.dls_lds, default): a wave
// runs kLdsLanes searches, each with a kLdsVis-slot visited table of 32-bit ids (overflow at
// vmax <= 3/4, as set_insert) and a kLdsStk-entry stack (id + depth byte): 26 KB per 64-thread
// workgroup, six per CU, one launch for any number of candidates (no scratch). Searches that
// overflow report -1 and run again with the global-scratch kernel and larger caps, as before;
// results are the same for any caps that do not overflow. Needs D < 2^32 - 1 (~0 marks an empty
// slot). Pushed neighbours come from dev_outgoing (valid only), so only the start's validity is
// tested (the loop's first pop did that). Measured at C5 (3.8 M candidates): 41.7 ms against
// 42.4 for the global-scratch batches — DepthLevelSearch is bound by its two dependent graph
// reads per expansion (out_info, then the targets' validity window), not by the visited set or
// the stack; a variant feeding each lane its next candidate from a counter (so no lane waits
// for its wave's longest search) took 47.7 ms (fewer resident searches, a ballot per step).
// (round 6) Being latency-bound, it gains from more resident searches at smaller caps (overflows
// re-run): 40 searches per wave with 128 visited slots (96 used) and 16 stack entries, 23.7 KB,
// six workgroups and 240 searches per CU (round 5: 16 x 256 / 128, 96 per CU). C5 DLS 41.6 ->
// 34.1 ms, C3 2.9 -> 2.5 (`profiles/r06_c5_dls_lanes_ab.txt`: 32 x 128 / 64 39.1, 40 x 128 / 32
// 36.3, 48 x 128 / 16 34.8, 64 x 64 / 32 51.9).
#ifndef MCAAT_DLS_LANES
#define MCAAT_DLS_LANES 40
#define MCAAT_DLS_VIS 128
#define MCAAT_DLS_STK 16
#endif
constexpr int kLdsLanes = MCAAT_DLS_LANES, kLdsVis = MCAAT_DLS_VIS, kLdsStk = MCAAT_DLS_STK;
__global__ void __launch_bounds__(64) k_dls_lds(GraphView g, const uint64_t *cand, uint64_t n, int limit, int8_t *res,
                                                uint32_t vmax, uint32_t smax) {
    __shared__ uint32_t vis_s[kLdsLanes][kLdsVis];
    __shared__ uint32_t stk_s[kLdsLanes][kLdsStk];
    __shared__ uint8_t dep_s[kLdsLanes][kLdsStk];
    const int lane = threadIdx.x;
    for (int j = lane; j < kLdsLanes * kLdsVis; j += 64) (&vis_s[0][0])[j] = ~0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (lane >= kLdsLanes) return;
    const uint64_t i = (uint64_t)blockIdx.x * kLdsLanes + lane;
    if (i >= n) return;
    uint32_t *vis = vis_s[lane];
    uint32_t *stk = stk_s[lane];
    uint8_t *dep = dep_s[lane];
    const uint64_t start = cand[i];
    if (!bit_get(g.valid, start)) {
        res[i] = 0;
        return;
    }
    uint32_t sp = 1, vsize = 0;
    bool over = false;
    stk[0] = (uint32_t)start;
    dep[0] = 0;
    int8_t found = 0;
    while (sp > 0) {
        --sp;
        const uint64_t v = stk[sp];
        const int depth = dep[sp];
        uint64_t nb[4];
        const int od = dev_outgoing(g, v, nb);
        if (od == 0) continue;  // EdgeOutdegreeZero
        if (depth >= limit) continue;
        for (int j = 0; j < od; ++j) {
            const uint32_t x = (uint32_t)nb[j];
            uint32_t sl = (uint32_t)(mix64(nb[j]) & (kLdsVis - 1));
            bool present = false;
            for (;;) {
                const uint32_t c = vis[sl];
                if (c == x) { present = true; break; }
                if (c == ~0u) break;
                sl = (sl + 1) & (kLdsVis - 1);
            }
            const bool sr = (nb[j] == start && depth > 0);
            if (!present || sr) {
                if (!present) {
                    if (vsize + 1 > vmax) over = true;
                    else {
                        vis[sl] = x;
                        ++vsize;
                    }
                }
                if (sp >= smax) over = true;
                if (over) break;
                stk[sp] = x;
                dep[sp] = (uint8_t)(depth + 1);
                ++sp;
            }
        }
        if (over) break;
        if (v == start && depth > 1) { found = 1; break; }
    }
    res[i] = over ? -1 : found;
}

// ---------------------------- FindCycle ----------------------------------------
struct FcCaps {
    uint32_t P;    // path/frames capacity (max_len + 2)
    uint32_t CL;   // lock/footprint table (power of two)
    uint32_t CR;   // relax stack
    uint32_t CO;   // output nodes
    uint32_t CC;   // output cycle count (cluster bound)
};
struct FcParams {
    int maxl, minl, cluster;
    int64_t step_cap;
};
// lock / footprint table entry: key and value in one 16-B record (one line per probe)
struct __attribute__((aligned(16))) LockRec {
    uint64_t key;
    int32_t val;
    uint32_t onpath;  // 1 while the node is on the search path (path nodes are distinct)
};
// Per search: the hot state read every step (path, neighbour frames, backtrack lengths) is in
// the workgroup's LDS; the lock table, relax stack, the frames' out_info words and the outputs
// are in global scratch (fc_per_search bytes per search).
// A frame keeps, per candidate, the lock slot and out_info word loaded when the frame was
// built, and a relax record keeps its node's lock slot and in_info word, so a push or a
// relaxation waits for one round of graph loads (every load of it issued together), not three.
struct RelaxRec {
    uint64_t ub;    // node << 16 | backtrack length
    uint64_t ii;    // node's in_info word (0: no predecessors to visit)
    int32_t slot;   // node's lock slot
    uint32_t pad;
};
struct FcScratch {
    uint64_t *path;     // P      (LDS)
    int32_t *bl;        // P      (LDS)
    int32_t *psl;       // P      (LDS) lock slot of each path node
    uint64_t *fr;       // 4P     (LDS) frame candidates
    int32_t *frs;       // 4P     (LDS) their lock slots
    uint8_t *frm;       // P      (LDS) live-candidate mask of each frame
    LockRec *lk;        // CL     (global)
    RelaxRec *relax;    // CR     (global)
    uint64_t *froi;     // 4P     (global) frame candidates' out_info words
    uint64_t *out;      // CO     (global)
    uint16_t *olen;     // CC     (global)
};
__host__ __device__ inline uint64_t fc_out_offset(const FcCaps &c) {
    return (uint64_t)c.CL * 16 + (uint64_t)c.CR * sizeof(RelaxRec) + (uint64_t)c.P * 32;
}
__host__ __device__ inline uint64_t fc_per_search(const FcCaps &c) {
    const uint64_t per = fc_out_offset(c) + (uint64_t)c.CO * 8 + (uint64_t)c.CC * 2;
    return (per + 255) & ~255ULL;
}
__host__ __device__ inline uint32_t fc_lds_bytes(const FcCaps &c) { return c.P * (8 + 4 + 4 + 32 + 16 + 1) + 16; }
struct FcStatus {
    int32_t status;     // 0 ok, 1 lock table full, 2 relax stack full, 3 output full
    int32_t ncyc;
    uint32_t nnodes;
    uint32_t steps;  // main-loop iterations (diagnostics: MCAAT_VERBOSE)
    uint32_t relax;  // lock-relaxation expansions (diagnostics)
    uint32_t locks;  // lock-table entries at the end (diagnostics)
};

// x % 13 with 32-bit arithmetic (2^32 = 9 mod 13)
__device__ __forceinline__ uint32_t mod13(uint64_t x) {
    return (((uint32_t)(x >> 32) % 13u) * 9u + (uint32_t)x % 13u) % 13u;
}

struct FcThread {
    const GraphView &g;
    const uint64_t *visited;
    FcScratch s;
    FcCaps c;
    uint32_t lsize = 0;
    int32_t status = 0;

    __device__ FcThread(const GraphView &gv, const uint64_t *vis, FcScratch sc, FcCaps cp)
        : g(gv), visited(vis), s(sc), c(cp) {}

    // lock.try_emplace(x, maxl): returns slot (inserting default), -1 on overflow
    __device__ int lock_slot(uint64_t x, int dflt) {
        uint32_t h = (uint32_t)(mix64(x) & (c.CL - 1));
        for (;;) {
            const uint64_t k = s.lk[h].key;
            if (k == x) return (int)h;
            if (k == kNone) {
                if (lsize + 1 > c.CL / 4 * 3) { status = 1; return -1; }
                s.lk[h].key = x;
                s.lk[h].val = dflt;
                s.lk[h].onpath = 0;
                ++lsize;
                return (int)h;
            }
            h = (h + 1) & (c.CL - 1);
        }
    }
    // lock_slot(x) whose first probe record (slot h0, key k0) was loaded ahead of this call's
    // insertions: a prefetched slot filled since (wr[0..nwr)) is read again
    __device__ int lock_from(uint64_t x, int dflt, uint32_t h0, uint64_t k0, uint32_t *wr, int &nwr) {
        uint32_t h = h0;
        uint64_t k = k0;
        for (int w = 0; w < nwr; ++w)
            if (wr[w] == h) k = s.lk[h].key;
        for (;;) {
            if (k == x) return (int)h;
            if (k == kNone) {
                if (lsize + 1 > c.CL / 4 * 3) { status = 1; return -1; }
                s.lk[h].key = x;
                s.lk[h].val = dflt;
                s.lk[h].onpath = 0;
                ++lsize;
                wr[nwr++] = h;
                return (int)h;
            }
            h = (h + 1) & (c.CL - 1);
            k = s.lk[h].key;
        }
    }
    // _BackgroundCheck (cycle_finder.cpp:40-52) of neighbour x (multiplicity mu, visited bit
    // q) after its footprint record: integer rm / mu > 500 rejects (mu = 0 as well: the
    // device's division by zero is all ones)
    __device__ static bool background_ok(uint64_t node, uint64_t x, uint64_t rm, uint32_t mu, bool q) {
        if (q) return false;
        if (mu == 0 || rm / mu > 500) return false;
        return node != x;
    }

    // Frame of node (out_info oi, node valid): _GetOutgoings(node, set, rm) in the libstdc++
    // unordered_set insertion order, each candidate with its lock slot and out_info word. The
    // successors are the consecutive ids [lo, lo + cnt): their valid and visited windows and,
    // per id, the multiplicity, out_info word and first lock record are one round of loads.
    // Written to frame d; returns its live mask.
    __device__ uint8_t build_frame(uint64_t node, uint64_t oi, uint64_t rm, int maxl, uint32_t d) {
        const uint64_t nw = (g.D + 63) / 64;
        const uint64_t lo = oi & kIdxMask;
        const int cnt = __popc((unsigned)(oi >> kIdxBits) & 0xF);
        if (cnt == 0) return 0;
        const WordPair vw = word_pair(g.valid, lo, nw), qw = word_pair(visited, lo, nw);
        uint32_t mu[4];
        uint64_t no[4], k0[4];
        uint32_t h0[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            mu[i] = 0;
            no[i] = 0;
            h0[i] = 0;
            k0[i] = 0;
            if (i < cnt) {
                const uint64_t x = lo + i;
                mu[i] = g.mult[x];
                no[i] = g.out_info[x];
                h0[i] = (uint32_t)(mix64(x) & (c.CL - 1));
                k0[i] = s.lk[h0[i]].key;
            }
        }
        const uint32_t vb = bits16(vw.a, vw.b, lo) & ((1u << cnt) - 1);
        const uint32_t qb = bits16(qw.a, qw.b, lo);
        uint64_t fx[4] = {0, 0, 0, 0}, fo[4] = {0, 0, 0, 0};
        int32_t fs[4] = {0, 0, 0, 0};
        uint32_t fm[4] = {0, 0, 0, 0};
        uint32_t wr[4];
        int nwr = 0, n = 0;
        // valid successors in descending id order (OutgoingEdges), each recorded in the
        // footprint before its check
#pragma unroll
        for (int i = 3; i >= 0; --i) {
            if (i >= cnt || !((vb >> i) & 1)) continue;
            const uint64_t x = lo + i;
            const int sl = lock_from(x, maxl, h0[i], k0[i], wr, nwr);
            if (sl < 0) continue;
            if (!background_ok(node, x, rm, mu[i], (qb >> i) & 1)) continue;
            // 13 buckets, hash(x) = x: before the first element of x's bucket, else at front
            const uint32_t xm = mod13(g.gid ? g.gid[x] : x);  // region replicas: the edge id's bucket
            int pos = 0;
            bool hit = false;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (!hit && j < n && fm[j] == xm) { pos = j; hit = true; }
#pragma unroll
            for (int j = 3; j > 0; --j)
                if (j <= n && j > pos) { fx[j] = fx[j - 1]; fo[j] = fo[j - 1]; fs[j] = fs[j - 1]; fm[j] = fm[j - 1]; }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j == pos) { fx[j] = x; fo[j] = no[i]; fs[j] = sl; fm[j] = xm; }
            ++n;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < n) {
                s.fr[4 * d + j] = fx[j];
                s.frs[4 * d + j] = fs[j];
                s.froi[4 * d + j] = fo[j];
            }
        return (uint8_t)((1u << n) - 1);
    }

    // valid predecessors of node (in_info ii; node valid) passing the background check, in
    // ascending ids, with their lock slots and in_info words; one round of loads as above.
    __device__ int preds_of(uint64_t node, uint64_t ii, uint64_t rm, uint64_t *f, int32_t *fs, uint64_t *fii, int maxl) {
        const uint64_t nw = (g.D + 63) / 64;
        const uint64_t lo = ii & kIdxMask;
        uint32_t mask = (uint32_t)(ii >> kIdxBits) & 0xFFFF;
        if (mask == 0) return 0;
        // positions of the mask (an in-group holds one edge per source node: at most 4)
        int pj[4];
        int m = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            pj[q] = 0;
            if (mask) {
                pj[q] = __ffs(mask) - 1;
                mask &= mask - 1;
                m = q + 1;
            }
        }
        const WordPair vw = word_pair(g.valid, lo, nw), qw = word_pair(visited, lo, nw);
        uint32_t mu[4];
        uint64_t ni[4], k0[4];
        uint32_t h0[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            mu[q] = 0;
            ni[q] = 0;
            h0[q] = 0;
            k0[q] = 0;
            if (q < m) {
                const uint64_t x = lo + pj[q];
                mu[q] = g.mult[x];
                ni[q] = g.in_info[x];
                h0[q] = (uint32_t)(mix64(x) & (c.CL - 1));
                k0[q] = s.lk[h0[q]].key;
            }
        }
        const uint32_t vb = bits16(vw.a, vw.b, lo);
        const uint32_t qb = bits16(qw.a, qw.b, lo);
        uint32_t wr[4];
        int nwr = 0, n = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q >= m || !((vb >> pj[q]) & 1)) continue;
            const uint64_t x = lo + pj[q];
            const int sl = lock_from(x, maxl, h0[q], k0[q], wr, nwr);
            if (sl < 0) continue;
            if (!background_ok(node, x, rm, mu[q], (qb >> pj[q]) & 1)) continue;
            f[n] = x;
            fs[n] = sl;
            fii[n] = ni[q];
            ++n;
        }
        return n;
    }
};

// A/B knob: minimum waves per SIMD (6 or 8 force 80 / 64 VGPRs with spills; measured no
// faster at C3: the kernel's time is its longest search, not its occupancy)
#ifndef MCAAT_FC_MINW
#define MCAAT_FC_MINW 1
#endif
// One search per workgroup of one wave: the search itself is sequential (lane 0); the other
// lanes clear its lock table first. Its path and frames live in LDS (fc_lds_bytes), so every
// step touches global memory only for the graph, the visited bits, the lock table and the
// frames' out_info words.
// (Per-step latency, not occupancy, bounds this kernel: at C3 ~1.5K steps per search, each a
// chain of dependent loads.)
__global__ void __launch_bounds__(64, MCAAT_FC_MINW) k_findcycle(GraphView g, const uint64_t *visited, const uint64_t *starts,
                                                  uint64_t n, FcCaps caps, FcParams prm, uint64_t *sbase,
                                                  FcStatus *stat) {
    extern __shared__ __attribute__((aligned(16))) unsigned char fc_lds[];
    const uint64_t i = blockIdx.x;
    if (i >= n) return;
    uint8_t *base = (uint8_t *)sbase + i * fc_per_search(caps);
    FcScratch s;
    s.lk = (LockRec *)base; base += (uint64_t)caps.CL * 16;
    s.relax = (RelaxRec *)base; base += (uint64_t)caps.CR * sizeof(RelaxRec);
    s.froi = (uint64_t *)base; base += (uint64_t)caps.P * 32;
    s.out = (uint64_t *)base; base += (uint64_t)caps.CO * 8;
    s.olen = (uint16_t *)base;
    unsigned char *lb = fc_lds;
    s.path = (uint64_t *)lb; lb += (uint64_t)caps.P * 8;
    s.fr = (uint64_t *)lb; lb += (uint64_t)caps.P * 32;
    s.frs = (int32_t *)lb; lb += (uint64_t)caps.P * 16;
    s.bl = (int32_t *)lb; lb += (uint64_t)caps.P * 4;
    s.psl = (int32_t *)lb; lb += (uint64_t)caps.P * 4;
    s.frm = lb;
    for (uint32_t j = threadIdx.x; j < caps.CL; j += blockDim.x) s.lk[j].key = kNone;
    __syncthreads();  // the workgroup is one wave: lane 0 sees every lane's clear
    if (threadIdx.x != 0) return;

    FcThread t(g, visited, s, caps);
    const int maxl = prm.maxl, minl = prm.minl;
    const uint64_t st = starts[i];
    const uint64_t rm = g.mult[st];
    uint32_t plen = 0, depth = 0, nnodes = 0;
    int32_t ncyc = 0;
    int64_t counter = 0, steps = 0;
    uint32_t relaxed = 0;

    // FindCycleUtil (cycle_finder.cpp:231-243)
    {
        const int sl = t.lock_slot(st, maxl);
        if (sl >= 0) {
            s.lk[sl].val = 0;
            s.lk[sl].onpath = 1;
        }
        s.psl[plen] = sl;
    }
    s.path[plen++] = st;
    {
        const uint64_t oi = g.out_info[st];
        const bool vst = (g.valid[st >> 6] >> (st & 63)) & 1;
        s.frm[0] = vst ? t.build_frame(st, oi, rm, maxl, 0) : 0;
    }
    s.bl[0] = maxl;
    depth = 1;

    // FindCycle main loop (cycle_finder.cpp:147-212)
    while (depth > 0 && t.status == 0) {
        if (++steps > prm.step_cap) break;
        const uint32_t top = depth - 1;
        const uint32_t live = s.frm[top];
        // the live candidates, their lock values and out_info words: one round of loads
        uint64_t N[4], OI[4];
        int32_t SL[4], VAL[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            N[j] = 0;
            OI[j] = 0;
            SL[j] = 0;
            VAL[j] = 0;
            if ((live >> j) & 1) {
                N[j] = s.fr[4 * top + j];
                SL[j] = s.frs[4 * top + j];
                OI[j] = s.froi[4 * top + j];
                VAL[j] = s.lk[SL[j]].val;
            }
        }
        bool flag = true, pushed = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (!((live >> j) & 1)) continue;
            const uint64_t x = N[j];
            if (x == st) {
                s.bl[top] = 1;
                if ((int)plen > minl) {
                    if (nnodes + plen > caps.CO || ncyc >= (int)caps.CC) { t.status = 3; break; }
                    for (uint32_t q = 0; q < plen; ++q) s.out[nnodes + q] = s.path[q];
                    nnodes += plen;
                    s.olen[ncyc++] = (uint16_t)plen;
                    counter += 1;
                    if (counter >= prm.cluster) { ncyc = 0; nnodes = 0; flag = false; }
                }
            } else if ((int)plen < VAL[j]) {
                // erase x from the top frame (the rest keep their order) and push it
                const int sl = SL[j];
                s.frm[top] = (uint8_t)(live & ~(1u << j));
                s.psl[plen] = sl;
                s.path[plen++] = x;
                s.bl[depth] = maxl;
                s.lk[sl].val = (int)plen;
                s.lk[sl].onpath = 1;
                s.frm[depth] = t.build_frame(x, OI[j], rm, maxl, depth);
                ++depth;
                flag = false;
                pushed = true;
                break;
            }
        }
        if (t.status) break;
        if (flag) {
            --depth;
            const uint64_t v = s.path[--plen];
            const int vsl = s.psl[plen];
            if (vsl >= 0) s.lk[vsl].onpath = 0;
            const int b = s.bl[depth];
            if (depth > 0) s.bl[depth - 1] = min(s.bl[depth - 1], b);
            if (b < maxl) {
                // lock relaxation (cycle_finder.cpp:191-209); its fixpoint does not depend on
                // the processing order, so a plain stack is used.
                const uint64_t vii = g.in_info[v];
                const bool vv = (g.valid[v >> 6] >> (v & 63)) & 1;
                uint32_t rs = 0;
                {
                    RelaxRec r0;
                    r0.ub = (v << 16) | (uint64_t)b;
                    r0.ii = vv ? vii : 0;  // an invalid node has no predecessors to visit
                    r0.slot = vsl;
                    r0.pad = 0;
                    s.relax[rs++] = r0;
                }
                while (rs > 0 && t.status == 0) {
                    const RelaxRec e = s.relax[--rs];
                    const int blv = (int)(e.ub & 0xFFFF);
                    const uint64_t u = e.ub >> 16;
                    const int sl = e.slot;
                    if (sl < 0) break;
                    if (s.lk[sl].val < maxl - blv + 1) {
                        s.lk[sl].val = maxl - blv + 1;
                        ++relaxed;
                        uint64_t ins[4], iii[4];
                        int32_t isl[4];
                        const int ni = t.preds_of(u, e.ii, rm, ins, isl, iii, maxl);
                        for (int j = 0; j < ni; ++j) {
                            // std::find(path, ins[j]): the path flag of its lock record
                            if (s.lk[isl[j]].onpath) continue;
                            if (rs >= caps.CR) { t.status = 2; break; }
                            RelaxRec r;
                            r.ub = (ins[j] << 16) | (uint64_t)(blv + 1);
                            r.ii = iii[j];
                            r.slot = isl[j];
                            r.pad = 0;
                            s.relax[rs++] = r;
                        }
                    }
                }
            }
        } else if (!pushed) {
            // the cluster bound cleared the cycles and nothing was pushed: the state is a
            // fixed point, the reference spins until the step cap and returns {}.
            ncyc = 0;
            nnodes = 0;
            break;
        }
    }
    FcStatus o;
    o.status = t.status;
    o.ncyc = ncyc;
    o.nnodes = nnodes;
    o.steps = (uint32_t)(steps < 0xFFFFFFFFLL ? steps : 0xFFFFFFFFLL);
    o.relax = relaxed;
    o.locks = t.lsize;
    stat[i] = o;
}

// gather thread outputs into one contiguous buffer
__global__ void k_fc_gather(const uint64_t *sbase, uint64_t per_al, FcCaps caps, const uint64_t *sel,
                            const uint64_t *node_off, const uint64_t *cyc_off, uint64_t *nodes, uint16_t *lens,
                            uint64_t nsel) {
    const uint64_t q = blockIdx.x;
    if (q >= nsel) return;
    const uint64_t i = sel[q];
    const uint8_t *base = (const uint8_t *)sbase + i * per_al;
    const uint64_t *out = (const uint64_t *)(base + fc_out_offset(caps));
    const uint16_t *olen = (const uint16_t *)(base + fc_out_offset(caps) + (uint64_t)caps.CO * 8);
    const uint64_t nn = node_off[q + 1] - node_off[q];
    const uint64_t nc = cyc_off[q + 1] - cyc_off[q];
    for (uint64_t j = threadIdx.x; j < nn; j += blockDim.x) nodes[node_off[q] + j] = out[j];
    for (uint64_t j = threadIdx.x; j < nc; j += blockDim.x) lens[cyc_off[q] + j] = olen[j];
}

// conflict[q] = 1 if a node first visited by a tentative commit c < jlist[q] is in the
// footprint (lock table) of speculative start jlist[q]
// (jslot[q]: the scratch slot of that start on this rank)
__global__ void k_fc_conflict(const uint64_t *sbase, uint64_t per_al, uint32_t CL, const uint64_t *newly,
                              const uint32_t *newly_c, uint64_t n_newly, const uint32_t *jlist,
                              const uint32_t *jslot, uint64_t nj, int *conflict) {
    const uint64_t tot = n_newly * nj;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < tot; idx += stride) {
        const uint64_t a = idx / nj, q = idx - a * nj;
        const uint32_t j = jlist[q];
        if (j <= newly_c[a] || conflict[q]) continue;
        const LockRec *lk = (const LockRec *)((const uint8_t *)sbase + (uint64_t)jslot[q] * per_al);
        const uint64_t x = newly[a];
        for (uint32_t h = (uint32_t)(mix64(x) & (CL - 1));; h = (h + 1) & (CL - 1)) {
            const uint64_t k = lk[h].key;
            if (k == x) { conflict[q] = 1; break; }
            if (k == kNone) break;
        }
    }
}

// ---- FindCycle commit on the device (FcRunner::commit_round) ----
// open-addressing tables keyed by node id (kNone = empty slot), power-of-two capacity
__device__ __forceinline__ uint32_t node_slot(uint64_t x, uint32_t cap) { return (uint32_t)(mix64(x) & (cap - 1)); }

// the round's start nodes (start j -> j) and whether each was visited before the round
__global__ void k_fc_starts(const uint64_t *starts, uint32_t n, uint64_t *skeys, uint32_t *svals, uint32_t cap,
                            const uint64_t *vis, uint8_t *pre_vis) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t x = starts[i];
    pre_vis[i] = bit_get(vis, x) ? 1 : 0;
    for (uint32_t h = node_slot(x, cap);; h = (h + 1) & (cap - 1)) {
        const unsigned long long prev = atomicCAS((unsigned long long *)&skeys[h], kNone, (unsigned long long)x);
        if (prev == kNone || prev == x) {
            svals[h] = i;  // start nodes are distinct
            return;
        }
    }
}

// (j', j) for every start node s_j that an output of an earlier start j' passes through
__global__ void k_fc_pairs(const uint64_t *nodes, const uint32_t *nodej, uint64_t n, const uint64_t *skeys,
                           const uint32_t *svals, uint32_t cap, uint64_t *pairs, unsigned long long *np) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t a = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; a < n; a += stride) {
        const uint64_t x = nodes[a];
        for (uint32_t h = node_slot(x, cap);; h = (h + 1) & (cap - 1)) {
            const uint64_t k = skeys[h];
            if (k == kNone) break;
            if (k == x) {
                if (svals[h] > nodej[a]) pairs[atomicAdd(np, 1ull)] = ((uint64_t)nodej[a] << 32) | svals[h];
                break;
            }
        }
    }
}

// (round 6) a pair (i << 32 | j) as the sort key (j << b | i): by the start reached, then by the
// start whose cycles reach it (b bits hold any start index of the round)
__global__ void k_fc_pair_keys(const uint64_t *pairs, uint64_t n, int b, uint64_t *keys) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t a = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; a < n; a += stride)
        keys[a] = ((pairs[a] & 0xFFFFFFFFull) << b) | (pairs[a] >> 32);
}
// segments of a device list into one compact list (one block per segment; seg = {from, count, to})
__global__ void k_fc_segs(const uint64_t *src, const uint64_t *seg, uint64_t *dst) {
    const uint64_t *sg = seg + 3 * (uint64_t)blockIdx.x;
    const uint64_t from = sg[0], n = sg[1], to = sg[2];
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) dst[to + i] = src[from + i];
}

// first[x] = the smallest committing start whose cycles pass through x, for x not yet visited
__global__ void k_fc_first(const uint64_t *nodes, const uint32_t *nodej, uint64_t n, const uint8_t *active,
                           const uint64_t *vis, uint64_t *hkeys, uint32_t *hvals, uint32_t cap) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t a = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; a < n; a += stride) {
        const uint32_t j = nodej[a];
        const uint64_t x = nodes[a];
        if (!active[j] || bit_get(vis, x)) continue;
        for (uint32_t h = node_slot(x, cap);; h = (h + 1) & (cap - 1)) {
            const unsigned long long prev = atomicCAS((unsigned long long *)&hkeys[h], kNone, (unsigned long long)x);
            if (prev == kNone || prev == x) {
                atomicMin(&hvals[h], j);
                break;
            }
        }
    }
}

// one wave per start j of jl: j conflicts when its footprint (lock table) holds a node that an
// earlier start of the round visits first; *first = the smallest conflicting j
__global__ void k_fc_conf(const uint8_t *sbase, uint64_t per_al, uint32_t CL, const uint32_t *jl, const uint32_t *js,
                          uint32_t nj, const uint64_t *hkeys, const uint32_t *hvals, uint32_t cap, unsigned int *first) {
    const uint32_t q = blockIdx.x;
    if (q >= nj) return;
    const uint32_t j = jl[q];
    if (__hip_atomic_load(first, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= j) return;
    const LockRec *lk = (const LockRec *)(sbase + (uint64_t)js[q] * per_al);
    for (uint32_t t = threadIdx.x; t < CL; t += blockDim.x) {
        const uint64_t x = lk[t].key;
        if (x == kNone) continue;
        for (uint32_t h = node_slot(x, cap);; h = (h + 1) & (cap - 1)) {
            const uint64_t k = hkeys[h];
            if (k == kNone) break;
            if (k == x) {
                if (hvals[h] < j) atomicMin(first, j);
                break;
            }
        }
    }
}

// dj[noff[q] .. noff[q+1]) = sel[q] (the start owning each gathered node; one GPU: slot = start)
__global__ void k_fc_owner(const uint64_t *sel, const uint64_t *noff, uint32_t *dj, uint64_t nsel) {
    const uint64_t q = blockIdx.x;
    if (q >= nsel) return;
    for (uint64_t a = noff[q] + threadIdx.x; a < noff[q + 1]; a += blockDim.x) dj[a] = (uint32_t)sel[q];
}

// visited |= every node first visited by a start before the commit point f
__global__ void k_fc_mark(const uint64_t *hkeys, const uint32_t *hvals, uint32_t cap, uint32_t f, uint64_t *vis) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= cap) return;
    const uint64_t x = hkeys[h];
    if (x != kNone && hvals[h] < f) atomicOr((unsigned long long *)&vis[x >> 6], 1ull << (x & 63));
}

__global__ void k_get_bits(const uint64_t *bm, const uint64_t *ids, uint64_t n, uint8_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = bit_get(bm, ids[i]) ? 1 : 0;
}

__global__ void k_set_bits(uint64_t *bm, const uint64_t *ids, uint64_t n, int value) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t x = ids[i];
        if (value) atomicOr((unsigned long long *)&bm[x >> 6], 1ull << (x & 63));
        else atomicAnd((unsigned long long *)&bm[x >> 6], ~(1ull << (x & 63)));
    }
}

__global__ void k_gather_mult(const uint16_t *mult, const uint64_t *ids, uint64_t n, uint16_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = mult[ids[i]];
}

__global__ void k_neighbors(GraphView g, const uint64_t *ids, uint64_t n, int incoming, uint64_t *out,
                            int32_t *counts) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t t[4] = {kNone, kNone, kNone, kNone};
    const int c = incoming ? dev_incoming(g, ids[i], t) : dev_outgoing(g, ids[i], t);
    for (int j = 0; j < 4; ++j) out[4 * i + j] = t[j];
    counts[i] = c;
}

__global__ void k_unpack_bits(const uint64_t *bm, uint64_t D, uint8_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < D; e += stride) out[e] = bit_get(bm, e);
}

unsigned long long read_counter(mcaat_ctx *ctx, unsigned long long *d) {
    unsigned long long h = 0;
    HIP_OK(hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    return h;
}

// ids i in [0, n) with flags[i] != 0, in ascending order; returns the count
uint64_t select_flagged(mcaat_ctx *ctx, const uint8_t *flags, uint64_t n, uint64_t *out, unsigned long long *d_num) {
    hipcub::CountingInputIterator<uint64_t> it(0);
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceSelect::Flagged(nullptr, tmp, it, flags, out, d_num, (size_t)n, ctx->stream));
    DevBuf<uint8_t> t(tmp);
    HIP_OK(hipcub::DeviceSelect::Flagged(t.p, tmp, it, flags, out, d_num, (size_t)n, ctx->stream));
    return read_counter(ctx, d_num);
}



}  // namespace

// ------------------------------ peel driver -----------------------------------
// the peel's per-edge arrays; with `ready` set, k_tips_filter has already filled nf and nxk
// (round 4) with post / wpre the arrays hold `slots` compact slots, one per edge valid after the
// filter (PeelArrays::cidx); otherwise one per edge
struct PeelState {
    DevBuf<uint8_t> nf;
    DevBuf<uint64_t> nxk;
    bool ready = false;
    const uint64_t *post = nullptr;
    const uint32_t *wpre = nullptr;
    uint64_t slots = 0;
};

static void run_peel_rulers(mcaat_graph *g, const uint64_t *seed_bm, PeelState *pre = nullptr) {
    mcaat_ctx *ctx = g->ctx;
    hipStream_t st = ctx->stream;
    const uint64_t D = g->D;
    if (!D) return;
    GraphView v = g->view();
    PeelState local;
    PeelState &ps = pre ? *pre : local;
    if (!ps.wpre) ps.slots = D;
    const uint64_t S = std::max<uint64_t>(ps.slots, 1);
    DevBuf<uint32_t> owner(S);
    if (!ps.ready) {
        ps.nf.alloc(4 * S);
        ps.nxk.alloc(S);
        HIP_OK(hipMemsetAsync(ps.nf.p, 0, ps.nf.bytes(), st));  // the flag bytes other nodes set
    }
    // identity slots: the graph's filtered bitmap tells prep which edges are valid
    PeelArrays pa{ps.nf.p, ps.nxk.p, owner.p, nullptr, nullptr, seed_bm,
                  ps.wpre ? ps.post : (const uint64_t *)g->valid.p, ps.wpre, g->n_words()};
    if (!ps.ready) {
        hipLaunchKernelGGL(k_peel_init, dim3(grid_for(D, kBlock)), dim3(kBlock), 0, st, v, pa);
        LAUNCH_OK();
    }
    // 1 in (ruler_mask + 1) unary nodes is a ruler besides the chain heads: a walk costs one
    // random read per node whatever the spacing; the rulers are then ranked one level up
    // (1 in 64 of them, plus the heads, are super rulers) before pointer jumping
    const uint64_t ruler_mask = (uint64_t)std::max<int64_t>(0, knob(ctx, "cf.ruler_mask", 63));
    // the ruler and branch lists start at a fraction of D (rulers: the chain heads plus 1 in 64
    // unary nodes; branch nodes are rarer still) and the pass runs again if either overflowed
    const int64_t div = std::max<int64_t>(1, knob(ctx, "cf.peel_list_div", 16));
    uint64_t cap = std::min<uint64_t>(S, S / (uint64_t)div + (1u << 16)), bcap = std::min<uint64_t>(S, S / 64 + (1u << 16));
    if (knob_set(ctx, "cf.peel_list_cap"))  // test knob: both lists start this small
        cap = bcap = (uint64_t)std::max<int64_t>(1, knob(ctx, "cf.peel_list_cap", 1));
    DevBuf<unsigned long long> cur(4);
    DevBuf<uint64_t> list, blist;
    uint64_t nr = 0, nb = 0;
    for (;;) {
        list.alloc(cap);
        blist.alloc(bcap);
        HIP_OK(hipMemsetAsync(cur.p, 0, cur.bytes(), st));
        const int64_t pb = knob(ctx, "cf.prep_batch", 2);  // edges per thread in flight: C3 2 / 4 / 8 / 16 -> peel 22.8 / 23.3 / 24.3 / 26.0 ms
        auto prep = pb == 4 ? k_peel_prep<4> : pb == 8 ? k_peel_prep<8> : pb == 16 ? k_peel_prep<16> : k_peel_prep<2>;
        hipLaunchKernelGGL(prep, dim3(grid_for(D, kBlock * kTileJ)), dim3(kBlock), 0, st, D, pa, ruler_mask, list.p,
                           cap, cur.p, blist.p, bcap, cur.p + 1);
        LAUNCH_OK();
        unsigned long long hc[2];
        HIP_OK(hipMemcpyAsync(hc, cur.p, 16, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        nr = hc[0];
        nb = hc[1];
        if (nr <= cap && nb <= bcap) break;
        cap = std::max<uint64_t>(cap, nr);
        bcap = std::max<uint64_t>(bcap, nb);
    }
    if (nr >= kNoOwner) throw Error(MCAAT_E_CAPACITY, "peel: 2^32 or more rulers");
    DevBuf<uint64_t> jump(nr ? nr : 1);
    DevBuf<uint32_t> sowner(nr ? nr : 1);
    pa.jump = jump.p;
    pa.sowner = sowner.p;
    if (nr) {
        hipLaunchKernelGGL(k_peel_walk, dim3(grid_for(nr, kBlock)), dim3(kBlock), 0, st, pa, list.p, nr);
        LAUNCH_OK();
        HIP_OK(hipMemsetAsync(sowner.p, 0xFF, 4 * nr, st));
        DevBuf<uint32_t> slist(nr);
        hipLaunchKernelGGL(k_peel_super, dim3(grid_for(nr, kBlock)), dim3(kBlock), 0, st, pa, list.p, nr, slist.p,
                           cur.p + 2);
        LAUNCH_OK();
        const uint64_t ns = read_counter(ctx, cur.p + 2);
        int rounds = 2;
        while ((1ULL << rounds) < ns + 1) ++rounds;
        rounds += 1;
        // log2(ns)+1 rounds bound the chain depth; most inputs converge far earlier, which
        // a round without changes proves (checked from the fourth round on)
        DevBuf<int> chg(1);
        int hchg = 1;
        for (int r = 0; ns && r < rounds; ++r) {
            if (r >= 4) HIP_OK(hipMemsetAsync(chg.p, 0, 4, st));
            hipLaunchKernelGGL(k_peel_jump, dim3(grid_for(ns, kBlock)), dim3(kBlock), 0, st, pa, slist.p, ns, chg.p);
            LAUNCH_OK();
            if (r >= 4) {
                HIP_OK(hipMemcpyAsync(&hchg, chg.p, 4, hipMemcpyDeviceToHost, st));
                HIP_OK(hipStreamSynchronize(st));
                if (!hchg) break;
            }
        }
        hipLaunchKernelGGL(k_peel_final, dim3(grid_for(nr, kBlock)), dim3(kBlock), 0, st, pa, nr);
        LAUNCH_OK();
    }
    DevBuf<int> changed(1);
    for (uint64_t it = 0; nb && it < D + 1; ++it) {
        HIP_OK(hipMemsetAsync(changed.p, 0, 4, st));
        hipLaunchKernelGGL(k_peel_branch, dim3(grid_for(nb, kBlock)), dim3(kBlock), 0, st, v, pa, blist.p, nb,
                           changed.p);
        LAUNCH_OK();
        int h = 0;
        HIP_OK(hipMemcpyAsync(&h, changed.p, 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        if (!h) break;
    }
    // resolution reads valid bits (dev_outgoing), so removal waits until it is complete
    if (nb) {
        hipLaunchKernelGGL(k_peel_apply_list, dim3(grid_for(nb, kBlock)), dim3(kBlock), 0, st, v, pa, blist.p, nb);
        LAUNCH_OK();
    }
    if (nr) {
        hipLaunchKernelGGL(k_peel_apply_rulers, dim3(grid_for(nr, kBlock)), dim3(kBlock), 0, st, v, pa, list.p, nr);
        LAUNCH_OK();
    }
    HIP_OK(hipStreamSynchronize(st));
}

// RecursiveReduction from every seed: counter-driven walks (work proportional to what is
// removed) with a per-thread step budget; if chains are longer than that, the pending
// frontier seeds the parallel ruler/list-ranking peel, whose fixpoint from this state is
// the same (every pending node is valid, has no valid successor and must be removed).
static void run_peel(mcaat_graph *g, const uint64_t *seed_bm, PeelState *pre = nullptr) {
    mcaat_ctx *ctx = g->ctx;
    // C3: the reduction walks chains of tens of thousands of edges back from a few hundred
    // seeds (budget 512: 164 walks still pending; 32768: 12, at 0.5 s), so by default the
    // list-ranking peel runs alone from the seeds (the same fixpoint); cf.walk_budget > 0 runs
    // counter-driven walks with that step budget first
    const int64_t walk_budget = knob(ctx, "cf.walk_budget", 0);
    if (walk_budget <= 0) {
        run_peel_rulers(g, seed_bm, pre);
        return;
    }
    const uint32_t kBudget = (uint32_t)std::min<int64_t>(walk_budget, 0xFFFFFFFFLL);
    hipStream_t st = ctx->stream;
    const uint64_t D = g->D, nw = g->n_words();
    if (!D) return;
    GraphView v = g->view();
    DevBuf<unsigned long long> cur(2);
    DevBuf<uint32_t> rem(D);
    DevBuf<uint64_t> fa(D), fb(D), pend(D);
    HIP_OK(hipMemsetAsync(cur.p, 0, 16, st));
    hipLaunchKernelGGL(k_kahn_init, dim3(grid_for(nw * 64, kBlock)), dim3(kBlock), 0, st, v, seed_bm, rem.p, fa.p,
                       cur.p);
    LAUNCH_OK();
    uint64_t n = read_counter(ctx, cur.p);
    static const bool verbose = getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1';
    while (n) {
        if (verbose) fprintf(stderr, "[mcaat] peel: kahn frontier %llu\n", (unsigned long long)n);
        HIP_OK(hipMemsetAsync(cur.p, 0, 8, st));
        hipLaunchKernelGGL(k_kahn_walk, dim3(grid_for(n, 64)), dim3(64), 0, st, v, rem.p, fa.p, n, fb.p, cur.p,
                           kBudget, pend.p, cur.p + 1);
        LAUNCH_OK();
        n = read_counter(ctx, cur.p);
        std::swap(fa, fb);
    }
    const uint64_t np = read_counter(ctx, cur.p + 1);
    if (verbose) fprintf(stderr, "[mcaat] peel: pending after kahn walks %llu\n", (unsigned long long)np);
    if (np) {
        DevBuf<uint64_t> bm(nw);
        HIP_OK(hipMemsetAsync(bm.p, 0, bm.bytes(), st));
        hipLaunchKernelGGL(k_ids_to_bits, dim3(grid_for(np, kBlock)), dim3(kBlock), 0, st, pend.p, np, bm.p);
        LAUNCH_OK();
        run_peel_rulers(g, bm.p);
    }
    HIP_OK(hipStreamSynchronize(st));
}

// ---------------------------- DLS driver -------------------------------------
static std::vector<uint64_t> run_dls(mcaat_graph *g, const std::vector<uint64_t> &cand, int limit) {
    mcaat_ctx *ctx = g->ctx;
    hipStream_t st = ctx->stream;
    std::vector<int8_t> res(cand.size(), -1);
    std::vector<uint64_t> todo(cand.size());
    for (size_t i = 0; i < cand.size(); ++i) todo[i] = i;
    // first-try scratch per candidate (stack + visited set, 8 B entries; overflows re-run x8):
    // 24 KB while every candidate fits one 8-GB launch, else 8x less (C5: 3.8M candidates, most
    // of them short searches, in one launch instead of eleven)
    const bool many = cand.size() * 8ULL * (1024 + 2048) > (8ULL << 30);
    uint32_t cs = (uint32_t)std::max<int64_t>(1, knob(ctx, "cf.dls_stack", many ? 128 : 1024));
    uint32_t cv = (uint32_t)next_pow2((uint64_t)std::max<int64_t>(2, knob(ctx, "cf.dls_visited", many ? 256 : 2048)));
    while (!todo.empty()) {
        // scratch for every candidate at once (C3: 65K candidates x 24 KB = 1.6 GB): one launch,
        // whose time is its longest search (512 MB batches made C3 three launches, 6.6 ms)
        const uint64_t batch_cap = std::max<uint64_t>(64, (8ULL << 30) / (8ULL * (cs + cv)));
        std::vector<uint64_t> next;
        for (size_t b0 = 0; b0 < todo.size(); b0 += batch_cap) {
            const uint64_t n = std::min<uint64_t>(batch_cap, todo.size() - b0);
            std::vector<uint64_t> ids(n);
            for (uint64_t j = 0; j < n; ++j) ids[j] = cand[todo[b0 + j]];
            DevBuf<uint64_t> dids(n), dstk(n * cs), dvis(n * cv);
            DevBuf<int8_t> dres(n);
            h2d(g->ctx, dids.p, ids.data(), 8 * n);
            // searches per wave: a wave runs as long as its longest search, but more searches
            // per wave keep more loads in flight (C5, 3.8M candidates: 4 / 16 / 64 lanes ->
            // DLS 91 / 60 / 69 ms; C3 2.7-3.0 ms for any)
            const int lanes = (int)std::max<int64_t>(1, std::min<int64_t>(64, knob(ctx, "cf.dls_lanes", 16)));
            hipLaunchKernelGGL(k_dls, dim3(grid_for(n, (unsigned)lanes)), dim3(64), 0, st, g->view(), dids.p, n, limit,
                               dstk.p, cs, dvis.p, cv, dres.p, lanes);
            LAUNCH_OK();
            std::vector<int8_t> h(n);
            HIP_OK(hipMemcpyAsync(h.data(), dres.p, n, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            static const bool verbose = getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1';
            if (verbose) {
                uint64_t over = 0, found = 0;
                for (int8_t x : h) over += x < 0, found += x > 0;
                fprintf(stderr, "[mcaat] dls: batch of %llu (stack %u, visited %u): found %llu, overflow %llu\n",
                        (unsigned long long)n, cs, cv, (unsigned long long)found, (unsigned long long)over);
            }
            for (uint64_t j = 0; j < n; ++j) {
                if (h[j] < 0) next.push_back(todo[b0 + j]);
                else res[todo[b0 + j]] = h[j];
            }
        }
        todo.swap(next);
        if (!todo.empty()) {
            if (cs >= (1u << 26)) throw Error(MCAAT_E_CAPACITY, "DepthLevelSearch scratch exceeded 2^26 entries");
            cs *= 8;
            cv *= 8;
        }
    }
    std::vector<uint64_t> pass;
    for (size_t i = 0; i < cand.size(); ++i)
        if (res[i] == 1) pass.push_back(cand[i]);
    return pass;
}

__global__ void __launch_bounds__(kBlock) k_iota(uint64_t *x, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = i;
}
__global__ void __launch_bounds__(kBlock) k_gather_ids(const uint64_t *cand, const uint64_t *idx, uint64_t n, uint64_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = cand[idx[i]];
}
__global__ void __launch_bounds__(kBlock) k_scatter_res(const int8_t *r, const uint64_t *idx, uint64_t n, int8_t *res,
                                                        uint8_t *ovf) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        res[idx[i]] = r[i];
        ovf[i] = r[i] < 0;
    }
}
__global__ void __launch_bounds__(kBlock) k_res_pass(const int8_t *res, uint64_t n, uint8_t *f) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) f[i] = res[i] == 1;
}

template <class T>
static uint64_t select_dev(mcaat_ctx *ctx, const T *in, const uint8_t *flags, uint64_t n, T *out) {
    hipStream_t st = ctx->stream;
    DevBuf<unsigned long long> num(1);
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceSelect::Flagged(nullptr, tmp, in, flags, out, num.p, (size_t)n, st));
    DevBuf<uint8_t> t(tmp);
    HIP_OK(hipcub::DeviceSelect::Flagged(t.p, tmp, in, flags, out, num.p, (size_t)n, st));
    return read_counter(ctx, num.p);
}

// DepthLevelSearch over candidates already on the device (ascending ids; one GPU): the same
// searches, batches and x8 scratch regrowth as run_dls, with the overflowed candidates and the
// passing ids selected on the device, so only the passing ids cross to the host (C5: 3.8M
// candidate ids went to the host and back, and their results were looped over there)
static std::vector<uint64_t> run_dls_dev(mcaat_graph *g, const uint64_t *dcand, uint64_t n, int limit) {
    mcaat_ctx *ctx = g->ctx;
    hipStream_t st = ctx->stream;
    std::vector<uint64_t> pass;
    if (!n) return pass;
    // (round 4) cf.dls_persist=1: per-lane scratch, candidates strided over the lanes; 0 (default):
    // one scratch slot per candidate in batches
    // measured: C3 2.6 ms either way, C5 49.0 ms against 42.4 for the batches (a persistent
    // wave runs its lanes' candidate sequences to the longest sum, and finished waves leave their
    // CU idle): off by default
    const bool persist = knob(ctx, "cf.dls_persist", 0) != 0;
    // scratch budget of one launch (knob cf.dls_budget, GB)
    const uint64_t budget = (uint64_t)std::max<int64_t>(1, knob(ctx, "cf.dls_budget", 8)) << 30;
    const bool many = !persist && n * 8ULL * (1024 + 2048) > budget;
    uint32_t cs = (uint32_t)std::max<int64_t>(1, knob(ctx, "cf.dls_stack", many ? 128 : 1024));
    uint32_t cv = (uint32_t)next_pow2((uint64_t)std::max<int64_t>(2, knob(ctx, "cf.dls_visited", many ? 256 : 2048)));
    const int lanes = (int)std::max<int64_t>(1, std::min<int64_t>(64, knob(ctx, "cf.dls_lanes", 16)));
    DevBuf<int8_t> res(n);
    DevBuf<uint64_t> idx(n), idx2(n), ids(n);
    DevBuf<uint8_t> flags(n);
    hipLaunchKernelGGL(k_iota, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, idx.p, n);
    LAUNCH_OK();
    uint64_t nt = n;
    bool first = true;
    // (round 5) first pass in LDS (cf.dls_lds, default 1, graphs below 2^32 - 1 edges); what
    // overflows its tables continues below with global scratch at 8x the first caps
    if (!persist && knob(ctx, "cf.dls_lds", 1) != 0 && g->D < 0xFFFFFFFFull && limit < 255) {
        DevBuf<int8_t> r(n);
        // cf.dls_lds_cap (tests): fewer visited / stack entries, so searches overflow to the re-run
        const uint32_t lc = (uint32_t)std::max<int64_t>(1, knob(ctx, "cf.dls_lds_cap", kLdsVis));
        hipLaunchKernelGGL(k_dls_lds, dim3((unsigned)((n + kLdsLanes - 1) / kLdsLanes)), dim3(64), 0, st, g->view(), dcand,
                           n, limit, r.p, std::min<uint32_t>(lc, kLdsVis / 4 * 3), std::min<uint32_t>(lc, kLdsStk));
        LAUNCH_OK();
        hipLaunchKernelGGL(k_scatter_res, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, (const int8_t *)r.p,
                           (const uint64_t *)idx.p, n, res.p, flags.p);
        LAUNCH_OK();
        nt = select_dev(ctx, (const uint64_t *)idx.p, flags.p, n, idx2.p);
        std::swap(idx, idx2);
        first = false;
        cs = std::max<uint32_t>(cs, 8 * kLdsStk);
        cv = std::max<uint32_t>(cv, 8 * kLdsVis);
        verbose_mark(ctx, "dls.lds_pass");
    }
    for (; nt; first = false) {
        const uint64_t batch_cap = std::max<uint64_t>(64, budget / (8ULL * (cs + cv)));
        const uint64_t *src = dcand;
        if (!first) {  // the candidates to search again, in candidate order
            hipLaunchKernelGGL(k_gather_ids, dim3(grid_for(nt, kBlock)), dim3(kBlock), 0, st, dcand,
                               (const uint64_t *)idx.p, nt, ids.p);
            LAUNCH_OK();
            src = ids.p;
        }
        DevBuf<int8_t> r(nt);
        if (persist) {
            // scratch per lane: as many lanes as the GPU holds at once (or fewer candidates),
            // within the same 8-GB scratch budget
            const uint64_t nl = std::max<uint64_t>(
                1, std::min<uint64_t>({nt, (uint64_t)ctx->n_cu * 32 * (uint64_t)lanes, batch_cap}));
            DevBuf<uint64_t> dstk(nl * cs), dvis(nl * cv);
            HIP_OK(hipMemsetAsync(dvis.p, 0, dvis.bytes(), st));
            hipLaunchKernelGGL(k_dls_lanes, dim3(grid_for(nl, (unsigned)lanes)), dim3(64), 0, st, g->view(), src, nt,
                               limit, dstk.p, cs, dvis.p, cv, r.p, lanes, nl);
            LAUNCH_OK();
            HIP_OK(hipStreamSynchronize(st));  // the scratch is freed on scope exit
        } else {
            for (uint64_t b0 = 0; b0 < nt; b0 += batch_cap) {
                const uint64_t m = std::min<uint64_t>(batch_cap, nt - b0);
                DevBuf<uint64_t> dstk(m * cs), dvis(m * cv);
                hipLaunchKernelGGL(k_dls, dim3(grid_for(m, (unsigned)lanes)), dim3(64), 0, st, g->view(), src + b0, m,
                                   limit, dstk.p, cs, dvis.p, cv, r.p + b0, lanes);
                LAUNCH_OK();
                HIP_OK(hipStreamSynchronize(st));  // the batch's scratch is freed on scope exit
            }
        }
        hipLaunchKernelGGL(k_scatter_res, dim3(grid_for(nt, kBlock)), dim3(kBlock), 0, st, (const int8_t *)r.p,
                           (const uint64_t *)idx.p, nt, res.p, flags.p);
        LAUNCH_OK();
        const uint64_t again = select_dev(ctx, (const uint64_t *)idx.p, flags.p, nt, idx2.p);
        std::swap(idx, idx2);
        nt = again;
        if (nt) {
            if (cs >= (1u << 26)) throw Error(MCAAT_E_CAPACITY, "DepthLevelSearch scratch exceeded 2^26 entries");
            cs *= 8;
            cv *= 8;
        }
    }
    verbose_mark(ctx, "dls.reruns");
    hipLaunchKernelGGL(k_res_pass, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, (const int8_t *)res.p, n, flags.p);
    LAUNCH_OK();
    const uint64_t np = select_dev(ctx, dcand, flags.p, n, ids.p);
    pass.resize(np);
    if (np) d2h(ctx, pass.data(), ids.p, 8 * np);
    return pass;
}

// ---------------------------- FindCycle driver -----------------------------------
struct FcRunner {
    mcaat_graph *g;
    Comm *comm;  // null: one GPU
    int N = 1, R = 0;
    FcParams prm;
    FcCaps caps;
    DevBuf<uint64_t> dvis;
    mcaat_cycles *out;
    uint64_t rounds = 0, reruns = 0;

    FcRunner(mcaat_graph *gr, const mcaat_cf_params &p, mcaat_cycles *o, Comm *cm)
        : g(gr), comm(cm), out(o) {
        if (comm) {
            N = comm->world;
            R = comm->rank;
        }
        prm.maxl = p.cycle_max_length;
        prm.minl = p.cycle_min_length;
        prm.cluster = p.cluster_bound;
        prm.step_cap = p.step_cap;
        caps.P = (uint32_t)std::max(4, p.cycle_max_length + 2);
        const mcaat_ctx *ctx = gr->ctx;
        caps.CL = (uint32_t)next_pow2((uint64_t)std::max<int64_t>(4, knob(ctx, "cf.fc_lock", 4096)));
        caps.CR = (uint32_t)std::max<int64_t>(1, knob(ctx, "cf.fc_relax", 2048));
        caps.CC = (uint32_t)std::max(1, p.cluster_bound);
        caps.CO = (uint32_t)std::max<uint64_t>(caps.P, (uint64_t)caps.CC * (caps.P - 1));
        if (const int64_t co = knob(ctx, "cf.fc_out", 0)) caps.CO = (uint32_t)co;
        dvis.alloc(mcaat_graph::bitmap_words(gr->D));
        HIP_OK(hipMemsetAsync(dvis.p, 0, dvis.bytes(), gr->ctx->stream));
    }
    uint64_t per_al() const { return fc_per_search(caps); }

    // One speculative round's outputs as seen by every rank: the window's starts are dealt
    // round-robin (start j runs on rank j % N in its slot j / N), each rank runs its share
    // against the same visited snapshot, and the statuses and found cycles are all-gathered,
    // so every rank commits the same prefix in the same order (threads=1 semantics).
    struct RankOut {
        std::vector<FcStatus> st;
        std::vector<uint64_t> nodes;
        std::vector<uint16_t> lens;
    };

    // Commit of one round on the device, in the reference's threads=1 order:
    //  (1) start j is skipped when it was visited before the round or when the cycles of an
    //      earlier committed start pass through it (k_fc_pairs finds the pairs; resolved in
    //      order on the host, a few per round);
    //  (2) every node not yet visited gets the smallest committing start whose cycles contain
    //      it (k_fc_first: atomicMin in a table keyed by node);
    //  (3) start j (after the first committing one) conflicts when its footprint — its lock
    //      table holds every node whose visited bit it read — contains a node first visited by
    //      an earlier start of the round (k_fc_conf, on the rank that ran j);
    //  the prefix before the first conflict or overflow commits (k_fc_mark sets its visited
    //  bits) and the rest re-runs. Returns the commit point f; skip[j] for j < f.
    uint64_t commit_round(const std::vector<uint64_t> &pending, uint64_t W, uint64_t first_bad,
                          const std::vector<uint32_t> &selj, const std::vector<const uint64_t *> &jn,
                          const std::vector<const FcStatus *> &hs, uint64_t n_nodes, const uint8_t *scratch,
                          uint64_t pa, std::vector<uint8_t> &skip, const uint64_t *dev_nodes,
                          const uint32_t *dev_owner) {
        hipStream_t st = g->ctx->stream;
        skip.assign(W, 0);
        const uint32_t nb = (uint32_t)first_bad;
        if (nb == 0) return 0;
        const uint32_t scap = (uint32_t)next_pow2(2ULL * nb + 16);
        const uint32_t hcap = (uint32_t)next_pow2(2ULL * n_nodes + 16);
        DevBuf<uint64_t> dstarts(nb), skeys(scap), dnb, hkeys(hcap), dpairs(n_nodes + 1);
        DevBuf<uint32_t> svals(scap), djb, hvals(hcap);
        DevBuf<uint8_t> prev(nb), act(nb);
        DevBuf<unsigned long long> dnp(1);
        DevBuf<unsigned int> dfirst(1);
        HIP_OK(hipMemcpyAsync(dstarts.p, pending.data(), 8ULL * nb, hipMemcpyHostToDevice, st));
        HIP_OK(hipMemsetAsync(skeys.p, 0xFF, skeys.bytes(), st));
        HIP_OK(hipMemsetAsync(dnp.p, 0, 8, st));
        // node lists of the starts with cycles, in start order, and each node's start (one GPU:
        // already on the device from the gather; several: assembled from every rank's outputs)
        const uint64_t *dn = dev_nodes;
        const uint32_t *dj = dev_owner;
        if (n_nodes && (!dn || !dj)) {
            std::vector<uint64_t> hn(n_nodes);
            std::vector<uint32_t> hj(n_nodes);
            uint64_t a = 0;
            for (uint32_t j : selj) {
                const uint64_t nn = hs[j]->nnodes;
                std::copy(jn[j], jn[j] + nn, hn.begin() + a);
                std::fill(hj.begin() + a, hj.begin() + a + nn, j);
                a += nn;
            }
            dnb.alloc(n_nodes);
            djb.alloc(n_nodes);
            HIP_OK(hipMemcpyAsync(dnb.p, hn.data(), 8 * n_nodes, hipMemcpyHostToDevice, st));
            HIP_OK(hipMemcpyAsync(djb.p, hj.data(), 4 * n_nodes, hipMemcpyHostToDevice, st));
            dn = dnb.p;
            dj = djb.p;
            HIP_OK(hipStreamSynchronize(st));  // hn/hj go out of scope
        }
        hipLaunchKernelGGL(k_fc_starts, dim3(grid_for(nb, kBlock)), dim3(kBlock), 0, st, dstarts.p, nb, skeys.p,
                           svals.p, scap, dvis.p, prev.p);
        LAUNCH_OK();
        if (n_nodes) {
            hipLaunchKernelGGL(k_fc_pairs, dim3(grid_for(n_nodes, kBlock)), dim3(kBlock), 0, st, dn, dj, n_nodes,
                               skeys.p, svals.p, scap, dpairs.p, dnp.p);
            LAUNCH_OK();
        }
        std::vector<uint8_t> pv(nb);
        unsigned long long np = 0;
        HIP_OK(hipMemcpyAsync(pv.data(), prev.p, nb, hipMemcpyDeviceToHost, st));
        HIP_OK(hipMemcpyAsync(&np, dnp.p, 8, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        // (round 6) the pairs sorted and made unique on the device, as (j << pb | i): a start's
        // cycles pass through another start once per cycle and node, so the raw pairs repeat
        // (C5: 6.5 ms of copies and a host sort per round before)
        int pb = 1;
        while ((1ull << pb) < (uint64_t)nb) ++pb;
        std::vector<uint64_t> pairs;
        if (np) {
            DevBuf<uint64_t> k1(np), k2(np);
            DevBuf<unsigned long long> nu(1);
            hipLaunchKernelGGL(k_fc_pair_keys, dim3(grid_for(np, kBlock)), dim3(kBlock), 0, st, (const uint64_t *)dpairs.p,
                               (uint64_t)np, pb, k1.p);
            LAUNCH_OK();
            size_t t1 = 0, t2 = 0;
            HIP_OK(hipcub::DeviceRadixSort::SortKeys(nullptr, t1, k1.p, k2.p, (int)np, 0, 2 * pb, st));
            HIP_OK(hipcub::DeviceSelect::Unique(nullptr, t2, k2.p, k1.p, nu.p, (int)np, st));
            DevBuf<uint8_t> tmp(std::max<size_t>({t1, t2, 1}));
            HIP_OK(hipcub::DeviceRadixSort::SortKeys(tmp.p, t1, k1.p, k2.p, (int)np, 0, 2 * pb, st));
            HIP_OK(hipcub::DeviceSelect::Unique(tmp.p, t2, k2.p, k1.p, nu.p, (int)np, st));
            unsigned long long nuq = 0;
            d2h(g->ctx, &nuq, nu.p, 8);
            pairs.resize(nuq);
            if (nuq) d2h(g->ctx, pairs.data(), k1.p, 8 * nuq);
        }
        const uint64_t pmask = (1ull << pb) - 1;
        verbose_mark(g->ctx, "fc.commit_pairs");
        // (1) skips, in start order (pairs sorted by the start they reach)
        std::vector<uint8_t> active(nb, 0);
        for (uint32_t j = 0, q = 0; j < nb; ++j) {
            bool sk = pv[j] != 0;
            for (; q < pairs.size() && (pairs[q] >> pb) == j; ++q)
                if (!skip[pairs[q] & pmask]) sk = true;
            skip[j] = sk ? 1 : 0;
            active[j] = sk ? 0 : 1;
        }
        // (2) first visitor of each node
        HIP_OK(hipMemcpyAsync(act.p, active.data(), nb, hipMemcpyHostToDevice, st));
        HIP_OK(hipMemsetAsync(hkeys.p, 0xFF, hkeys.bytes(), st));
        HIP_OK(hipMemsetAsync(hvals.p, 0xFF, hvals.bytes(), st));
        if (n_nodes) {
            hipLaunchKernelGGL(k_fc_first, dim3(grid_for(n_nodes, kBlock)), dim3(kBlock), 0, st, dn, dj, n_nodes,
                               act.p, dvis.p, hkeys.p, hvals.p, hcap);
            LAUNCH_OK();
        }
        verbose_mark(g->ctx, "fc.commit_first");
        // (3) conflicts: only starts that commit after some other start can conflict
        uint64_t f = first_bad;
        std::vector<uint32_t> jm, js;
        bool seen_commit = false;
        for (uint32_t j = 0; j < nb; ++j) {
            if (skip[j]) continue;
            if (seen_commit && (int)(j % N) == R) {
                jm.push_back(j);
                js.push_back(j / N);
            }
            seen_commit = true;
        }
        uint64_t my_first = W;
        if (n_nodes && !jm.empty()) {
            DevBuf<uint32_t> djm(jm.size()), djs(js.size());
            const unsigned int none = 0xFFFFFFFFu;
            HIP_OK(hipMemcpyAsync(dfirst.p, &none, 4, hipMemcpyHostToDevice, st));
            HIP_OK(hipMemcpyAsync(djm.p, jm.data(), 4 * jm.size(), hipMemcpyHostToDevice, st));
            HIP_OK(hipMemcpyAsync(djs.p, js.data(), 4 * js.size(), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_fc_conf, dim3((unsigned)jm.size()), dim3(64), 0, st, scratch, pa, caps.CL, djm.p,
                               djs.p, (uint32_t)jm.size(), hkeys.p, hvals.p, hcap, dfirst.p);
            LAUNCH_OK();
            unsigned int h = none;
            HIP_OK(hipMemcpyAsync(&h, dfirst.p, 4, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            if (h != none) my_first = h;
        }
        verbose_mark(g->ctx, "fc.commit_conf");
        if (N > 1)
            for (uint64_t x : comm->allgather_one(my_first)) my_first = std::min(my_first, x);
        f = std::min(f, my_first);
        // commit [0, f): visited bits of the nodes its starts visit first
        if (n_nodes && f > 0) {
            hipLaunchKernelGGL(k_fc_mark, dim3(grid_for(hcap, kBlock)), dim3(kBlock), 0, st, hkeys.p, hvals.p, hcap,
                               (uint32_t)f, dvis.p);
            LAUNCH_OK();
        }
        HIP_OK(hipStreamSynchronize(st));
        return f;
    }

    void run_bucket(const std::vector<uint64_t> &bucket) {
        hipStream_t st = g->ctx->stream;
        std::vector<uint64_t> pending(bucket);
        uint64_t window = (uint64_t)std::max<int64_t>(1, knob(g->ctx, "cf.fc_window", 8192));
        if (N > 1) window *= (uint64_t)N;  // each rank keeps the single-GPU window of searches
        while (!pending.empty()) {
            // starts already visited are skipped by the reference (:476) -> no entry
            {
                DevBuf<uint64_t> ids(pending.size());
                DevBuf<uint8_t> bits(pending.size());
                std::vector<uint8_t> hb(pending.size());
                HIP_OK(hipMemcpyAsync(ids.p, pending.data(), 8 * pending.size(), hipMemcpyHostToDevice, st));
                hipLaunchKernelGGL(k_get_bits, dim3(grid_for(pending.size(), kBlock)), dim3(kBlock), 0, st, dvis.p, ids.p,
                                   (uint64_t)pending.size(), bits.p);
                LAUNCH_OK();
                HIP_OK(hipMemcpyAsync(hb.data(), bits.p, pending.size(), hipMemcpyDeviceToHost, st));
                HIP_OK(hipStreamSynchronize(st));
                std::vector<uint64_t> keep;
                keep.reserve(pending.size());
                for (size_t i = 0; i < pending.size(); ++i)
                    if (!hb[i]) keep.push_back(pending[i]);
                pending.swap(keep);
            }
            if (pending.empty()) break;
            ++rounds;
            const uint64_t W = std::min<uint64_t>(window, pending.size());
            const uint64_t Wl = W > (uint64_t)R ? (W - R + N - 1) / N : 0;  // this rank's starts
            const uint64_t pa = per_al();
            DevBuf<uint64_t> dst(Wl);
            DevBuf<uint8_t> scratch(Wl * pa);
            DevBuf<FcStatus> dstat(Wl);
            RankOut mine;
            mine.st.resize(Wl);
            if (Wl) {
                std::vector<uint64_t> ls(Wl);
                for (uint64_t i = 0; i < Wl; ++i) ls[i] = pending[R + N * i];
                HIP_OK(hipMemcpyAsync(dst.p, ls.data(), 8 * Wl, hipMemcpyHostToDevice, st));
                // one search per one-wave workgroup (more searches per wave serialise each
                // other's divergent branches: measured 64 per wave 93 ms, 16: 44, 4: 30, 1: 23 at C3)
                hipLaunchKernelGGL(k_findcycle, dim3((unsigned)Wl), dim3(64), fc_lds_bytes(caps), st, g->view(), dvis.p,
                                   dst.p, Wl, caps, prm, (uint64_t *)scratch.p, dstat.p);
                LAUNCH_OK();
                d2h(g->ctx, mine.st.data(), dstat.p, Wl * sizeof(FcStatus));
            }
            verbose_mark(g->ctx, "fc.round_kernel");
            static const bool verbose = getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1';
            if (verbose && Wl) {
                std::vector<uint64_t> ord(Wl);
                for (uint64_t i = 0; i < Wl; ++i) ord[i] = i;
                const size_t top = std::min<size_t>(5, ord.size());
                std::partial_sort(ord.begin(), ord.begin() + top, ord.end(),
                                  [&](uint64_t a, uint64_t b) { return mine.st[a].steps > mine.st[b].steps; });
                uint64_t tot = 0, trl = 0, mlk = 0;
                for (const auto &x : mine.st) {
                    tot += x.steps;
                    trl += x.relax;
                    mlk = std::max<uint64_t>(mlk, x.locks);
                }
                fprintf(stderr, "[mcaat] fc: %llu searches, %llu steps, %llu relaxations, max locks %llu; longest:",
                        (unsigned long long)Wl, (unsigned long long)tot, (unsigned long long)trl,
                        (unsigned long long)mlk);
                for (size_t q = 0; q < top; ++q)
                    fprintf(stderr, " %u (relax %u, locks %u, ncyc %d, nodes %u)", mine.st[ord[q]].steps,
                            mine.st[ord[q]].relax, mine.st[ord[q]].locks, mine.st[ord[q]].ncyc, mine.st[ord[q]].nnodes);
                fprintf(stderr, "\n");
            }
            // this rank's finished searches (status 0) with cycles, in slot order; on one GPU
            // their nodes stay on the device for the commit (dn_keep, node -> start in dj_keep)
            DevBuf<uint64_t> dn_keep;
            DevBuf<uint32_t> dj_keep;
            {
                std::vector<uint64_t> sel, noff{0}, coff{0};
                for (uint64_t i = 0; i < Wl; ++i) {
                    if (mine.st[i].status != 0 && N == 1) break;  // one GPU: nothing past the first overflow is used
                    if (mine.st[i].status == 0 && mine.st[i].ncyc > 0) {
                        sel.push_back(i);
                        noff.push_back(noff.back() + mine.st[i].nnodes);
                        coff.push_back(coff.back() + mine.st[i].ncyc);
                    }
                }
                // (round 6) one GPU: the nodes stay on the device until the commit says which
                // starts' cycles are results (a window's skipped starts often hold most of them)
                if (N > 1) mine.nodes.resize(noff.back());
                mine.lens.resize(coff.back());
                if (!sel.empty()) {
                    DevBuf<uint64_t> dsel(sel.size()), dno(noff.size()), dco(coff.size()), dn(noff.back());
                    DevBuf<uint16_t> dl(coff.back());
                    HIP_OK(hipMemcpyAsync(dsel.p, sel.data(), 8 * sel.size(), hipMemcpyHostToDevice, st));
                    HIP_OK(hipMemcpyAsync(dno.p, noff.data(), 8 * noff.size(), hipMemcpyHostToDevice, st));
                    HIP_OK(hipMemcpyAsync(dco.p, coff.data(), 8 * coff.size(), hipMemcpyHostToDevice, st));
                    hipLaunchKernelGGL(k_fc_gather, dim3((unsigned)sel.size()), dim3(256), 0, st, (uint64_t *)scratch.p,
                                       pa, caps, dsel.p, dno.p, dco.p, dn.p, dl.p, (uint64_t)sel.size());
                    LAUNCH_OK();
                    if (N > 1) d2h(g->ctx, mine.nodes.data(), dn.p, 8 * mine.nodes.size());
                    d2h(g->ctx, mine.lens.data(), dl.p, 2 * mine.lens.size());
                    if (N == 1) {  // one GPU: slot i is start i
                        dj_keep.alloc(noff.back());
                        hipLaunchKernelGGL(k_fc_owner, dim3((unsigned)sel.size()), dim3(256), 0, st, dsel.p, dno.p,
                                           dj_keep.p, (uint64_t)sel.size());
                        LAUNCH_OK();
                        dn_keep = std::move(dn);
                    }
                    HIP_OK(hipStreamSynchronize(st));
                }
            }
            verbose_mark(g->ctx, "fc.gather_nodes");
            // every rank's outputs (one GPU: its own)
            std::vector<RankOut> others;
            std::vector<const RankOut *> ro(N);
            if (N == 1) {
                ro[0] = &mine;
            } else {
                others.resize(N);
                std::vector<uint64_t> cs, cn, cl;
                auto st_all = comm->allgather_vec(mine.st, &cs);
                auto nd_all = comm->allgather_vec(mine.nodes, &cn);
                auto ln_all = comm->allgather_vec(mine.lens, &cl);
                uint64_t a = 0, b = 0, c = 0;
                for (int r = 0; r < N; ++r) {
                    others[r].st.assign(st_all.begin() + a, st_all.begin() + a + cs[r]);
                    others[r].nodes.assign(nd_all.begin() + b, nd_all.begin() + b + cn[r]);
                    others[r].lens.assign(ln_all.begin() + c, ln_all.begin() + c + cl[r]);
                    a += cs[r];
                    b += cn[r];
                    c += cl[r];
                    ro[r] = &others[r];
                }
            }
            // global view: status of start j and, for starts with cycles, their nodes/lengths
            std::vector<const FcStatus *> hs(W);
            uint64_t first_bad = W;
            for (uint64_t j = 0; j < W; ++j) {
                hs[j] = &ro[j % N]->st[j / N];
                if (hs[j]->status != 0 && first_bad == W) first_bad = j;
            }
            std::vector<const uint64_t *> jn(W, nullptr);
            std::vector<const uint16_t *> jc(W, nullptr);
            std::vector<uint64_t> joff(N == 1 ? W : 0);  // one GPU: start j's nodes at joff[j] on the device
            std::vector<uint32_t> selj;  // starts before the first overflow that found cycles
            uint64_t n_nodes = 0;
            {
                // each rank's outputs are in slot order; only starts before the first overflow
                // are used (one GPU gathers nothing past it)
                std::vector<uint64_t> nptr(N, 0), cptr(N, 0);
                for (uint64_t j = 0; j < first_bad; ++j) {
                    const int o = (int)(j % N);
                    if (hs[j]->ncyc > 0) {
                        if (N == 1) joff[j] = nptr[o];
                        else jn[j] = ro[o]->nodes.data() + nptr[o];
                        jc[j] = ro[o]->lens.data() + cptr[o];
                        nptr[o] += hs[j]->nnodes;
                        cptr[o] += hs[j]->ncyc;
                        selj.push_back((uint32_t)j);
                        n_nodes += hs[j]->nnodes;
                    }
                }
            }
            verbose_mark(g->ctx, "fc.round_gather");
            std::vector<uint8_t> skip;
            const uint64_t f = commit_round(pending, W, first_bad, selj, jn, hs, n_nodes, scratch.p, pa, skip,
                                            dn_keep.p ? dn_keep.p : nullptr, dj_keep.p ? dj_keep.p : nullptr);
            verbose_mark(g->ctx, "fc.commit_device");
            // one GPU: the committed results' nodes, gathered from the device in one copy
            std::vector<uint64_t> hres;
            if (N == 1 && dn_keep.p) {
                std::vector<uint64_t> seg;
                uint64_t tot = 0;
                for (uint64_t j = 0; j < f; ++j)
                    if (!skip[j] && hs[j]->ncyc > 0 && hs[j]->nnodes) {
                        seg.insert(seg.end(), {joff[j], (uint64_t)hs[j]->nnodes, tot});
                        tot += hs[j]->nnodes;
                    }
                if (tot) {
                    DevBuf<uint64_t> dseg(seg.size()), dres(tot);
                    h2d(g->ctx, dseg.p, seg.data(), 8 * seg.size());
                    hipLaunchKernelGGL(k_fc_segs, dim3((unsigned)(seg.size() / 3)), dim3(256), 0, st,
                                       (const uint64_t *)dn_keep.p, (const uint64_t *)dseg.p, dres.p);
                    LAUNCH_OK();
                    hres.resize(tot);
                    d2h(g->ctx, hres.data(), dres.p, 8 * tot);
                    uint64_t at = 0;
                    for (uint64_t j = 0; j < f; ++j)
                        if (!skip[j] && hs[j]->ncyc > 0 && hs[j]->nnodes) {
                            jn[j] = hres.data() + at;
                            at += hs[j]->nnodes;
                        }
                }
            }
            // results of the committed prefix [0, f)
            for (uint64_t j = 0; j < f; ++j) {
                if (skip[j]) continue;
                out->starts.push_back(pending[j]);
                std::vector<uint64_t> fl, of{0};
                if (jn[j]) {
                    fl.assign(jn[j], jn[j] + hs[j]->nnodes);
                    for (int32_t c = 0; c < hs[j]->ncyc; ++c) of.push_back(of.back() + jc[j][c]);
                }
                out->stats[5] += of.size() - 1;
                out->flat.push_back(std::move(fl));
                out->offsets.push_back(std::move(of));
            }
            verbose_mark(g->ctx, "fc.round_commit");
            if (f < W) ++reruns;
            if (f == first_bad && first_bad < W) {
                // scratch overflow at position f: grow the exhausted structure and re-run
                const int code = hs[f]->status;
                if (code == 1) caps.CL *= 4;
                else if (code == 2) caps.CR *= 4;
                else caps.CO *= 2;
                if (caps.CL > (1u << 26) || caps.CR > (1u << 26) || caps.CO > (1u << 28))
                    throw Error(MCAAT_E_CAPACITY, "FindCycle scratch exceeded its growth limit");
            }
            pending.erase(pending.begin(), pending.begin() + f);
            // adapt the speculation window to the observed conflict rate
            const uint64_t wmax = 8192ULL * N;
            if (f < W / 4) window = std::max<uint64_t>(16, window / 2);
            else if (f == W) window = std::min<uint64_t>(wmax, window * 2);
        }
    }
};

// sorted union of every rank's ascending id list
static std::vector<uint64_t> gather_sorted(Comm *comm, const std::vector<uint64_t> &mine) {
    std::vector<uint64_t> all = comm->allgather_vec(mine);
    std::sort(all.begin(), all.end());
    return all;
}

std::vector<uint64_t> cf_depth_level_search(mcaat_graph *g, const std::vector<uint64_t> &cand, int limit, Comm *comm) {
    if (comm && comm->world == 1) comm = nullptr;
    if (comm) {  // candidate i is searched on rank i % N
        std::vector<uint64_t> mine;
        for (size_t i = comm->rank; i < cand.size(); i += comm->world) mine.push_back(cand[i]);
        return gather_sorted(comm, run_dls(g, mine, limit));
    }
    if (knob(g->ctx, "cf.dls_host", 0) != 0 || cand.empty()) return run_dls(g, cand, limit);
    DevBuf<uint64_t> d(cand.size());
    h2d(g->ctx, d.p, cand.data(), 8 * cand.size());
    verbose_mark(g->ctx, "dls.upload");
    return run_dls_dev(g, d.p, cand.size(), limit);
}

void cf_find_cycles(mcaat_graph *g, const mcaat_cf_params &p, const std::vector<uint64_t> &starts, mcaat_cycles *out,
                    Comm *comm) {
    if (comm && comm->world == 1) comm = nullptr;
    FcRunner fr(g, p, out, comm);
    // with threads=1 the reference's bucket loop is one ordered sequence of starts, so the
    // speculative windows run across bucket boundaries
    fr.run_bucket(starts);
    out->stats[6] = fr.rounds;
    out->stats[7] = fr.reruns;
}

void cycle_finder(mcaat_graph *g, const mcaat_cf_params &p, mcaat_cycles *out, Comm *comm) {
    mcaat_ctx *ctx = g->ctx;
    hipStream_t st = ctx->stream;
    const uint64_t D = g->D;
    const uint64_t nw = g->n_words();
    GraphView v = g->view();
    StageTimer timer(ctx);
    if (comm && comm->world == 1) comm = nullptr;
    const int N = comm ? comm->world : 1, R = comm ? comm->rank : 0;
    // grid-stride scans whose per-block totals meet in one counter: a capped grid keeps that
    // counter's atomics to a few thousand
    const unsigned wgrid = grid_for(nw * 64, kBlock, (unsigned)ctx->n_cu * 16);
    const int64_t scan_u = knob(ctx, "cf.scan_u", kScanUDefault);  // words in flight per wave (1, 2, 4)

    // The scans are split over the ranks by 64-edge words ([R*nw/N, (R+1)*nw/N): rank R's ids
    // are whole words): the tips / filter pass's two bitmaps are all-gathered (D/8 bytes each),
    // the recount's counts summed and the candidates gathered. The peel is a global fixpoint
    // over the whole graph and runs on every rank's replica (its first pass then runs as its
    // own kernel: its arrays are 12 B per edge, too much to gather); the searches of steps 5-6
    // are split over the ranks.
    const uint64_t w_lo = nw * (uint64_t)R / (uint64_t)N, w_hi = nw * (uint64_t)(R + 1) / (uint64_t)N;
    // 1-2. CollectTips (before the multiplicity filter) -> seeds of the reduction, and
    // InvalidateMultiplicityOneNodes, in one pass (the filtered bits go to a second bitmap)
    DevBuf<uint64_t> seeds(nw);
    // the list-ranking peel (the default) gets its first pass from this one (cf.fused_init=0:
    // its own k_peel_init)
    PeelState ps;
    const bool fuse = !comm && knob(ctx, "cf.walk_budget", 0) <= 0 && knob(ctx, "cf.fused_init", 1) != 0 && D;
    // (round 4) cf.compact=1: peel arrays over compact slots of the filtered edges (default one per
    // edge; the slots are 32-bit prefix counts, so graphs of 2^32 or more edges use one per edge)
    // Measured (C3): compact slots 36.1 ms of peel against 23.2 with one slot per edge — the
    // removal walks of long chains pay a binary search per edge (PeelArrays::gid) and the tips
    // pass a prefix load per successor; C5 68.1 either way. Off by default (the memory saving
    // stays available: C5's peel state 63 -> 12 GB).
    // (round 6) unset, it is decided after the multiplicity filter (below): compact when the filter
    // keeps under cf.compact_pct % (30) of a fresh graph's edges. C5 keeps 18 %: its peel state
    // falls from 63 to 12 GB at the same peel time (68.1 ms either way); C3 keeps 59 % and stays
    // per id (compact costs it 12 ms there)
    bool compact = knob(ctx, "cf.compact", 0) != 0 && D && D < (1ULL << 32) && knob(ctx, "cf.walk_budget", 0) <= 0;
    // the recount's counts and ChunkStartNodes' filter come from the tips / filter pass
    // (cf.recount = 1: the separate post-peel pass of round 2)
    const bool fold = knob(ctx, "cf.recount", 0) == 0;
    const uint64_t c_lo = std::min<uint64_t>(D, 64 * w_lo), c_hi = std::min<uint64_t>(D, 64 * w_hi);
    uint64_t ccap = std::min<uint64_t>(c_hi - c_lo, (c_hi - c_lo) / 64 + (1u << 20));
    if (knob_set(ctx, "cf.cand_cap")) ccap = (uint64_t)std::max<int64_t>(1, knob(ctx, "cf.cand_cap", 1));  // test knob
    DevBuf<uint64_t> clist;
    uint64_t n_cand = 0, tips_after = 0;
    // every edge valid (as built): the passes before the filter read no unfiltered bitmap
    const bool fresh = g->all_valid && knob(ctx, "cf.fresh", 1) != 0;
    // (round 4) cf.pull_flags=1: the tips pass writes each edge's predecessor flags from its own
    // side (k_tips_filter). Measured slower, off: C3 tips 14.3 -> 15.8 ms, C5 55.2 -> 61.9 ms (the
    // in-edge window gather and in_info read for every filter-valid edge cost more than the
    // scattered flag bytes and the clearing pass they replace)
    const bool pull = knob(ctx, "cf.pull_flags", 0) != 0;
    g->all_valid = false;  // the filter and the peel clear bits from here on
    // the filtered bitmap (whole graph); the peel's compact slots index it, so it stays unchanged
    // until the peel is done (the graph's own copy is the one the peel clears)
    DevBuf<uint64_t> post(mcaat_graph::bitmap_words(D));
    DevBuf<uint32_t> wpre;
    {
        HIP_OK(hipMemsetAsync(post.p + nw, 0, 8, st));  // the padding word
        DevBuf<unsigned long long> c2(4);
        HIP_OK(hipMemsetAsync(c2.p, 0, 32, st));
        std::vector<uint64_t> sz(N);
        for (int r = 0; r < N; ++r) sz[r] = 8 * (nw * (uint64_t)(r + 1) / N - nw * (uint64_t)r / N);
        // 2. InvalidateMultiplicityOneNodes: this rank's words of the filtered bitmap, gathered
        {
            DevBuf<uint64_t> mpost;
            if (comm) mpost.alloc(std::max<uint64_t>(w_hi - w_lo, 1));
            if (w_hi > w_lo) {
                auto kern = scan_u == 1 ? k_post_filter<1> : scan_u == 4 ? k_post_filter<4> : k_post_filter<2>;
                hipLaunchKernelGGL(kern, dim3(wgrid), dim3(kBlock), 0, st, v, w_lo, w_hi, comm ? mpost.p : post.p + w_lo,
                                   c2.p, fresh);
                LAUNCH_OK();
            }
            if (comm) {
                HIP_OK(hipStreamSynchronize(st));
                comm->allgatherv_dev(mpost.p, post.p, sz.data());
            }
        }
        if (!knob_set(ctx, "cf.compact") && !comm && fresh && fuse && D && D < (1ULL << 32) &&
            knob(ctx, "cf.walk_budget", 0) <= 0) {
            unsigned long long low = 0;  // every mult <= 1 edge: on a fresh graph, the edges the filter clears
            d2h(ctx, &low, c2.p + 1, 8);
            const uint64_t kept = D - std::min<uint64_t>(D, low);
            compact = kept * 100 < (uint64_t)std::max<int64_t>(0, knob(ctx, "cf.compact_pct", 30)) * D;
        }
        if (compact) {  // compact slots: exclusive prefix of the filtered words' popcounts
            DevBuf<uint32_t> pc(nw + 1);
            wpre.alloc(nw + 1);
            HIP_OK(hipMemsetAsync(pc.p + nw, 0, 4, st));
            hipLaunchKernelGGL(k_word_pop, dim3(grid_for(nw, kBlock, (unsigned)ctx->n_cu * 16)), dim3(kBlock), 0, st,
                               (const uint64_t *)post.p, nw, pc.p);
            LAUNCH_OK();
            size_t tmp = 0;
            HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, pc.p, wpre.p, (size_t)(nw + 1), st));
            DevBuf<uint8_t> t(tmp);
            HIP_OK(hipcub::DeviceScan::ExclusiveSum(t.p, tmp, pc.p, wpre.p, (size_t)(nw + 1), st));
            uint32_t slots = 0;
            d2h(ctx, &slots, wpre.p + nw, 4);
            ps.post = post.p;
            ps.wpre = wpre.p;
            ps.slots = slots;
        }
        if (fuse) {
            const uint64_t S = std::max<uint64_t>(compact ? ps.slots : D, 1);
            ps.nf.alloc(4 * S);
            ps.nxk.alloc(S);
            if (!pull) HIP_OK(hipMemsetAsync(ps.nf.p, 0, ps.nf.bytes(), st));  // pull: every slot read is written
            ps.ready = true;
        }
        // 1. CollectTips (before the filter: the seeds of the reduction), with the peel's first
        // pass and the candidate filter
        PeelArrays fa{fuse ? ps.nf.p : nullptr, fuse ? ps.nxk.p : nullptr, nullptr, nullptr, nullptr, nullptr,
                      post.p, compact ? wpre.p : nullptr, nw};
      for (;;) {
        if (fold) clist.alloc(ccap ? ccap : 1);
        HIP_OK(hipMemsetAsync(c2.p, 0, 8, st));
        HIP_OK(hipMemsetAsync(c2.p + 2, 0, 16, st));
        DevBuf<uint64_t> mseeds;  // this rank's words when the bitmap is gathered
        if (comm) mseeds.alloc(std::max<uint64_t>(w_hi - w_lo, 1));
        if (w_hi > w_lo) {
            auto pick = [&](auto su) {
                constexpr int U = decltype(su)::value;
                return fresh ? (pull ? k_tips_filter<U, true, true> : k_tips_filter<U, true, false>)
                             : (pull ? k_tips_filter<U, false, true> : k_tips_filter<U, false, false>);
            };
            auto kern = scan_u == 1 ? pick(std::integral_constant<int, 1>{})
                        : scan_u == 4 ? pick(std::integral_constant<int, 4>{}) : pick(std::integral_constant<int, 2>{});
            hipLaunchKernelGGL(kern, dim3(wgrid), dim3(kBlock), 0, st, v, w_lo, w_hi, comm ? mseeds.p : seeds.p + w_lo,
                               (const uint64_t *)post.p, c2.p, fa, (uint64_t)p.threshold_multiplicity,
                               fold ? clist.p : (uint64_t *)nullptr, ccap);
            LAUNCH_OK();
        }
        unsigned long long hc[4];
        HIP_OK(hipMemcpyAsync(hc, c2.p, 32, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        if (fold && hc[3] > ccap) {  // more candidates than the list held: the pass again (idempotent), sized
            ccap = hc[3];
            if (fuse && !pull) HIP_OK(hipMemsetAsync(ps.nf.p, 0, ps.nf.bytes(), st));  // its flag bytes are set again
            continue;
        }
        n_cand = fold ? hc[3] : 0;
        tips_after = hc[2];
        if (comm) {
            comm->allgatherv_dev(mseeds.p, seeds.p, sz.data());
            const auto all = comm->allgather_vec(std::vector<unsigned long long>{hc[0], hc[1]});
            hc[0] = hc[1] = 0;
            for (int r = 0; r < N; ++r) hc[0] += all[2 * r], hc[1] += all[2 * r + 1];
        }
        out->stats[0] = hc[0];
        out->stats[1] = hc[1];
        // the graph's bitmap becomes the filtered one (its pre-filter bits are no longer read)
        HIP_OK(hipMemcpyAsync(g->valid.p, post.p, 8 * nw, hipMemcpyDeviceToDevice, st));
        v = g->view();
        break;
      }
    }
    timer.mark("tips_filter");
    verbose_mark(ctx, "cf.tips_filter");
    // 3. RecursiveReduction from every seed
    if (!fuse) ps.ready = false;
    run_peel(g, seeds.p, (fuse || compact) ? &ps : nullptr);
    seeds.release();
    ps.nf.release();
    ps.nxk.release();
    post.release();
    wpre.release();
    timer.mark("peel");
    verbose_mark(ctx, "cf.peel");
    // 4-5. valid count + tips after pruning, and ChunkStartNodes' candidate filter (its
    // InvalidateMultiplicityOneNodes, cycle_finder.cpp:391-393, is a no-op here: step 2 already
    // cleared every mult <= 1 edge and nothing since sets a valid bit, and the count it would
    // print is stats[1], every mult <= 1 edge, valid or not)
    std::vector<uint64_t> cand;
    DevBuf<uint64_t> dcand;  // one GPU, fold path: the sorted candidates stay on the device
    uint64_t n_dcand = 0;
    const bool dev_dls = knob(ctx, "cf.dls_host", 0) == 0;
    if (fold) {
        // valid count: a popcount of this rank's words; tips: the post-filter tips that were
        // not seeds (tips pass); candidates: the listed ones still valid, in ascending id order
        DevBuf<unsigned long long> c1(1);
        HIP_OK(hipMemsetAsync(c1.p, 0, 8, st));
        if (w_hi > w_lo) {
            hipLaunchKernelGGL(k_popcount, dim3(wgrid), dim3(kBlock), 0, st, (const uint64_t *)g->valid.p, w_lo, w_hi, c1.p);
            LAUNCH_OK();
        }
        out->stats[2] = read_counter(ctx, c1.p);
        out->stats[3] = tips_after;  // this rank's words (summed over the ranks below)
        if (n_cand) {
            DevBuf<uint8_t> fl(n_cand);
            DevBuf<uint64_t> kept(n_cand), sorted(n_cand);
            DevBuf<unsigned long long> nk(1);
            hipLaunchKernelGGL(k_still_valid, dim3(grid_for(n_cand, kBlock)), dim3(kBlock), 0, st, (const uint64_t *)g->valid.p,
                               (const uint64_t *)clist.p, n_cand, fl.p);
            LAUNCH_OK();
            size_t tmp = 0;
            HIP_OK(hipcub::DeviceSelect::Flagged(nullptr, tmp, clist.p, fl.p, kept.p, nk.p, (size_t)n_cand, st));
            {
                DevBuf<uint8_t> t(tmp);
                HIP_OK(hipcub::DeviceSelect::Flagged(t.p, tmp, clist.p, fl.p, kept.p, nk.p, (size_t)n_cand, st));
            }
            const uint64_t nkept = read_counter(ctx, nk.p);
            if (nkept) {
                tmp = 0;
                HIP_OK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, kept.p, sorted.p, (size_t)nkept, 0, 40, st));
                DevBuf<uint8_t> t(tmp);
                HIP_OK(hipcub::DeviceRadixSort::SortKeys(t.p, tmp, kept.p, sorted.p, (size_t)nkept, 0, 40, st));
            }
            if (comm || !dev_dls) {
                cand.resize(nkept);
                if (nkept) d2h(ctx, cand.data(), sorted.p, 8 * nkept);
            } else {  // one GPU: DepthLevelSearch straight from the device list
                dcand = std::move(sorted);
                n_dcand = nkept;
            }
        }
        clist.release();
    } else {
        // rank R takes the candidates among its words' ids, and counts over its words
        const uint64_t lo = std::min<uint64_t>(D, 64 * w_lo), hi = std::min<uint64_t>(D, 64 * w_hi);
        uint64_t cap = std::min<uint64_t>(hi - lo, (hi - lo) / 64 + (1u << 20));
        if (knob_set(ctx, "cf.cand_cap")) cap = (uint64_t)std::max<int64_t>(1, knob(ctx, "cf.cand_cap", 1));  // test knob
        DevBuf<unsigned long long> c3(3);
        for (;;) {
            DevBuf<uint64_t> list(cap ? cap : 1);
            HIP_OK(hipMemsetAsync(c3.p, 0, 24, st));
            if (w_hi > w_lo) {
                auto kern = scan_u == 1 ? k_recount_candidates<1> : scan_u == 4 ? k_recount_candidates<4>
                                                                                : k_recount_candidates<2>;
                hipLaunchKernelGGL(kern, dim3(wgrid), dim3(kBlock), 0, st, v,
                                   (uint64_t)p.threshold_multiplicity, lo, hi, w_lo, w_hi, list.p, cap, c3.p);
                LAUNCH_OK();
            }
            unsigned long long hc[3];
            HIP_OK(hipMemcpyAsync(hc, c3.p, 24, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            out->stats[2] = hc[0];
            out->stats[3] = hc[1];
            if (hc[2] > cap) {  // more candidates than the first list held: the pass again, sized
                cap = hc[2];
                continue;
            }
            cand.resize(hc[2]);
            if (hc[2]) {
                // ascending id order (the append order is the atomics'): sorted on the device
                // (C5: 3.8M candidates, 0.25 s of host sort)
                DevBuf<uint64_t> sorted(hc[2]);
                size_t tmp = 0;
                HIP_OK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, list.p, sorted.p, (size_t)hc[2], 0, 40, st));
                DevBuf<uint8_t> t(tmp);
                HIP_OK(hipcub::DeviceRadixSort::SortKeys(t.p, tmp, list.p, sorted.p, (size_t)hc[2], 0, 40, st));
                d2h(ctx, cand.data(), sorted.p, 8 * hc[2]);
            }
            break;
        }
    }
    if (comm) {  // the ranks' word counts summed
        const auto all = comm->allgather_vec(std::vector<uint64_t>{out->stats[2], out->stats[3]});
        out->stats[2] = out->stats[3] = 0;
        for (int r = 0; r < N; ++r) out->stats[2] += all[2 * r], out->stats[3] += all[2 * r + 1];
    }
    timer.mark("recount");
    if (comm) cand = gather_sorted(comm, cand);
    timer.mark("candidates");
    verbose_mark(ctx, "cf.candidates");
    std::vector<uint64_t> pass;
    if (comm) {
        // candidate i is searched on rank i % N
        std::vector<uint64_t> mine;
        for (size_t i = R; i < cand.size(); i += N) mine.push_back(cand[i]);
        pass = gather_sorted(comm, run_dls(g, mine, p.cycle_max_length));
    } else if (fold && dev_dls) {
        pass = run_dls_dev(g, dcand.p, n_dcand, p.cycle_max_length);
        dcand.release();
    } else {
        pass = run_dls(g, cand, p.cycle_max_length);
    }
    timer.mark("dls");
    verbose_mark(ctx, "cf.dls");
    std::map<int, std::vector<uint64_t>, std::greater<int>> chunks;
    if (!pass.empty()) {
        DevBuf<uint64_t> ids(pass.size());
        DevBuf<uint16_t> m(pass.size());
        HIP_OK(hipMemcpyAsync(ids.p, pass.data(), 8 * pass.size(), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_gather_mult, dim3(grid_for(pass.size(), kBlock)), dim3(kBlock), 0, st, g->mult.p, ids.p,
                           (uint64_t)pass.size(), m.p);
        LAUNCH_OK();
        std::vector<uint16_t> hm(pass.size());
        HIP_OK(hipMemcpyAsync(hm.data(), m.p, 2 * pass.size(), hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        for (size_t i = 0; i < pass.size(); ++i) {
            const double l2 = std::ceil(std::log2(double(hm[i])));  // cycle_finder.cpp:414
            chunks[(int)l2].push_back(pass[i]);
        }
    }
    for (auto &kv : chunks)
        for (uint64_t id : kv.second) { out->cand_ids.push_back(id); out->cand_bucket.push_back(kv.first); }
    out->stats[4] = out->cand_ids.size();
    // 6. bucket loop
    verbose_mark(ctx, "cf.chunks");
    FcRunner fr(g, p, out, comm);
    verbose_mark(ctx, "cf.fc_setup");
    // with threads=1 the reference's bucket loop is one ordered sequence of starts, so the
    // speculative windows run across bucket boundaries
    fr.run_bucket(out->cand_ids);
    out->stats[6] = fr.rounds;
    out->stats[7] = fr.reruns;
    timer.mark("find_cycle");
    verbose_mark(ctx, "cf.find_cycle");
    HIP_OK(hipStreamSynchronize(st));
    timer.finish();
}
// the valid edges in ascending id order (their rank = their position) and each one's valid
// out-neighbours as ranks, DESCENDING ids as OutgoingEdges (step 7's SCC split over a small
// valid set: dense arrays instead of a hash lookup per neighbour)
__global__ void __launch_bounds__(kBlock) k_word_popc(const uint64_t *bm, uint64_t nw, uint64_t *cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) cnt[w] = __popcll(bm[w]);
}
__global__ void __launch_bounds__(kBlock) k_valid_out_ranks(GraphView g, const uint64_t *wpre, uint64_t *ids,
                                                            uint32_t *nbr, uint8_t *cnt) {
    const uint64_t nw = (g.D + 63) / 64, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nw * 64; e += stride) {
        const uint64_t w = e >> 6, word = g.valid[w];
        if (!((word >> (e & 63)) & 1)) continue;
        const uint64_t r = wpre[w] + __popcll(word & ((1ull << (e & 63)) - 1));
        ids[r] = e;
        uint64_t out[4];
        const int n = dev_outgoing(g, e, out);
        for (int j = 0; j < n; ++j) {
            const uint64_t y = out[j], wy = g.valid[y >> 6];
            nbr[4 * r + j] = (uint32_t)(wpre[y >> 6] + __popcll(wy & ((1ull << (y & 63)) - 1)));
        }
        cnt[r] = (uint8_t)n;
    }
}

uint64_t graph_valid_out_ranks(const mcaat_graph *g, uint64_t *ids, uint32_t *nbr, uint8_t *cnt) {
    hipStream_t st = g->ctx->stream;
    const uint64_t nw = g->n_words();
    if (!nw) return 0;
    DevBuf<uint64_t> pc(nw + 1), wpre(nw + 1);
    HIP_OK(hipMemsetAsync(pc.p + nw, 0, 8, st));
    hipLaunchKernelGGL(k_word_popc, dim3(grid_for(nw, kBlock, (unsigned)g->ctx->n_cu * 16)), dim3(kBlock), 0, st,
                       (const uint64_t *)g->valid.p, nw, pc.p);
    LAUNCH_OK();
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, pc.p, wpre.p, (size_t)(nw + 1), st));
    DevBuf<uint8_t> t(tmp);
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(t.p, tmp, pc.p, wpre.p, (size_t)(nw + 1), st));
    uint64_t n = 0;
    d2h(g->ctx, &n, wpre.p + nw, 8);
    if (!ids || !n) return n;
    if (n >= (1ULL << 32)) throw Error(MCAAT_E_CAPACITY, "valid subgraph of 2^32 or more edges");
    DevBuf<uint64_t> di(n);
    DevBuf<uint32_t> dn(4 * n);
    DevBuf<uint8_t> dc(n);
    hipLaunchKernelGGL(k_valid_out_ranks, dim3(grid_for(nw * 64, kBlock, (unsigned)g->ctx->n_cu * 32)), dim3(kBlock), 0,
                       st, g->view(), (const uint64_t *)wpre.p, di.p, dn.p, dc.p);
    LAUNCH_OK();
    d2h(g->ctx, ids, di.p, 8 * n);
    d2h(g->ctx, nbr, dn.p, 16 * n);
    d2h(g->ctx, cnt, dc.p, n);
    return n;
}

void graph_neighbors(const mcaat_graph *g, const uint64_t *ids, size_t n, int incoming, uint64_t *out,
                     int32_t *counts) {
    if (!n) return;
    hipStream_t st = g->ctx->stream;
    DevBuf<uint64_t> di(n), dout(4 * n);
    DevBuf<int32_t> dc(n);
    HIP_OK(hipMemcpyAsync(di.p, ids, 8 * n, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_neighbors, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, g->view(), di.p, (uint64_t)n,
                       incoming, dout.p, dc.p);
    LAUNCH_OK();
    HIP_OK(hipMemcpyAsync(out, dout.p, 32 * n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(counts, dc.p, 4 * n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
}

__global__ void k_gather_key_mult(const uint64_t *key, const uint16_t *mult, const uint64_t *ids, uint64_t n,
                                  uint64_t *ko, uint16_t *mo) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t e = ids[i];
    if (ko) ko[i] = key[e];
    if (mo) mo[i] = mult[e];
}

void graph_gather(const mcaat_graph *g, const uint64_t *ids, size_t n, uint64_t *keys, uint16_t *mult) {
    if (!n) return;
    hipStream_t st = g->ctx->stream;
    DevBuf<uint64_t> di(n), dk(keys ? n : 1);
    DevBuf<uint16_t> dm(mult ? n : 1);
    HIP_OK(hipMemcpyAsync(di.p, ids, 8 * n, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_gather_key_mult, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, g->key.p, g->mult.p, di.p,
                       (uint64_t)n, keys ? dk.p : (uint64_t *)nullptr, mult ? dm.p : (uint16_t *)nullptr);
    LAUNCH_OK();
    if (keys) HIP_OK(hipMemcpyAsync(keys, dk.p, 8 * n, hipMemcpyDeviceToHost, st));
    if (mult) HIP_OK(hipMemcpyAsync(mult, dm.p, 2 * n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
}

void graph_set_valid(mcaat_graph *g, const uint64_t *ids, size_t n, int valid) {
    if (!n) return;
    for (size_t i = 0; i < n; ++i)
        if (ids[i] >= g->D) throw Error(MCAAT_E_INVALID, "edge id out of range");
    hipStream_t st = g->ctx->stream;
    DevBuf<uint64_t> di(n);
    HIP_OK(hipMemcpyAsync(di.p, ids, 8 * n, hipMemcpyHostToDevice, st));
    if (!valid) g->all_valid = false;
    hipLaunchKernelGGL(k_set_bits, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, g->valid.p, di.p, (uint64_t)n,
                       valid);
    LAUNCH_OK();
    HIP_OK(hipStreamSynchronize(st));
}

void graph_download_valid(const mcaat_graph *g, uint8_t *valid) {
    if (!g->D) return;
    hipStream_t st = g->ctx->stream;
    DevBuf<uint8_t> d(g->D);
    hipLaunchKernelGGL(k_unpack_bits, dim3(grid_for(g->D, kBlock)), dim3(kBlock), 0, st, g->valid.p, g->D, d.p);
    LAUNCH_OK();
    HIP_OK(hipMemcpyAsync(valid, d.p, g->D, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
}

// loads this file's code object now (HIP defers it to the first launch of one of its kernels)
void preload_cycle_finder() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, (const void *)k_word_pop);
}

}  // namespace mcaat
