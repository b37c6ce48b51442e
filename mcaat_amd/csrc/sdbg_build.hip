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

__global__ void __launch_bounds__(kBlock) k_count_pal(const uint64_t *ckeys, uint64_t n, int k, unsigned long long *n_pal) {
    const int E = k + 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long c = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        c += ckeys[i] == lsb_rc(ckeys[i], E);
    block_add(n_pal, c);
}

// dir[p] = first index whose key prefix (top B of 2E bits) >= p, p in [0, 2^B]: one streaming
// pass over the sorted keys, edge e writing the prefixes (prefix(e-1), prefix(e)] (every prefix
// is written by exactly one edge: the first at or above it, or e = D for those above the last
// key). A wave takes 256 consecutive edges (four coalesced loads in flight); each edge's
// predecessor prefix comes from the neighbouring lane. Round 2 ran one binary search over all
// D keys per prefix (C2: 2^28 searches, 9.9 ms).
// The keys must be strictly ascending and below 2^2E (sorted unique BOSS keys): an edge that
// breaks either sets *bad and writes nothing past dir (its prefix is clamped), and the host
// turns the flag into MCAAT_E_INVALID.
constexpr int kDirU = 4;
__global__ void __launch_bounds__(kBlock) k_dir(const uint64_t *key, uint64_t D, int shift, uint64_t nprefix,
                                                uint64_t key_lim, uint64_t *dir, int *bad) {
    const int lane = threadIdx.x & 63;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; c * 64 * kDirU <= D; c += nwaves) {
        const uint64_t base = c * 64 * kDirU;
        const uint64_t kprev = base ? key[base - 1] : 0;
        uint64_t p[kDirU];
        bool wrong = false;
#pragma unroll
        for (int j = 0; j < kDirU; ++j) {
            const uint64_t e = base + 64 * j + lane;
            const uint64_t kv = e < D ? key[e] : 0;
            const uint64_t kl = __shfl_up(kv, 1);  // the predecessor's key (lanes > 0)
            p[j] = e < D ? kv >> shift : nprefix;
            if (e < D) wrong |= kv >= key_lim;
            if (e < D && lane) wrong |= kv <= kl;
            p[j] = p[j] < nprefix ? p[j] : nprefix;
        }
        // the first key of each 64-edge row against the last of the row before it
#pragma unroll
        for (int j = 0; j < kDirU; ++j) {
            const uint64_t e = base + 64 * j;
            if (lane == 0 && e < D && e > 0) wrong |= key[e] <= (j ? key[e - 1] : kprev);
        }
        if (wrong) *bad = 1;
        uint64_t before = base ? (kprev >> shift) + 1 : 0;  // first prefix of this chunk
        before = before < nprefix + 1 ? before : nprefix + 1;
#pragma unroll
        for (int j = 0; j < kDirU; ++j) {
            const uint64_t e = base + 64 * j + lane;
            const uint64_t up = __shfl_up(p[j], 1);
            const uint64_t last = j ? __shfl(p[j - 1], 63) + 1 : before;
            const uint64_t first = lane ? up + 1 : last;
            if (e <= D)
                for (uint64_t q = first; q <= p[j]; ++q) dir[q] = e;
        }
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

// out_info[e]: the target node's first edge and its W mask, by a directory-bounded search
// (consecutive edges' targets form 4 monotone streams, one per W). in_info is written from
// the predecessor side: the in-edges of node N are the edges with W == c in the (k-1)-suffix
// group of any of them, so the first such edge of the group (a local scan around e) writes
// in_info for every edge of N = target(e) — no search from the random in-group of each edge.
// Edges of nodes without predecessors keep in_info = 0 (an empty mask).
__global__ void __launch_bounds__(kBlock) k_adjacency(const uint64_t *key, uint64_t D, int k, const uint64_t *dir,
                                                      int shift, uint64_t *out_info, uint64_t *in_info) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < D; e += stride) {
        const uint64_t K = key[e];
        const uint64_t W = K & 3, R = K >> 2;
        // out: edges of node target(e) = label s[1..k-1]W
        const uint64_t Rt = (W << (2 * (k - 1))) | (R >> 2);
        const uint64_t lo = lower_bound_dir(key, dir, shift, Rt << 2);
        unsigned m = 0;
        for (uint64_t i = lo; i < D && (key[i] >> 2) == Rt; ++i) m |= 1u << (key[i] & 3);
        out_info[e] = lo | ((uint64_t)m << kIdxBits);
        if (!m) continue;  // target has no out-edges: no edge has it as source
        // e's group: edges whose labels share s[1..k-1] (key >> 4); positions with W == W_e
        const uint64_t gk = K >> 4;
        uint64_t gs = e;
        while (gs > 0 && (key[gs - 1] >> 4) == gk) --gs;
        unsigned pm = 0;
        int j = 0;
        for (uint64_t i = gs; i < D && (key[i] >> 4) == gk && j < 16; ++i, ++j)
            if ((key[i] & 3) == W) pm |= 1u << j;
        if ((uint64_t)(__ffs(pm) - 1) != e - gs) continue;  // another in-edge of N writes
        const uint64_t v = gs | ((uint64_t)pm << kIdxBits);
        const int deg = __popc(m);
        for (int r = 0; r < deg; ++r) in_info[lo + r] = v;
    }
}

// The same for the block's run of kAdjB consecutive edges, with every search and scan in LDS.
// Sources are sorted, so for each W the targets (W, s[1..k-1]) of the run lie in one key
// range, bounded by the run's first and last source; the four ranges (~kAdjB/4 keys each)
// and the run's own keys (with a group-sized halo on each side, for the in-group scans) are
// loaded once, coalesced. A range larger than cap (skewed key spaces) falls back to the
// directory search in global memory. The ranges come from k_adj_bounds (one thread per
// (run, W)), so a run's range and own-key loads go out together: round 2 searched the
// directory inside the run's workgroup first, a chain of dependent loads per run (C2 30 ms).
constexpr int kAdjB = 2048;
constexpr int kAdjT = 1024;   // threads per run: two edges each
constexpr int kAdjCap = 1024;
constexpr int kAdjHalo = 16;  // an in-group holds at most 16 edges
__global__ void __launch_bounds__(kBlock) k_adj_bounds(const uint64_t *key, uint64_t D, int k, const uint64_t *dir,
                                                       int shift, uint64_t nruns, uint64_t *bounds) {
    const uint64_t top = (uint64_t)1 << (2 * (k - 1));
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < 4 * nruns; t += stride) {
        const uint64_t r = t >> 2, W = t & 3;
        const uint64_t e0 = r * kAdjB, e1 = e0 + kAdjB < D ? e0 + kAdjB : D;
        const uint64_t a = (W * top) | (key[e0] >> 4), b = (W * top) | (key[e1 - 1] >> 4);
        const uint64_t lo = lower_bound_dir(key, dir, shift, a << 2);
        const uint64_t qb = (b + 1) << 2;  // past the key space when b is the last label
        const uint64_t hi = qb >> (2 * (k + 1)) ? D : lower_bound_dir(key, dir, shift, qb);
        bounds[8 * r + W] = lo;
        bounds[8 * r + 4 + W] = hi;
    }
}

__global__ void __launch_bounds__(kAdjT) k_adjacency_lds(const uint64_t *key, uint64_t D, int k, const uint64_t *dir,
                                                         int shift, uint32_t cap, const uint64_t *bounds,
                                                         uint64_t *out_info, uint64_t *in_info) {
    __shared__ uint64_t rng[4][kAdjCap];
    __shared__ uint64_t own[kAdjB + 2 * kAdjHalo];
    __shared__ uint64_t srlo[4];
    __shared__ uint32_t srn[4];
    const uint64_t e0 = (uint64_t)blockIdx.x * kAdjB;
    if (e0 >= D) return;
    const uint64_t e1 = e0 + kAdjB < D ? e0 + kAdjB : D;
    // the run's four ranges (uniform loads), also kept in LDS for the per-edge lookups
    uint64_t rlo[4];
    uint32_t rn[4];
#pragma unroll
    for (int W = 0; W < 4; ++W) {
        rlo[W] = bounds[8 * blockIdx.x + W];
        const uint64_t hi = bounds[8 * blockIdx.x + 4 + W];
        rn[W] = hi - rlo[W] <= (uint64_t)cap ? (uint32_t)(hi - rlo[W]) : 0xFFFFFFFFu;
    }
    if (threadIdx.x < 4) {
        srlo[threadIdx.x] = rlo[threadIdx.x];
        srn[threadIdx.x] = rn[threadIdx.x];
    }
    // own[j] = key[e0 - kAdjHalo + j]; outside [0, D): a value no group matches
    const uint64_t olo = e0 >= (uint64_t)kAdjHalo ? e0 - kAdjHalo : 0;
    const uint32_t opad = (uint32_t)(e0 - olo);  // halo entries actually before e0
    for (uint32_t j = threadIdx.x; j < kAdjB + 2 * kAdjHalo; j += kAdjT) {
        const uint64_t x = e0 + j - kAdjHalo;  // wraps below 0 for the first run
        own[j] = (j >= (uint32_t)kAdjHalo - opad && x < D) ? key[x] : ~0ULL;
    }
#pragma unroll
    for (int W = 0; W < 4; ++W) {
        const uint32_t n = rn[W];
        if (n == 0xFFFFFFFFu) continue;
        for (uint32_t i = threadIdx.x; i < n; i += kAdjT) rng[W][i] = key[rlo[W] + i];
    }
    __syncthreads();
    for (uint64_t e = e0 + threadIdx.x; e < e1; e += kAdjT) {
        const uint32_t oe = (uint32_t)(e - e0) + kAdjHalo;
        const uint64_t K = own[oe];
        const uint64_t W = K & 3, R = K >> 2;
        const uint64_t Rt = (W << (2 * (k - 1))) | (R >> 2);
        uint64_t lo;
        unsigned m = 0;
        const uint32_t n = srn[W];
        if (n != 0xFFFFFFFFu) {
            const uint64_t *r = rng[W];
            const uint64_t q = Rt << 2;
            uint32_t a = 0, b = n;
            while (a < b) {
                const uint32_t mid = (a + b) >> 1;
                if (r[mid] < q) a = mid + 1; else b = mid;
            }
            lo = srlo[W] + a;
            // the range holds every key below (last target + 1) << 2: all of Rt's edges
            for (uint32_t i = a; i < n && (r[i] >> 2) == Rt; ++i) m |= 1u << (r[i] & 3);
        } else {
            lo = lower_bound_dir(key, dir, shift, Rt << 2);
            for (uint64_t i = lo; i < D && (key[i] >> 2) == Rt; ++i) m |= 1u << (key[i] & 3);
        }
        out_info[e] = lo | ((uint64_t)m << kIdxBits);
        if (!m) continue;
        // e's in-group (labels sharing s[1..k-1], key >> 4) from the staged keys; a group cut
        // by the halo's edge cannot occur (groups hold at most kAdjHalo edges) except at the
        // ends of the key array, where the ~0 fill stops the scans
        const uint64_t gk = K >> 4;
        uint32_t gs = oe;
        while (gs > 0 && (own[gs - 1] >> 4) == gk) --gs;
        unsigned pm = 0;
        int j = 0;
        for (uint32_t q = gs; q < (uint32_t)(kAdjB + 2 * kAdjHalo) && (own[q] >> 4) == gk && j < 16; ++q, ++j)
            if ((own[q] & 3) == W) pm |= 1u << j;
        if ((uint32_t)(__ffs(pm) - 1) != oe - gs) continue;
        const uint64_t v = (e0 - kAdjHalo + gs) | ((uint64_t)pm << kIdxBits);
        const int deg = __popc(m);
        for (int r = 0; r < deg; ++r) in_info[lo + r] = v;
    }
}

// Round 3: in_info written from the owning side, coalesced. Runs start at group boundaries
// (edges sharing key >> 4; at most 16), so every in-edge of a node sits in one run: the run of
// the node's writer (the first in-edge of the group with the node's W, as above). Run r owns,
// for each W, the in_info slots of the targets between its first source and the next run's
// first source: [O_W(r), O_W(r + 1)) with O_W(r) = lower_bound((W, key[s_r] >> 4) << 2), run 0
// from the start of the W quarter and the last run to its end, so the owned ranges tile
// [0, D) and a run's targets (the old per-W search ranges) lie inside its owned ranges. A run
// stages the keys of its four owned ranges and their in_info words (zero: no predecessor) in
// LDS, searches and fills them there, and writes every owned slot once: no clearing pass and
// no scattered 8-B stores (C2: those cost 7.5 ms of 23 plus the 19-GB clear). A run whose owned
// ranges exceed the LDS cap clears them in global memory and writes directly (directory search).
constexpr int kOwnT = 1024;               // threads per run
constexpr int kOwnB = 2048;               // nominal edges per run (its start moves to a group start)
constexpr int kOwnMax = kOwnB + 16;       // a run holds at most this many edges
constexpr int kOwnCap = 3072;             // staged owned slots (~kOwnB on average)
// bounds[5 r] = s_r (run start, group aligned), bounds[5 r + 1 + W] = O_W(r); r = nruns: D, quarter ends
__global__ void __launch_bounds__(kBlock) k_own_bounds(const uint64_t *key, uint64_t D, int k, const uint64_t *dir,
                                                       int shift, uint64_t nruns, uint64_t *bounds) {
    const uint64_t top = (uint64_t)1 << (2 * (k - 1));
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= nruns; r += stride) {
        uint64_t s = r * kOwnB;
        if (r == nruns || s >= D) s = D;
        else if (s > 0) {
            const uint64_t g0 = key[s - 1] >> 4;
            while (s < D && (key[s] >> 4) == g0) ++s;  // the next group start (<= 15 steps)
        }
        bounds[5 * r] = s;
        for (uint64_t W = 0; W < 4; ++W) {
            // target key prefix (W, label s[1..k-1]) of the run's first source; run 0 and the
            // end sentinel take the W quarter's ends
            uint64_t t;
            if (r == 0) t = W * top;
            else if (s >= D) t = (W + 1) * top;
            else t = (W * top) | (key[s] >> 4);
            const uint64_t q = t << 2;
            bounds[5 * r + 1 + W] = q >> (2 * (k + 1)) ? D : lower_bound_dir(key, dir, shift, q);
        }
    }
}

__global__ void __launch_bounds__(kOwnT) k_adjacency_own(const uint64_t *key, uint64_t D, int k, const uint64_t *dir,
                                                         int shift, uint32_t cap, const uint64_t *bounds,
                                                         uint64_t *out_info, uint64_t *in_info) {
    __shared__ uint64_t own[kOwnMax];
    __shared__ uint64_t okey[kOwnCap];   // keys of the owned ranges, W after W
    __shared__ uint64_t ist[kOwnCap];    // their in_info words
    const uint64_t r = blockIdx.x;
    const uint64_t s0 = bounds[5 * r], s1 = bounds[5 * (r + 1)];
    if (s0 >= s1) return;
    const uint32_t n = (uint32_t)(s1 - s0);
    uint64_t a[4];
    uint32_t len[4], off[4];
    uint32_t tot = 0;
#pragma unroll
    for (int W = 0; W < 4; ++W) {
        a[W] = bounds[5 * r + 1 + W];
        len[W] = (uint32_t)(bounds[5 * (r + 1) + 1 + W] - a[W]);
        off[W] = tot;
        tot += len[W];
    }
    const bool staged = tot <= cap;
    for (uint32_t j = threadIdx.x; j < n; j += kOwnT) own[j] = key[s0 + j];
    if (staged) {
#pragma unroll
        for (int W = 0; W < 4; ++W)
            for (uint32_t i = threadIdx.x; i < len[W]; i += kOwnT) {
                okey[off[W] + i] = key[a[W] + i];
                ist[off[W] + i] = 0;
            }
    } else {
#pragma unroll
        for (int W = 0; W < 4; ++W)
            for (uint32_t i = threadIdx.x; i < len[W]; i += kOwnT) in_info[a[W] + i] = 0;
    }
    __syncthreads();  // (also drains the clearing stores of an unstaged run before its direct writes)
    for (uint32_t j = threadIdx.x; j < n; j += kOwnT) {
        const uint64_t e = s0 + j;
        const uint64_t K = own[j];
        const uint32_t W = (uint32_t)(K & 3);
        const uint64_t Rt = ((uint64_t)W << (2 * (k - 1))) | (K >> 4);
        uint64_t lo;
        unsigned m = 0;
        if (staged) {
            const uint64_t *rk = okey + off[W];
            const uint32_t nn = len[W], q = 0;
            (void)q;
            const uint64_t qk = Rt << 2;
            uint32_t x = 0, y = nn;
            while (x < y) {
                const uint32_t mid = (x + y) >> 1;
                if (rk[mid] < qk) x = mid + 1; else y = mid;
            }
            lo = a[W] + x;
            for (uint32_t i = x; i < nn && (rk[i] >> 2) == Rt; ++i) m |= 1u << (rk[i] & 3);
        } else {
            lo = lower_bound_dir(key, dir, shift, Rt << 2);
            for (uint64_t i = lo; i < D && (key[i] >> 2) == Rt; ++i) m |= 1u << (key[i] & 3);
        }
        out_info[e] = lo | ((uint64_t)m << kIdxBits);
        if (!m) continue;
        // e's group lies inside the run (runs start at group starts)
        const uint64_t gk = K >> 4;
        uint32_t gs = j;
        while (gs > 0 && (own[gs - 1] >> 4) == gk) --gs;
        unsigned pm = 0;
        int t = 0;
        for (uint32_t q = gs; q < n && (own[q] >> 4) == gk && t < 16; ++q, ++t)
            if ((own[q] & 3) == W) pm |= 1u << t;
        if ((uint32_t)(__ffs(pm) - 1) != j - gs) continue;  // another in-edge of the node writes
        const uint64_t v = (s0 + gs) | ((uint64_t)pm << kIdxBits);
        const int deg = __popc(m);
        if (staged)
            for (int q = 0; q < deg; ++q) ist[off[W] + (uint32_t)(lo - a[W]) + q] = v;
        else
            for (int q = 0; q < deg; ++q) in_info[lo + q] = v;
    }
    if (!staged) return;
    __syncthreads();
#pragma unroll
    for (int W = 0; W < 4; ++W)
        for (uint32_t i = threadIdx.x; i < len[W]; i += kOwnT) in_info[a[W] + i] = ist[off[W] + i];
}

__global__ void __launch_bounds__(kBlock) k_valid_init(uint64_t *valid, uint64_t D) {
    const uint64_t nw = (D + 63) / 64;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
        const uint64_t rem = D - w * 64;
        valid[w] = rem >= 64 ? ~0ULL : ((1ULL << rem) - 1);
    }
}

// ---- MSD edge sort (k <= 28) ------------------------------------------------------------
// Oriented edges are items (key remainder << 16 | mult): level 1 scatters them by the top 11
// key bits into 2048 buckets, level 2 by the next 11 bits into 2048 sub-buckets each, both
// with per-chunk runs aligned to 64-B lines and LDS line buffers (whole-line HBM writes);
// level 3 sorts each ~D/4M-item bucket in LDS (bitonic, one wave per bucket; a workgroup
// for large ones) and writes keys and multiplicities. Padding items are ~0 (sort last).
constexpr int kMB = 11;               // bits per MSD level
constexpr int kMS = 1 << kMB;         // buckets per level
constexpr int kIL = 8;                // items per 64-B line
constexpr uint64_t kPad = ~0ULL;
constexpr uint32_t kCh1 = 32768;      // canonical entries per level-1 chunk (<= 2 items each)
constexpr uint32_t kCh2 = 65536;      // items per level-2 chunk
constexpr int kWaveSort = 512;        // largest level-3 bucket sorted by one wave
constexpr int kMidSort = 2048;        // largest sorted by a 256-thread workgroup (16 KB)
constexpr int kSmallMid = 1024;       // largest sorted by a 128-thread workgroup (8 KB)
constexpr int kBlockSort = 16384;     // largest sorted by a 1024-thread workgroup (128 KB)

__device__ __forceinline__ uint32_t round8(uint32_t x) { return (x + kIL - 1) & ~(uint32_t)(kIL - 1); }

// oriented items of a canonical count: top-11-bit bucket and the item word
__device__ __forceinline__ int msd_items(uint64_t a, uint32_t c, int k, uint32_t *bk, uint64_t *it) {
    const int E = k + 1, rb = 2 * E - kMB;
    const uint64_t b = lsb_rc(a, E);
    const uint64_t m = a == b ? 2ull * c : (uint64_t)c;
    const uint64_t mult = m > 65535 ? 65535 : m;
    const uint64_t K0 = boss_key(a, k);
    bk[0] = (uint32_t)(K0 >> rb);
    it[0] = ((K0 & mask_bits(rb)) << 16) | mult;
    if (a == b) return 1;
    const uint64_t K1 = boss_key(b, k);
    bk[1] = (uint32_t)(K1 >> rb);
    it[1] = ((K1 & mask_bits(rb)) << 16) | mult;
    return 2;
}

// level-1 per-chunk bucket counts: written per chunk (cc[c][b]), and their line counts summed
// per block of kBlkCh chunks (blk[j][b]); k_blk_scan / k_chunk_off turn them into each chunk's
// line-aligned run start per bucket, so the scatter needs no counting pass of its own and no
// cursor atomics (round 2: every chunk counted its items twice and reserved by atomics)
constexpr int kBlkCh = 64;
__global__ void __launch_bounds__(kBlock) k_msd1_hist(const uint64_t *ckeys, const uint32_t *ccnt, uint64_t n, int k,
                                                      uint32_t *cc, unsigned long long *blk) {
    __shared__ uint32_t lc[kMS];
    const uint64_t c0 = (uint64_t)blockIdx.x * kCh1, c1 = c0 + kCh1 < n ? c0 + kCh1 : n;
    for (int i = threadIdx.x; i < kMS; i += kBlock) lc[i] = 0;
    __syncthreads();
    for (uint64_t i = c0 + threadIdx.x; i < c1; i += kBlock) {
        uint32_t bk[2];
        uint64_t it[2];
        const int no = msd_items(ckeys[i], ccnt[i], k, bk, it);
        for (int j = 0; j < no; ++j) atomicAdd(&lc[bk[j]], 1u);
    }
    __syncthreads();
    const uint64_t c = blockIdx.x;
    for (int i = threadIdx.x; i < kMS; i += kBlock) {
        const uint32_t x = lc[i];
        cc[c * kMS + i] = x;
        if (x) atomicAdd(&blk[(c / kBlkCh) * kMS + i], (unsigned long long)(round8(x) / kIL));
    }
}

// per bucket b: exclusive scan of the block line totals over the blocks (in place), total in tot[b]
__global__ void __launch_bounds__(kBlock) k_blk_scan(unsigned long long *blk, uint64_t nblk, uint64_t nb,
                                                     unsigned long long *tot) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    unsigned long long run = 0;
    for (uint64_t j = 0; j < nblk; ++j) {
        const unsigned long long v = blk[j * nb + b];
        blk[j * nb + b] = run;
        run += v;
    }
    tot[b] = run;
}

// chunk run starts (in lines), in place of the chunk counts: chunk c of segment g (a run of
// chunks sharing one set of nb buckets) starts bucket b at base[g * nb + b] + the earlier
// blocks' lines (blk, when given) + the lines of the segment's earlier chunks in its block
__global__ void __launch_bounds__(kBlock) k_chunk_off(uint32_t *cc, uint64_t nch, uint64_t nb,
                                                      const unsigned long long *blk, const unsigned long long *base,
                                                      const uint64_t *seg_first, uint64_t nseg, int base_in_items) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t b = t % nb, q = t / nb;  // q: block (level 1) or segment (level 2)
    uint64_t c0, c1;
    unsigned long long run;
    if (seg_first) {  // level 2: segment q = the chunks of L1 bucket q
        if (q >= nseg) return;
        c0 = seg_first[q];
        c1 = seg_first[q + 1];
        run = base[q * nb + b];
    } else {           // level 1: block q of kBlkCh chunks, one segment
        c0 = q * kBlkCh;
        if (c0 >= nch) return;
        c1 = c0 + kBlkCh < nch ? c0 + kBlkCh : nch;
        run = base[b] + blk[q * nb + b];
    }
    if (base_in_items) run /= kIL;
    for (uint64_t c = c0; c < c1; ++c) {
        const uint32_t x = cc[c * nb + b];
        cc[c * nb + b] = (uint32_t)run;
        run += round8(x) / kIL;
    }
}

// line-buffered placement of one item (see k_l2_scatter in node_counter.hip): the lane that
// completes a buffered line writes it whole; the excess of a round goes directly and is
// copied into the new partial line after the round's flush
struct LinePlace {
    uint64_t *buf;  // [kMS][kIL]
    uint32_t *lb, *lc, *bl;
    uint64_t *out;
    uint64_t gbase;
    __device__ __forceinline__ void put(uint32_t b, uint64_t it, uint32_t &r, uint32_t &line, bool &buffered) {
        r = atomicAdd(&lc[b], 1u);
        line = bl[b];
        buffered = r / kIL == line;
        if (buffered) buf[b * kIL + (r & (kIL - 1))] = it;
        else out[(uint64_t)lb[b] * kIL + r - gbase] = it;
    }
    __device__ __forceinline__ void flush(uint32_t b, uint32_t r, uint32_t line, bool buffered, uint32_t &nline) {
        if (buffered && (r & (kIL - 1)) == kIL - 1) {
            uint64_t *o = out + (((uint64_t)lb[b] + line) * kIL - gbase);
#pragma unroll
            for (int z = 0; z < kIL; ++z) o[z] = buf[b * kIL + z];
        }
        nline = lc[b] / kIL;
        bl[b] = nline;
    }
    // (round 5) the lines completed this round leave the wave cooperatively, as pass B's do
    // (node_counter.hip k_l2_scatter): kIL lanes per line, one 8-B piece each, so one store
    // instruction writes 64 / kIL whole lines instead of each completing lane storing its line in
    // kIL pieces. Called by every lane of the wave (live: the lane has an item here).
    __device__ __forceinline__ void flush_coop(uint32_t b, uint32_t r, uint32_t line, bool live, bool buffered,
                                               uint32_t &nline) {
        const bool done = live && buffered && (r & (kIL - 1)) == kIL - 1;
        const unsigned long long dm = __ballot(done);
        const uint32_t lane = threadIdx.x & 63;
        const uint64_t dst = done ? ((uint64_t)lb[b] + line) * kIL - gbase : 0;
        const uint32_t src = done ? b * kIL : 0;
        const int nd = __popcll(dm);
        for (int b0 = 0; b0 < nd; b0 += 64 / kIL) {
            const int j = b0 + (int)(lane / kIL);  // the line this lane helps write
            int pos = 0;                           // lane holding the j-th set bit of dm
            if (j < nd) {
#pragma unroll
                for (int step = 32; step; step >>= 1) {
                    const unsigned long long below = dm & ((pos + step >= 64) ? ~0ull : ((1ull << (pos + step)) - 1));
                    if (__popcll(below) <= j) pos += step;
                }
            }
            const uint64_t d = __shfl(dst, pos);
            const uint32_t sidx = __shfl(src, pos);
            if (j < nd) out[d + (lane & (kIL - 1))] = buf[sidx + (lane & (kIL - 1))];
        }
        if (live) {
            nline = lc[b] / kIL;
            bl[b] = nline;
        }
    }
    __device__ __forceinline__ void backfill(uint32_t b, uint64_t it, uint32_t r, bool buffered, uint32_t nline) {
        if (!buffered && r / kIL == nline) buf[b * kIL + (r & (kIL - 1))] = it;
    }
    __device__ __forceinline__ void tails(int nb) {
        for (int i = threadIdx.x; i < nb; i += blockDim.x) {
            const uint32_t c = lc[i];
            if (c & (kIL - 1)) {
                uint64_t *o = out + (((uint64_t)lb[i] + c / kIL) * kIL - gbase);
                for (uint32_t z = 0; z < kIL; ++z) o[z] = z < (c & (kIL - 1)) ? buf[i * kIL + z] : kPad;
            }
        }
    }
};

constexpr int kSBlock = 1024;
// rounds of entries in flight in the level-1/2 scatters (MCAAT_SPF). Measured (round 6, C3):
// 1 / 2 / 4 rounds: sdbg_build 36.0 / 39.3 / 37.9 ms, so 1 (profiles/r06_c3_msd_prefetch_ab.txt)
#ifndef MCAAT_SPF
#define MCAAT_SPF 1
#endif
constexpr int kSPF = MCAAT_SPF;

__global__ void __launch_bounds__(kSBlock) k_msd1_scatter(const uint64_t *ckeys, const uint32_t *ccnt, uint64_t n,
                                                          int k, const uint32_t *off, uint64_t *out) {
    __shared__ uint64_t buf[kMS * kIL];
    __shared__ uint32_t lb[kMS], lc[kMS], bl[kMS];
    const uint64_t c0 = (uint64_t)blockIdx.x * kCh1, c1 = c0 + kCh1 < n ? c0 + kCh1 : n;
    for (int i = threadIdx.x; i < kMS; i += kSBlock) {
        lb[i] = off[(uint64_t)blockIdx.x * kMS + i];
        lc[i] = 0;
        bl[i] = 0;
    }
    __syncthreads();
    LinePlace lp{buf, lb, lc, bl, out, 0};
    // the entries of the next kSPF rounds are loaded while this round places its items
    uint64_t na[kSPF];
    uint32_t nc[kSPF];
#pragma unroll
    for (int u = 0; u < kSPF; ++u) {
        const uint64_t i = c0 + (uint64_t)u * kSBlock + threadIdx.x;
        na[u] = i < c1 ? ckeys[i] : 0;
        nc[u] = i < c1 ? ccnt[i] : 0;
    }
    for (uint64_t i00 = c0; i00 < c1; i00 += (uint64_t)kSPF * kSBlock)
#pragma unroll
    for (int u = 0; u < kSPF; ++u) {
        const uint64_t i0 = i00 + (uint64_t)u * kSBlock;
        if (i0 >= c1) break;  // uniform: every thread reaches the same barriers
        const uint64_t i = i0 + threadIdx.x;
        const uint64_t a = na[u];
        const uint32_t cn = nc[u];
        const uint64_t ni = i + (uint64_t)kSPF * kSBlock;
        if (ni < c1) {
            na[u] = ckeys[ni];
            nc[u] = ccnt[ni];
        }
        uint32_t bk[2] = {0, 0}, r[2] = {0, 0}, line[2] = {0, 0}, nl[2] = {0, 0};
        uint64_t it[2] = {0, 0};
        bool bf[2] = {false, false};
        int no = 0;
        if (i < c1) no = msd_items(a, cn, k, bk, it);
        for (int j = 0; j < no; ++j) lp.put(bk[j], it[j], r[j], line[j], bf[j]);
        lds_barrier();
        for (int j = 0; j < 2; ++j) lp.flush_coop(bk[j], r[j], line[j], j < no, bf[j], nl[j]);
        lds_barrier();
        for (int j = 0; j < no; ++j) lp.backfill(bk[j], it[j], r[j], bf[j], nl[j]);
    }
    lds_barrier();
    lp.tails(kMS);
}

// level-2 chunks: [start, start+len) of one level-1 bucket
__device__ __forceinline__ uint32_t msd_sub(uint64_t it, int k) {
    const int E = k + 1;
    return (uint32_t)(it >> (16 + 2 * E - 2 * kMB)) & (kMS - 1);
}

__global__ void __launch_bounds__(kBlock) k_msd2_hist(const uint64_t *in, const uint64_t *cstart, const uint32_t *clen,
                                                      const uint32_t *cbucket, int k, unsigned long long *tot,
                                                      unsigned long long *real, uint32_t *cc) {
    __shared__ uint32_t lc[kMS];
    const uint64_t c = blockIdx.x;
    for (int i = threadIdx.x; i < kMS; i += kBlock) lc[i] = 0;
    __syncthreads();
    const uint64_t s0 = cstart[c];
    const uint32_t n = clen[c];
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) {
        const uint64_t it = in[s0 + i];
        if (it != kPad) atomicAdd(&lc[msd_sub(it, k)], 1u);
    }
    __syncthreads();
    const uint64_t fb = (uint64_t)cbucket[c] * kMS;
    for (int i = threadIdx.x; i < kMS; i += kBlock) {
        cc[c * kMS + i] = lc[i];
        if (lc[i]) {
            atomicAdd(&tot[fb + i], (unsigned long long)round8(lc[i]));
            atomicAdd(&real[fb + i], (unsigned long long)lc[i]);
        }
    }
}

__global__ void __launch_bounds__(kSBlock) k_msd2_scatter(const uint64_t *in, const uint64_t *cstart,
                                                          const uint32_t *clen, const uint32_t *off, int k,
                                                          uint64_t *out) {
    __shared__ uint64_t buf[kMS * kIL];
    __shared__ uint32_t lb[kMS], lc[kMS], bl[kMS];
    const uint64_t c = blockIdx.x;
    for (int i = threadIdx.x; i < kMS; i += kSBlock) {
        lb[i] = off[c * kMS + i];
        lc[i] = 0;
        bl[i] = 0;
    }
    __syncthreads();
    const uint64_t s0 = cstart[c];
    const uint32_t n = clen[c];
    LinePlace lp{buf, lb, lc, bl, out, 0};
    uint64_t nxt[kSPF];
#pragma unroll
    for (int u = 0; u < kSPF; ++u) {
        const uint32_t i = (uint32_t)u * kSBlock + threadIdx.x;
        nxt[u] = i < n ? in[s0 + i] : kPad;
    }
    for (uint32_t i00 = 0; i00 < n; i00 += (uint32_t)kSPF * kSBlock)
#pragma unroll
    for (int u = 0; u < kSPF; ++u) {
        const uint32_t i0 = i00 + (uint32_t)u * kSBlock;
        if (i0 >= n) break;  // uniform
        const uint64_t it = nxt[u];
        const uint32_t ni = i0 + (uint32_t)kSPF * kSBlock + threadIdx.x;
        nxt[u] = ni < n ? in[s0 + ni] : kPad;
        const bool live = it != kPad;
        uint32_t b = 0, r = 0, line = 0, nl = 0;
        bool bf = false;
        if (live) {
            b = msd_sub(it, k);
            lp.put(b, it, r, line, bf);
        }
        lds_barrier();
        lp.flush_coop(b, r, line, live, bf, nl);
        lds_barrier();
        if (live) lp.backfill(b, it, r, bf, nl);
    }
    lds_barrier();
    lp.tails(kMS);
}

// bitonic sort of P (power of two) items in LDS by `nth` threads starting at thread t0
__device__ __forceinline__ void lds_bitonic(uint64_t *s, uint32_t P, uint32_t t, uint32_t nth, bool wave_only) {
    for (uint32_t kk = 2; kk <= P; kk <<= 1)
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            for (uint32_t q = t; q < P / 2; q += nth) {
                const uint32_t i = ((q & ~(j - 1)) << 1) | (q & (j - 1)), l = i + j;
                const uint64_t a = s[i], b = s[l];
                if ((a > b) == ((i & kk) == 0)) {
                    s[i] = b;
                    s[l] = a;
                }
            }
            if (wave_only) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            } else {
                lds_barrier();
            }
        }
}

__device__ __forceinline__ void msd_emit(const uint64_t *s, uint32_t nreal, uint32_t t, uint32_t nth, uint64_t hi,
                                         uint64_t *key, uint16_t *mult, uint64_t base) {
    for (uint32_t i = t; i < nreal; i += nth) {
        const uint64_t it = s[i];
        key[base + i] = hi | (it >> 16);
        mult[base + i] = (uint16_t)(it & 0xFFFF);
    }
}

// one wave per level-2 bucket of <= kWaveSort items; larger ones are listed. A bucket is
// counting-sorted by the next lg(P) key bits (P = its size rounded up to a power of two, so
// about one item per bin): each item's rank inside its bin comes from the LDS histogram atomic,
// a wave scan turns counts into bin starts, items go from registers to their bins in LDS, and
// each then finds its final rank among the few items of its own bin and is written straight to
// HBM (ranks are nearly the LDS order, so the writes stay coalesced). A bucket whose largest
// bin holds more than kMaxBin items (clustered keys) takes the bitonic network instead.
// The items stay in the registers they were loaded into until they are placed (padding is
// skipped, never compacted), so a wave holds 6 KB of LDS and five workgroups share a CU (the
// register limit at 96).
constexpr int kL3Waves = 4;
constexpr uint32_t kMaxBin = 16;
__global__ void __launch_bounds__(kL3Waves * 64) __attribute__((amdgpu_waves_per_eu(5))) k_msd3_wave(const uint64_t *in, const uint64_t *off2,
                                                             const uint64_t *real2, const uint64_t *base3, int k,
                                                             uint64_t *key, uint16_t *mult, uint32_t *big,
                                                             unsigned long long *nbig, uint32_t limit, int counting) {
    __shared__ uint64_t so[kL3Waves][kWaveSort];
    __shared__ uint32_t sc[kL3Waves][kWaveSort];
    // buckets above the limit are listed 64 at a time per wave (one cursor atomic per 64: at
    // C5 ~3M of the 4M buckets are listed, and one atomic each on a single counter took 50 ms);
    // lane j holds the j-th pending bucket in a register
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t npend = 0, mypend = 0;
    auto flush_pend = [&]() {
        unsigned long long at = 0;
        if (lane == 0) at = atomicAdd(nbig, (unsigned long long)npend);
        at = __shfl(at, 0);
        if ((uint32_t)lane < npend) big[at + lane] = mypend;
        npend = 0;
    };
    uint64_t *o = so[wave];
    uint32_t *cnt = sc[wave];
    const int E = k + 1;
    const int rb = 2 * E - 2 * kMB;  // key bits below the two MSD levels (item bits 16 .. 16 + rb)
    const uint64_t nb = (uint64_t)kMS * kMS;
    const uint64_t bstride = (uint64_t)gridDim.x * kL3Waves;
    constexpr int NL = 10;  // loads per lane: buckets of up to 640 padded items
    constexpr int NR = kWaveSort / 64;  // sorted items per lane
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    uint64_t b = (uint64_t)blockIdx.x * kL3Waves + wave;
    // bucket metadata one bucket ahead
    uint64_t m_lo = 0, m_hi = 0, m_real = 0, m_base = 0;
    if (b < nb) {
        m_lo = off2[b];
        m_hi = off2[b + 1];
        m_real = real2[b];
        m_base = base3[b];
    }
    for (; b < nb; b += bstride) {
        const uint64_t lo = m_lo, n = m_hi - m_lo, nr64 = m_real, base = m_base;
        const uint64_t bn = b + bstride;
        if (bn < nb) {
            m_lo = off2[bn];
            m_hi = off2[bn + 1];
            m_real = real2[bn];
            m_base = base3[bn];
        }
        if (n == 0) continue;
        if (nr64 > (uint64_t)limit || n > (uint64_t)NL * 64) {
            if ((uint32_t)lane == npend) mypend = (uint32_t)b;
            if (++npend == 64) flush_pend();
            continue;
        }
        // load the bucket (all loads in flight together); line padding is kPad
        const uint32_t nreal = (uint32_t)nr64;
        uint64_t v[NL];
#pragma unroll
        for (int t = 0; t < NL; ++t) {
            const uint32_t i = t * 64 + lane;
            v[t] = i < n ? in[lo + i] : kPad;
        }
        const uint64_t hi = (b >> kMB) << (2 * E - kMB);
        // bins: P >= nreal, at least 64 (one per lane), at most 2^rb
        uint32_t lgb = 6;
        while ((1u << lgb) < nreal) ++lgb;
        bool sorted = false;
        if (counting && lgb <= (uint32_t)rb) {
            const uint32_t nbins = 1u << lgb, per = nbins / 64, sh = 16 + rb - lgb;
            for (uint32_t i = lane; i < nbins; i += 64) cnt[i] = 0;
            wave_sync();
            uint32_t rk[NL];
#pragma unroll
            for (int t = 0; t < NL; ++t)
                rk[t] = v[t] != kPad ? atomicAdd(&cnt[(uint32_t)(v[t] >> sh) & (nbins - 1)], 1u) : 0;
            wave_sync();
            // bin counts -> bin starts (each lane owns `per` consecutive bins)
            uint32_t loc = 0, mx = 0;
            for (uint32_t j = 0; j < per; ++j) {
                const uint32_t c = cnt[lane * per + j];
                loc += c;
                mx = c > mx ? c : mx;
            }
            uint32_t incl = loc;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t u = __shfl_up(incl, d);
                if (lane >= d) incl += u;
            }
            for (int d = 32; d > 0; d >>= 1) {
                const uint32_t u = __shfl_xor(mx, d);
                mx = u > mx ? u : mx;
            }
            if (mx <= kMaxBin) {
                uint32_t run = incl - loc;
                for (uint32_t j = 0; j < per; ++j) {
                    const uint32_t c = cnt[lane * per + j];
                    cnt[lane * per + j] = run;
                    run += c;
                }
                wave_sync();
#pragma unroll
                for (int t = 0; t < NL; ++t)
                    if (v[t] != kPad) o[cnt[(uint32_t)(v[t] >> sh) & (nbins - 1)] + rk[t]] = v[t];
                wave_sync();
#pragma unroll
                for (int t = 0; t < NR; ++t) {
                    const uint32_t p = t * 64 + lane;
                    if (p < nreal) {
                        const uint64_t x = o[p];
                        const uint32_t bi = (uint32_t)(x >> sh) & (nbins - 1);
                        const uint32_t bs = cnt[bi], be = bi + 1 < nbins ? cnt[bi + 1] : nreal;
                        uint32_t r = bs;
                        for (uint32_t q = bs; q < be; ++q) r += o[q] < x;
                        key[base + r] = hi | (x >> 16);
                        mult[base + r] = (uint16_t)(x & 0xFFFF);
                    }
                }
                sorted = true;
            }
        }
        if (!sorted) {  // the items compacted into LDS, padded to a power of two, bitonic network
            uint32_t fill = 0;
#pragma unroll
            for (int t = 0; t < NL; ++t) {
                const unsigned long long m = __ballot(v[t] != kPad);
                if (v[t] != kPad)
                    o[fill + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] = v[t];
                fill += (uint32_t)__popcll(m);
            }
            uint32_t P = 8;
            while (P < nreal) P <<= 1;
            for (uint32_t i = nreal + lane; i < P; i += 64) o[i] = kPad;
            wave_sync();
            lds_bitonic(o, P, lane, 64, true);
            msd_emit(o, nreal, lane, 64, hi, key, mult, base);
        }
        wave_sync();
    }
    if (npend) flush_pend();
}

// k_msd3_wave's counting sort for the listed buckets above the one-wave limit (deep graphs:
// D / 2^22 above 512 items, C2 ~570, C5 ~935): one THREADS-thread workgroup per bucket of
// <= CAP items. Items are binned by the next lg(P) key bits (LDS histogram atomics give each
// item a slot in its bin; their order does not matter, as each item's final rank is its bin
// start plus the number of smaller items in its bin), the bin counts are scanned by the
// workgroup, items move to their bins and are written straight to HBM at their final ranks. A bucket whose largest bin holds more than kMaxBin items
// (clustered keys) is sorted by the bitonic network instead. Larger buckets are forwarded.
// Round 3: a bucket's metadata and items are loaded into registers while the previous bucket
// is sorted (all CAP / THREADS loads of a thread in flight together, LDS-only barriers so the
// sort does not drain them; round 2 loaded each 256-item round after the last had landed), and
// the items go from those registers straight to their bins (padding skipped, no compaction
// buffer): 24 KB of LDS, four workgroups per CU (the registers).
template <int THREADS, int CAP, int OCC>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(OCC))) k_msd3_count(const uint64_t *in, const uint64_t *off2, const uint64_t *real2,
                                                        const uint64_t *base3, int k, const uint32_t *big, uint64_t nbig,
                                                        uint64_t *key, uint16_t *mult, uint32_t *fwd,
                                                        unsigned long long *nfwd, uint32_t limit) {
    static_assert(CAP % THREADS == 0 && CAP >= THREADS && THREADS % 64 == 0, "bins per thread");
    constexpr int NW = THREADS / 64, NR = CAP / THREADS;
    __shared__ uint64_t o[CAP];
    __shared__ uint32_t cnt[CAP];
    __shared__ uint32_t wsum[NW], wfill[NW], wmax[NW];
    const int E = k + 1;
    const int rb = 2 * E - 2 * kMB;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t v[NR];
    uint64_t f_b = 0, f_lo = 0, f_n = 0;
    uint32_t f_real = 0;
    bool f_ok = false;
    auto fetch = [&](uint64_t q) {
        f_ok = false;
        f_n = 0;
        if (q < nbig) {
            f_b = big[q];
            f_lo = off2[f_b];
            f_n = off2[f_b + 1] - f_lo;
            f_real = (uint32_t)real2[f_b];
            f_ok = f_n <= (uint64_t)CAP && f_real <= limit;
        }
#pragma unroll
        for (int t = 0; t < NR; ++t) {
            const uint32_t i = t * THREADS + threadIdx.x;
            v[t] = f_ok && i < f_n ? in[f_lo + i] : kPad;
        }
    };
    fetch(blockIdx.x);
    for (uint64_t q = blockIdx.x; q < nbig; q += gridDim.x) {
        const uint64_t b = f_b;
        const uint32_t nreal = f_real;
        if (!f_ok) {
            if (threadIdx.x == 0) fwd[atomicAdd(nfwd, 1ull)] = (uint32_t)b;
            fetch(q + gridDim.x);
            continue;
        }
        const uint64_t base = base3[b], hi = (b >> kMB) << (2 * E - kMB);
        uint64_t x[NR];
#pragma unroll
        for (int t = 0; t < NR; ++t) x[t] = v[t];
        uint32_t lgb = 0;
        while ((1u << lgb) < (uint32_t)THREADS) ++lgb;  // at least one bin per thread
        while ((1u << lgb) < nreal) ++lgb;
        const bool counting = lgb <= (uint32_t)rb;
        const uint32_t nbins = 1u << lgb, per = nbins / THREADS, sh = counting ? 16 + rb - lgb : 0;
        lds_barrier();  // B1: every thread is past the previous bucket (o and cnt free)
        if (counting)
            for (uint32_t i = threadIdx.x; i < nbins; i += THREADS) cnt[i] = 0;
        fetch(q + gridDim.x);  // the next bucket's loads overlap this one's sort
        lds_barrier();  // B2: bins cleared
        bool done = false;
        if (counting) {
            uint32_t rk[NR];
#pragma unroll
            for (int t = 0; t < NR; ++t)
                rk[t] = x[t] != kPad ? atomicAdd(&cnt[(uint32_t)(x[t] >> sh) & (nbins - 1)], 1u) : 0;
            lds_barrier();  // B3: histogram complete
            uint32_t loc = 0, mx = 0;
            for (uint32_t j = 0; j < per; ++j) {
                const uint32_t c = cnt[threadIdx.x * per + j];
                loc += c;
                mx = c > mx ? c : mx;
            }
            uint32_t incl = loc;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t u = __shfl_up(incl, d);
                if (lane >= d) incl += u;
            }
            for (int d = 32; d > 0; d >>= 1) {
                const uint32_t u = __shfl_xor(mx, d);
                mx = u > mx ? u : mx;
            }
            if (lane == 63) wsum[wave] = incl;
            if (lane == 0) wmax[wave] = mx;
            lds_barrier();  // B4: per-wave sums and maxima
            uint32_t gmx = 0;
            for (int w = 0; w < NW; ++w) gmx = wmax[w] > gmx ? wmax[w] : gmx;
            if (gmx <= kMaxBin) {
                uint32_t run = incl - loc;
                for (int w = 0; w < wave; ++w) run += wsum[w];
                for (uint32_t j = 0; j < per; ++j) {
                    const uint32_t c = cnt[threadIdx.x * per + j];
                    cnt[threadIdx.x * per + j] = run;
                    run += c;
                }
                lds_barrier();  // B5: bin starts
#pragma unroll
                for (int t = 0; t < NR; ++t)
                    if (x[t] != kPad) o[cnt[(uint32_t)(x[t] >> sh) & (nbins - 1)] + rk[t]] = x[t];
                lds_barrier();  // B6: items in their bins
#pragma unroll
                for (int t = 0; t < NR; ++t) {
                    const uint32_t p = t * THREADS + threadIdx.x;
                    if (p < nreal) {
                        const uint64_t y = o[p];
                        const uint32_t bi = (uint32_t)(y >> sh) & (nbins - 1);
                        const uint32_t bs = cnt[bi], be = bi + 1 < nbins ? cnt[bi + 1] : nreal;
                        uint32_t r = bs;
                        for (uint32_t z = bs; z < be; ++z) r += o[z] < y;
                        key[base + r] = hi | (y >> 16);
                        mult[base + r] = (uint16_t)(y & 0xFFFF);
                    }
                }
                done = true;
            }
        }
        if (!done) {  // clustered keys: the items compacted into LDS, then the bitonic network
            unsigned long long m[NR];
            uint32_t wc = 0;
#pragma unroll
            for (int t = 0; t < NR; ++t) {
                m[t] = __ballot(x[t] != kPad);
                wc += (uint32_t)__popcll(m[t]);
            }
            if (lane == 0) wfill[wave] = wc;
            lds_barrier();
            uint32_t at = 0;
            for (int w = 0; w < wave; ++w) at += wfill[w];
#pragma unroll
            for (int t = 0; t < NR; ++t) {
                if (x[t] != kPad)
                    o[at + __builtin_amdgcn_mbcnt_hi((uint32_t)(m[t] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m[t], 0))] = x[t];
                at += (uint32_t)__popcll(m[t]);
            }
            uint32_t P = 8;
            while (P < nreal) P <<= 1;
            for (uint32_t i = nreal + threadIdx.x; i < P; i += THREADS) o[i] = kPad;
            lds_barrier();
            lds_bitonic(o, P, threadIdx.x, THREADS, false);
            msd_emit(o, nreal, threadIdx.x, THREADS, hi, key, mult, base);
        }
        // no trailing barrier: the next bucket writes LDS only after its B1
    }
}

// one workgroup per listed level-3 bucket of <= CAP items; larger ones are forwarded to the
// next list (or flagged when there is none: the caller falls back to the radix sort)
template <int THREADS, int CAP>
__global__ void __launch_bounds__(THREADS) k_msd3_block(const uint64_t *in, const uint64_t *off2, const uint64_t *real2,
                                                        const uint64_t *base3, int k, const uint32_t *big, uint64_t nbig,
                                                        uint64_t *key, uint16_t *mult, uint32_t *fwd,
                                                        unsigned long long *nfwd, int *too_big, uint32_t limit) {
    __shared__ uint64_t s[CAP];
    const int E = k + 1;
    for (uint64_t q = blockIdx.x; q < nbig; q += gridDim.x) {
        const uint64_t b = big[q], lo = off2[b], n = off2[b + 1] - lo;
        if (n > (uint64_t)CAP || n > (uint64_t)limit) {
            if (threadIdx.x == 0) {
                if (fwd) fwd[atomicAdd(nfwd, 1ull)] = (uint32_t)b;
                else *too_big = 1;
            }
            continue;
        }
        uint32_t P = 8;
        while (P < n) P <<= 1;
        for (uint32_t i = threadIdx.x; i < P; i += THREADS) s[i] = i < n ? in[lo + i] : kPad;
        __syncthreads();
        lds_bitonic(s, P, threadIdx.x, THREADS, false);
        const uint64_t hi = (b >> kMB) << (2 * E - kMB);
        msd_emit(s, (uint32_t)real2[b], threadIdx.x, THREADS, hi, key, mult, base3[b]);
        __syncthreads();
    }
}

template <class T>
void excl_scan(hipStream_t st, const T *in, T *out, uint64_t n) {
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, (size_t)n, st));
    DevBuf<uint8_t> t(tmp);
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(t.p, tmp, in, out, (size_t)n, st));
}

// returns false (nothing written) if a bucket exceeds the LDS sorts: caller uses the radix sort
bool msd_sort(mcaat_ctx *ctx, const uint64_t *ckeys, const uint32_t *ccnt, uint64_t n, int k, uint64_t D,
              uint64_t *key, uint16_t *mult) {
    hipStream_t st = ctx->stream;
    const uint64_t nch1 = (n + kCh1 - 1) / kCh1;
    // level 1: per-chunk counts -> per-block line totals -> bucket bases -> chunk run starts
    const uint64_t nblk1 = (nch1 + kBlkCh - 1) / kBlkCh;
    DevBuf<uint32_t> cc1(nch1 * kMS ? nch1 * kMS : 1);
    DevBuf<unsigned long long> blk1(nblk1 * kMS ? nblk1 * kMS : 1), tot1(kMS + 1), base1(kMS + 1);
    HIP_OK(hipMemsetAsync(blk1.p, 0, blk1.bytes(), st));
    HIP_OK(hipMemsetAsync(tot1.p, 0, tot1.bytes(), st));
    hipLaunchKernelGGL(k_msd1_hist, dim3((unsigned)nch1), dim3(kBlock), 0, st, ckeys, ccnt, n, k, cc1.p, blk1.p);
    LAUNCH_OK();
    hipLaunchKernelGGL(k_blk_scan, dim3(grid_for(kMS, kBlock)), dim3(kBlock), 0, st, blk1.p, nblk1, (uint64_t)kMS,
                       tot1.p);
    LAUNCH_OK();
    excl_scan(st, (const uint64_t *)tot1.p, (uint64_t *)base1.p, kMS + 1);  // in lines
    hipLaunchKernelGGL(k_chunk_off, dim3(grid_for(nblk1 * kMS, kBlock)), dim3(kBlock), 0, st, cc1.p, nch1,
                       (uint64_t)kMS, (const unsigned long long *)blk1.p, (const unsigned long long *)base1.p,
                       (const uint64_t *)nullptr, (uint64_t)0, 0);
    LAUNCH_OK();
    std::vector<uint64_t> off1(kMS + 1);
    HIP_OK(hipMemcpyAsync(off1.data(), base1.p, 8 * (kMS + 1), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    for (auto &x : off1) x *= kIL;  // lines -> items
    DevBuf<uint64_t> l1(off1[kMS] ? off1[kMS] : 1);
    hipLaunchKernelGGL(k_msd1_scatter, dim3((unsigned)nch1), dim3(kSBlock), 0, st, ckeys, ccnt, n, k,
                       (const uint32_t *)cc1.p, l1.p);
    LAUNCH_OK();
    blk1.release();
    // level 2: chunks of each level-1 bucket (consecutive), per-chunk sub counts
    std::vector<uint64_t> cstart, seg_first(kMS + 1);
    std::vector<uint32_t> clen, cbk;
    for (int b = 0; b < kMS; ++b) {
        seg_first[b] = cstart.size();
        for (uint64_t o = off1[b]; o < off1[b + 1]; o += kCh2) {
            cstart.push_back(o);
            clen.push_back((uint32_t)std::min<uint64_t>(kCh2, off1[b + 1] - o));
            cbk.push_back((uint32_t)b);
        }
    }
    seg_first[kMS] = cstart.size();
    const uint64_t nch2 = cstart.size(), NB = (uint64_t)kMS * kMS;
    DevBuf<uint64_t> dcs(nch2 ? nch2 : 1), dseg(kMS + 1);
    DevBuf<uint32_t> dcl(nch2 ? nch2 : 1), dcb(nch2 ? nch2 : 1), cc2(nch2 * kMS ? nch2 * kMS : 1);
    DevBuf<unsigned long long> tot2(NB + 1), real2(NB + 1), cur2(NB + 1), base3(NB + 1);
    HIP_OK(hipMemcpyAsync(dcs.p, cstart.data(), 8 * nch2, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(dcl.p, clen.data(), 4 * nch2, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(dcb.p, cbk.data(), 4 * nch2, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(dseg.p, seg_first.data(), 8 * (kMS + 1), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(tot2.p, 0, tot2.bytes(), st));
    HIP_OK(hipMemsetAsync(real2.p, 0, real2.bytes(), st));
    if (nch2) {
        hipLaunchKernelGGL(k_msd2_hist, dim3((unsigned)nch2), dim3(kBlock), 0, st, l1.p, dcs.p, dcl.p, dcb.p, k,
                           tot2.p, real2.p, cc2.p);
        LAUNCH_OK();
    }
    excl_scan(st, (const uint64_t *)tot2.p, (uint64_t *)cur2.p, NB + 1);
    excl_scan(st, (const uint64_t *)real2.p, (uint64_t *)base3.p, NB + 1);
    uint64_t n2 = 0, nreal = 0;
    HIP_OK(hipMemcpyAsync(&n2, cur2.p + NB, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(&nreal, base3.p + NB, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (nreal != D) throw Error(MCAAT_E_CAPACITY, "msd_sort: item count mismatch");
    if (n2 / kIL >= (1ull << 32)) throw Error(MCAAT_E_CAPACITY, "msd_sort: 2^32 or more lines");
    DevBuf<uint64_t> off2(NB + 1);
    HIP_OK(hipMemcpyAsync(off2.p, cur2.p, 8 * (NB + 1), hipMemcpyDeviceToDevice, st));
    DevBuf<uint64_t> l2(n2 ? n2 : 1);
    if (nch2) {
        hipLaunchKernelGGL(k_chunk_off, dim3(grid_for(NB, kBlock)), dim3(kBlock), 0, st, cc2.p, nch2, (uint64_t)kMS,
                           (const unsigned long long *)nullptr, (const unsigned long long *)cur2.p,
                           (const uint64_t *)dseg.p, (uint64_t)kMS, 1);
        LAUNCH_OK();
        hipLaunchKernelGGL(k_msd2_scatter, dim3((unsigned)nch2), dim3(kSBlock), 0, st, l1.p, dcs.p, dcl.p,
                           (const uint32_t *)cc2.p, k, l2.p);
        LAUNCH_OK();
    }
    l1.release();
    // level 3
    DevBuf<uint32_t> big(NB);
    DevBuf<unsigned long long> nbig(1);
    DevBuf<int> too(1);
    HIP_OK(hipMemsetAsync(nbig.p, 0, 8, st));
    HIP_OK(hipMemsetAsync(too.p, 0, 4, st));
    // 24 KB of LDS per workgroup, 96 registers: five resident per CU
    hipLaunchKernelGGL(k_msd3_wave, dim3((unsigned)ctx->n_cu * 5), dim3(kL3Waves * 64), 0, st, l2.p, off2.p,
                       (const uint64_t *)real2.p, (const uint64_t *)base3.p, k, key, mult, big.p, nbig.p,
                       (uint32_t)std::min<int64_t>(kWaveSort, knob(ctx, "sort.wave_limit", kWaveSort)),
                       (int)knob(ctx, "sort.l3_counting", 1));
    LAUNCH_OK();
    unsigned long long hb = 0;
    HIP_OK(hipMemcpyAsync(&hb, nbig.p, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (hb) {
        // mid-size buckets (deep graphs: D / 2^22 above the wave limit) by 256-thread
        // workgroups, many per CU; the rare larger ones by one 1024-thread workgroup each
        DevBuf<uint32_t> big2(hb);
        DevBuf<unsigned long long> nbig2(1);
        HIP_OK(hipMemsetAsync(nbig2.p, 0, 8, st));
        const uint32_t mid_limit = (uint32_t)std::min<int64_t>(kMidSort, knob(ctx, "sort.mid_limit", kMidSort));
        // buckets of <= 1024 items by 128-thread workgroups first (12 KB of LDS, two-wave
        // barriers, eight resident per CU), the larger ones forwarded; by default only where the
        // average level-3 bucket is small enough for that stage to take most of them (C2: D / 2^22
        // ~ 570, sdbg_build 97.4 -> 92.8 ms; C5 ~ 935: 152.8 -> 179.6, so not there)
        const int64_t small_knob = knob(ctx, "sort.small_mid", -1);
        const bool small = small_knob >= 0 ? small_knob != 0 : D / NB <= 768;
        if (small && knob(ctx, "sort.mid_counting", 1) && mid_limit >= kSmallMid) {
            DevBuf<uint32_t> big1(hb);
            DevBuf<unsigned long long> nbig1(1);
            HIP_OK(hipMemsetAsync(nbig1.p, 0, 8, st));
            hipLaunchKernelGGL((k_msd3_count<128, kSmallMid, 4>), dim3((unsigned)std::min<uint64_t>(hb, (uint64_t)ctx->n_cu * 8)),
                               dim3(128), 0, st, l2.p, off2.p, (const uint64_t *)real2.p, (const uint64_t *)base3.p, k,
                               big.p, (uint64_t)hb, key, mult, big1.p, nbig1.p,
                               (uint32_t)std::min<int64_t>(kSmallMid, knob(ctx, "sort.small_limit", kSmallMid)));
            LAUNCH_OK();
            HIP_OK(hipMemcpyAsync(&hb, nbig1.p, 8, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            HIP_OK(hipMemcpyAsync(big.p, big1.p, 4 * hb, hipMemcpyDeviceToDevice, st));
        }
        if (!hb) {
            // every listed bucket was sorted above
        } else if (knob(ctx, "sort.mid_counting", 1)) {
            // 24 KB of LDS per workgroup; the registers (125) allow four per CU (`sort.mid_occ=5`: five, at 96 registers with spills; C2 2 ms slower)
            if (knob(ctx, "sort.mid_occ", 4) >= 5)
                hipLaunchKernelGGL((k_msd3_count<256, kMidSort, 5>), dim3((unsigned)std::min<uint64_t>(hb, (uint64_t)ctx->n_cu * 5)),
                                   dim3(256), 0, st, l2.p, off2.p, (const uint64_t *)real2.p, (const uint64_t *)base3.p, k,
                                   big.p, (uint64_t)hb, key, mult, big2.p, nbig2.p, mid_limit);
            else
                hipLaunchKernelGGL((k_msd3_count<256, kMidSort, 4>), dim3((unsigned)std::min<uint64_t>(hb, (uint64_t)ctx->n_cu * 4)),
                                   dim3(256), 0, st, l2.p, off2.p, (const uint64_t *)real2.p, (const uint64_t *)base3.p, k,
                                   big.p, (uint64_t)hb, key, mult, big2.p, nbig2.p, mid_limit);
        } else {
            hipLaunchKernelGGL((k_msd3_block<256, kMidSort>), dim3((unsigned)std::min<uint64_t>(hb, (uint64_t)ctx->n_cu * 8)),
                               dim3(256), 0, st, l2.p, off2.p, (const uint64_t *)real2.p, (const uint64_t *)base3.p, k,
                               big.p, (uint64_t)hb, key, mult, big2.p, nbig2.p, too.p, mid_limit);
        }
        LAUNCH_OK();
        unsigned long long hb2 = 0;
        HIP_OK(hipMemcpyAsync(&hb2, nbig2.p, 8, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        if (hb2) {
            hipLaunchKernelGGL((k_msd3_block<1024, kBlockSort>), dim3((unsigned)std::min<uint64_t>(hb2, (uint64_t)ctx->n_cu)),
                               dim3(1024), 0, st, l2.p, off2.p, (const uint64_t *)real2.p, (const uint64_t *)base3.p, k,
                               big2.p, (uint64_t)hb2, key, mult, (uint32_t *)nullptr,
                               (unsigned long long *)nullptr, too.p,
                               (uint32_t)std::min<int64_t>(kBlockSort, knob(ctx, "sort.block_limit", kBlockSort)));
            LAUNCH_OK();
        }
        int h = 0;
        HIP_OK(hipMemcpyAsync(&h, too.p, 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        if (h) return false;
    }
    HIP_OK(hipStreamSynchronize(st));
    return true;
}

}  // namespace

void sdbg_build(mcaat_ctx *ctx, CountResult &c, int k, mcaat_graph *g) {
    hipStream_t st = ctx->stream;
    const int E = k + 1;
    const uint64_t n2 = 2 * c.n;
    g->k = k;
    DevBuf<unsigned long long> npal(1);
    HIP_OK(hipMemsetAsync(npal.p, 0, 8, st));
    if (c.n) {
        hipLaunchKernelGGL(k_count_pal, dim3(grid_for(c.n, kBlock, (unsigned)ctx->n_cu * 16)), dim3(kBlock), 0, st,
                           c.keys.p, c.n, k, npal.p);
        LAUNCH_OK();
    }
    unsigned long long n_pal = 0;
    HIP_OK(hipMemcpyAsync(&n_pal, npal.p, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    const uint64_t D = n2 - n_pal;
    g->D = D;
    g->key.alloc(D ? D : 1);
    g->mult.alloc(mcaat_graph::mult_entries(D));
    // MSD sort with LDS bucket sorts (k <= 28: key remainder and mult share one word);
    // the radix sort otherwise, or when a bucket is too skewed for LDS
    bool done = false;
    const int64_t msd = knob(ctx, "sort.msd", -1);  // test knob: 0 never, 1 whenever k <= 28
    if (k <= 28 && msd != 0 && (D >= (1u << 16) || (msd == 1 && D > 0))) {
        KernelTimer kt(ctx, "edge_sort", 64.0 * (double)D);
        done = msd_sort(ctx, c.keys.p, c.counts.p, c.n, k, D, g->key.p, g->mult.p);
        kt.stop();
    }
    if (!done && n2) {
        DevBuf<uint64_t> ek(n2);
        DevBuf<uint16_t> em(n2);
        HIP_OK(hipMemsetAsync(npal.p, 0, 8, st));
        hipLaunchKernelGGL(k_expand, dim3(grid_for(c.n, kBlock)), dim3(kBlock), 0, st, c.keys.p, c.counts.p, c.n, k,
                           ek.p, em.p, npal.p);
        LAUNCH_OK();
        DevBuf<uint64_t> sk(n2);
        DevBuf<uint16_t> sm(n2);
        size_t tmp = 0;
        HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, ek.p, sk.p, em.p, sm.p, (size_t)n2, 0, 2 * E + 1, st));
        DevBuf<uint8_t> t(tmp);
        HIP_OK(hipcub::DeviceRadixSort::SortPairs(t.p, tmp, ek.p, sk.p, em.p, sm.p, (size_t)n2, 0, 2 * E + 1, st));
        // palindromes left sentinels (1 << 2E) at the end
        if (D) {
            HIP_OK(hipMemcpyAsync(g->key.p, sk.p, 8 * D, hipMemcpyDeviceToDevice, st));
            HIP_OK(hipMemcpyAsync(g->mult.p, sm.p, 2 * D, hipMemcpyDeviceToDevice, st));
        }
        HIP_OK(hipStreamSynchronize(st));
    }
    c.keys.release();
    c.counts.release();
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
    DevBuf<uint64_t> &dir = g->dir;
    dir.alloc(nprefix + 1);
    g->dir_shift = shift;
    {
        DevBuf<int> bad(1);
        HIP_OK(hipMemsetAsync(bad.p, 0, sizeof(int), st));
        const uint64_t key_lim = E >= 32 ? ~0ULL : 1ULL << (2 * E);
        hipLaunchKernelGGL(k_dir, dim3(grid_for((D + kDirU) / kDirU, kBlock, (unsigned)ctx->n_cu * 16)), dim3(kBlock), 0,
                           st, g->key.p, D, shift, nprefix, key_lim, dir.p, bad.p);
        LAUNCH_OK();
        int hb = 0;
        d2h(ctx, &hb, bad.p, sizeof(int));
        if (hb) throw Error(MCAAT_E_INVALID, "sdbg: edge keys are not strictly ascending below 4^(k+1)");
    }
    g->out_info.alloc(D);
    g->in_info.alloc(D);
    if (D) {
        KernelTimer kt(ctx, "adjacency", 32.0 * (double)D);  // key read, in_info cleared, two words written
        // one edge per lane: neighbouring lanes search neighbouring key ranges, so the
        // searches' loads share lines across the wave (a thread-per-run merge walk that
        // loses this was 5x slower)
        const int64_t adj = knob(ctx, "sdbg.adj_lds", 1);  // 1: owner-side runs, 2: round-2 LDS runs, 0: global search
        if (adj == 1) {
            const uint32_t cap = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(kOwnCap, knob(ctx, "sdbg.adj_cap", kOwnCap)));
            const uint64_t nruns = (D + kOwnB - 1) / kOwnB;
            DevBuf<uint64_t> bounds(5 * (nruns + 1));
            hipLaunchKernelGGL(k_own_bounds, dim3(grid_for(nruns + 1, kBlock)), dim3(kBlock), 0, st, g->key.p, D, k,
                               dir.p, shift, nruns, bounds.p);
            LAUNCH_OK();
            hipLaunchKernelGGL(k_adjacency_own, dim3((unsigned)nruns), dim3(kOwnT), 0, st, g->key.p, D, k, dir.p, shift,
                               cap, (const uint64_t *)bounds.p, g->out_info.p, g->in_info.p);
        } else if (adj == 2) {
            HIP_OK(hipMemsetAsync(g->in_info.p, 0, 8 * D, st));
            const uint32_t cap = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(kAdjCap, knob(ctx, "sdbg.adj_cap", kAdjCap)));
            const uint64_t nruns = (D + kAdjB - 1) / kAdjB;
            DevBuf<uint64_t> bounds(8 * nruns);
            hipLaunchKernelGGL(k_adj_bounds, dim3(grid_for(4 * nruns, kBlock, (unsigned)ctx->n_cu * 16)), dim3(kBlock), 0,
                               st, g->key.p, D, k, dir.p, shift, nruns, bounds.p);
            LAUNCH_OK();
            hipLaunchKernelGGL(k_adjacency_lds, dim3((unsigned)nruns), dim3(kAdjT), 0, st, g->key.p, D, k, dir.p, shift,
                               cap, (const uint64_t *)bounds.p, g->out_info.p, g->in_info.p);
        } else {
            HIP_OK(hipMemsetAsync(g->in_info.p, 0, 8 * D, st));
            hipLaunchKernelGGL(k_adjacency, dim3(grid_for(D, kBlock)), dim3(kBlock), 0, st, g->key.p, D, k, dir.p,
                               shift, g->out_info.p, g->in_info.p);
        }
        LAUNCH_OK();
        kt.stop();
    }
    g->valid.alloc(mcaat_graph::bitmap_words(D));
    HIP_OK(hipMemsetAsync(g->valid.p + (D + 63) / 64, 0, 8, st));  // the padding word
    hipLaunchKernelGGL(k_valid_init, dim3(grid_for((D + 63) / 64, kBlock)), dim3(kBlock), 0, st, g->valid.p, D);
    g->all_valid = true;
    LAUNCH_OK();
    HIP_OK(hipStreamSynchronize(st));
}

// loads this file's code object now (HIP defers it to the first launch of one of its kernels)
void preload_sdbg_build() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, (const void *)k_count_pal);
}

}  // namespace mcaat
