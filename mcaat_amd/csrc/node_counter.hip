// node_counter.hip — exact canonical (k+1)-mer (edge) multiplicity counting on gfx950.
//
// Replaces the counting inside MEGAHIT Read2SdbgS2::Run (reference sdbg_build.cpp:171-187,
// "-m 1": every edge kept). Design and rooflines: DESIGN.md §node_counter.
//
// Every occurrence of a canonical edge has the same canonical minimizer (the m-mer of its
// window with the smallest hash), so edges are partitioned by minimizer hash and each
// partition is counted in LDS:
//   A  k_sk_scatter : reads -> super-k-mers (maximal runs of edges sharing a minimizer),
//                     written as 16-byte descriptors carrying their bases inline, staged
//                     in LDS and scattered to 256 L1 buckets (top 8 hash bits).
//   B  k_l2_hist / k_l2_scan / k_l2_scatter : one LDS-staged radix pass per L1 bucket
//                     on the next l2_bits hash bits -> 2^(8+l2_bits) fine partitions.
//   C  k_lds_count  : one workgroup per fine partition; expands its super-k-mers and
//                     counts canonical edges in an LDS open-addressing table; emits
//                     (key, count). A partition whose distinct edges overflow the LDS
//                     table is re-counted by the global-table fallback (k_fallback).
// Output order is irrelevant: sdbg_build sorts by BOSS key.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <functional>
#include <memory>
#include <mutex>
#include <type_traits>

#include "internal.h"

namespace mcaat {

namespace {

constexpr int kBlock = 256;

// ---- super-k-mer descriptor (16 B) ----------------------------------------------------
// w0: bases [0,32); w1: bases [32,54) in bits 0..43 | n edges (6 bits) at 44 | 14 hash bits at 50
constexpr int kDescBases = 54;
constexpr int kNShift = 44;
constexpr int kHShift = 50;
constexpr int kHBits = 14;

struct SkParams {
    int E;        // edge length k+1
    int m;        // minimizer length
    int w;        // m-mers per edge window = E - m + 1
    int nmax;     // max edges per descriptor = kDescBases - E + 1
    int l2_bits;  // hash bits after the 8 L1 bits used for fine partitions
    uint64_t salt;
    uint32_t mini;  // slots per reservation (a multiple of 8: every region starts 16-B aligned in the sub rows)
};

__device__ __forceinline__ uint64_t desc_window(uint64_t w0, uint64_t w1, int i, int E) {
    uint64_t v;
    if (i == 0) v = w0;
    else if (i < 32) v = (w0 >> (2 * i)) | (w1 << (64 - 2 * i));
    else v = w1 >> (2 * (i - 32));
    return v & mask_bits(2 * E);
}

// 32-bit helpers for m <= 16: reverse 2-bit groups, bijective mixer (lowbias32)
__device__ __forceinline__ uint32_t rev2_32(uint32_t x) {
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
    return __builtin_bswap32(x);
}
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// partition hash of a minimizer hash (a bijection; the minimum is biased towards 0): the L1
// bucket is its top 8 bits, the next 14 go into the descriptor (sub-partition + class bits).
// 32-bit mixing (lowbias32) instead of a 64-bit finaliser: two of these per super-k-mer in pass A
__device__ __forceinline__ uint32_t part_mix(uint32_t h) { return mix32(h ^ 0x70617274u); }

// canonical (smaller of the edge and its reverse complement); 2-bit reversal by the
// hardware bit reverse plus one swap of adjacent bits
__device__ __forceinline__ uint64_t canon_edge(uint64_t lsb, int E) {
    const uint64_t y = __builtin_bitreverse64(lsb);
    const uint64_t r2 = ((y >> 1) & 0x5555555555555555ULL) | ((y & 0x5555555555555555ULL) << 1);
    const uint64_t rc = (r2 >> (64 - 2 * E)) ^ mask_bits(2 * E);
    return lsb < rc ? lsb : rc;
}

// ---- A: super-k-mers -----------------------------------------------------------------
// One lane scans one work item (<= kItem edge positions of one read) left to right, kCk
// positions per step: a step hashes kCk new m-mers out of one 32-base window (forward and
// reverse-complement m-mers are funnel shifts of the window and of its reverse complement),
// takes the sliding minimum over the W = E-m+1 m-mers of each edge with compile-time
// register indices, and closes the open super-k-mer where the minimum changes (or it
// reaches nmax edges). Closed super-k-mers are appended to the wave's stage segment by
// ballot compaction as {first base, n edges, minimizer hash}; when a segment runs low on
// room the wave fills in the bases of its entries and the workgroup scatters all segments
// to the 256 L1 buckets.
// 4 waves x 900-entry segments: ~52 KB of LDS, so three workgroups (12 waves, the VGPR
// limit at 145 registers) share a CU and one's flush overlaps two others' scans (C3:
// 87.6 -> 77.8 ms against 2 x 1500)
#ifndef MCAAT_AWAVES
#define MCAAT_AWAVES 4
#define MCAAT_ASEG 900
#define MCAAT_APERCU 3
#endif
#ifndef MCAAT_HASH
// minimizer hash: 2 the multiply alone (default since round 5: sk_scatter -1.5 ms at C3, pass C
// unchanged at C3 and -2 ms at C5), 1 multiply-xorshift, 0 mix32
#define MCAAT_HASH 2
#endif
constexpr int kAWaves = MCAAT_AWAVES;
constexpr int kAThreads = kAWaves * 64;
constexpr int kAPerCu = MCAAT_APERCU;   // resident workgroups per CU (LDS <= 160 KB / kAPerCu)
constexpr int kItem = 127;              // edge positions per work item (the close at np fits 16 steps)
constexpr int kCk = 8;                  // positions per step
constexpr int kSeg = MCAAT_ASEG;        // per-wave stage segment (entries); a step appends <= 64*kCk
constexpr int kStage = kSeg * kAWaves;  // 8-B pre-entries
static_assert(kAThreads >= 256, "threads < 256 own one L1 bucket each");
static_assert(kSeg > 64 * kCk, "a segment must hold a worst-case step");
static_assert(kStage <= 65536, "perm holds 16-bit stage indices");

struct ItemSrc {
    const uint64_t *offsets;
    uint64_t n_reads;
    uint64_t fixed_len;   // >0: items computed on the fly
    uint64_t ipr;         // items per read (fixed)
    const uint64_t *item_base;  // explicit items (variable-length reads)
    const uint32_t *item_np;
    uint64_t n_items;
};

__device__ __forceinline__ void get_item(const ItemSrc &s, int E, uint64_t it, uint64_t &base, int &np) {
    if (s.fixed_len) {
        const uint64_t r = it / s.ipr, c = it - r * s.ipr;
        const uint64_t npos = s.fixed_len - E + 1;
        base = r * s.fixed_len + c * kItem;
        const uint64_t rem = npos - c * kItem;
        np = (int)(rem < (uint64_t)kItem ? rem : kItem);
    } else {
        base = s.item_base[it];
        np = (int)s.item_np[it];
    }
}

// two consecutive words of the packed stream, 8-B aligned: one global_load_dwordx4
struct __attribute__((aligned(8))) u64x2 {
    uint64_t a, b;
};

// 2-bit-group reversal by the hardware bit reverse
__device__ __forceinline__ uint64_t rev2_dev(uint64_t x) {
    // per 32-bit half (two 32-bit shifts and one bitfield select each, no 64-bit shifts)
    const uint32_t lo = __builtin_bitreverse32((uint32_t)(x >> 32)), hi = __builtin_bitreverse32((uint32_t)x);
    const uint32_t l = ((lo >> 1) & 0x55555555u) | ((lo << 1) & 0xAAAAAAAAu);
    const uint32_t h = ((hi >> 1) & 0x55555555u) | ((hi << 1) & 0xAAAAAAAAu);
    return ((uint64_t)h << 32) | l;
}

// 32 bases starting at absolute base B of the packed stream, from its two words
__device__ __forceinline__ uint64_t win32(uint64_t a, uint64_t b, uint64_t B) {
    const int sh = 2 * (int)(B & 31);
    return sh ? (a >> sh) | (b << (64 - sh)) : a;
}

// hashes of the kCk canonical m-mers starting at the bases 0..kCk-1 of win (m <= 16);
// FULL: m == 16, so the m-mers need no mask
#ifndef MCAAT_HTOP
#define MCAAT_HTOP 1
#endif
template <bool FULL>
__device__ __forceinline__ void hash_step(uint64_t win, int m, uint32_t mmask, uint32_t salt, uint32_t *h) {
#if MCAAT_HTOP
    // both m-mers extracted with their bases in the top 2m bits of a 32-bit word (one
    // alignbit each, none at t = 0; the bits below are other bases), so the mask becomes one
    // shift after the min: min(f_top, r_top) >> (32 - 2m) == min(f, r) (equal top fields
    // give equal results whichever one the min takes)
    const int lo = 32 - 2 * m;
    const uint64_t Wt = win << lo;          // base j at bits 2j + lo
    const uint64_t R = rev2_dev(win) ^ ~0ULL;  // complement of base j at bits 62 - 2j
    const uint32_t wl = (uint32_t)Wt, wh = (uint32_t)(Wt >> 32);
    const uint32_t rl = (uint32_t)R, rh = (uint32_t)(R >> 32);
    (void)mmask;
#pragma unroll
    for (int t = 0; t < kCk; ++t) {
        const uint32_t f = t ? __builtin_amdgcn_alignbit(wh, wl, 2 * t) : wl;
        const uint32_t r = t ? __builtin_amdgcn_alignbit(rh, rl, 32 - 2 * t) : rh;
        const uint32_t c = FULL ? min(f, r) : min(f, r) >> lo;
#if MCAAT_HASH == 2
        // a multiply by an odd constant: a bijection whose high bits, which decide the
        // minimizer order, mix every key bit (the buckets and sub-partitions come from a
        // re-hash, so the weak low bits do not matter)
        h[t] = (c ^ salt) * 0x9E3779B1u;
#elif MCAAT_HASH == 1
        uint32_t x = (c ^ salt) * 0x9E3779B1u;
        h[t] = x ^ (x >> 15);
#else
        h[t] = mix32(c ^ salt);
#endif
    }
#else
    const uint64_t R = (rev2_dev(win) ^ ~0ULL) >> (2 * (25 - m));  // rc, aligned for t = 7
    const uint32_t wl = (uint32_t)win, wh = (uint32_t)(win >> 32);
    const uint32_t rl = (uint32_t)R, rh = (uint32_t)(R >> 32);
#pragma unroll
    for (int t = 0; t < kCk; ++t) {
        uint32_t f = __builtin_amdgcn_alignbit(wh, wl, 2 * t);
        uint32_t r = __builtin_amdgcn_alignbit(rh, rl, 2 * (kCk - 1 - t));
        if (!FULL) {
            f &= mmask;
            r &= mmask;
        }
#if MCAAT_HASH == 2
        h[t] = (min(f, r) ^ salt) * 0x9E3779B1u;  // A/B: the multiply alone
#elif MCAAT_HASH == 1
        // multiply-xorshift: a bijection, and only the minimizer order depends on it (the
        // buckets and sub-partitions come from a re-hash), so a short one suffices
        uint32_t x = (min(f, r) ^ salt) * 0x9E3779B1u;
        h[t] = x ^ (x >> 15);
#else
        h[t] = mix32(min(f, r) ^ salt);
#endif
    }
#endif
}

// minimum over the hashes u .. u+W-1 (u < kCk) of the 3*kCk-entry ring H whose logical
// entry 0 is physical entry G*kCk (W <= 16)
template <int W, int G>
__device__ __forceinline__ void window_min(const uint32_t *H, uint32_t *hm) {
    auto at = [&](int u) { return H[(G * kCk + u) % (3 * kCk)]; };
    if constexpr (W > kCk) {
        // suffix minima of H[t..kCk-1] and prefix minima of H[kCk..kCk+u]
        uint32_t S[kCk], Pm[W - 1];
        S[kCk - 1] = at(kCk - 1);
#pragma unroll
        for (int t = kCk - 2; t >= 0; --t) S[t] = min(at(t), S[t + 1]);
        Pm[0] = at(kCk);
#pragma unroll
        for (int u = 1; u < W - 1; ++u) Pm[u] = min(Pm[u - 1], at(kCk + u));
#pragma unroll
        for (int t = 0; t < kCk; ++t) hm[t] = min(S[t], Pm[t + W - 1 - kCk]);
    } else {
#pragma unroll
        for (int t = 0; t < kCk; ++t) {
            uint32_t v = at(t);
#pragma unroll
            for (int q = 1; q < W; ++q) v = min(v, at(t + q));
            hm[t] = v;
        }
    }
}

// descriptors reserved per (workgroup, L1 bucket) grab (SkParams::mini, a power of two): 1024 on
// one GPU; (round 6) 256 for a rank of a sharded build, where the L1 buckets' headroom for every
// workgroup's two partly used reservations per bucket falls from 7.2 GB to 1.8 GB, so eight ranks
// of C3 fit one GPU in the tests (1024 ran out of memory). Pass A at C3: 72.3 ms at 1024, 73.3-73.8
// at 256 (more reservation atomics); knob nc.a_mini sets it
constexpr uint32_t kMiniOne = 1024, kMiniShard = 256;
constexpr uint16_t kDeadSub = 0xffff;  // sub-partition mark of an inert (n = 0) slot


#ifndef MCAAT_WB
#define MCAAT_WB 4
#endif
#ifndef MCAAT_APF
#define MCAAT_APF 1
#endif
constexpr int kAPF = MCAAT_APF;  // scan steps of window words in flight (1 or 2)
constexpr int kWB = MCAAT_WB;
#ifndef MCAAT_WPIPE
#define MCAAT_WPIPE 0
#endif
#ifndef MCAAT_CLOSEMASK
#define MCAAT_CLOSEMASK 1
#endif
constexpr bool kWPipe = MCAAT_WPIPE != 0;  // write phase: the next batch's loads before this batch's stores  // write batch (entries per thread per round: 3 loads each in flight)

// 8-byte pre-entry of a closed super-k-mer: minimizer hash (low 32 bits); above it the
// close position (7 bits), the first position (7), batch parity (1) and lane (6), all in
// its item. The item's first base comes from the wave's table of the current and previous
// batch (sbase), so the pre-entry is half a descriptor and the stage holds 1600 per wave;
// bases are fetched when the entry is written. The scan keeps the first position
// pre-shifted (p7 = p << 7) and the parity and lane pre-placed (ihc), so the high word is
// one add.
constexpr int kPeP = 7, kPePar = 14, kPeLane = 15;

template <int W, bool FULL>
__global__ void __launch_bounds__(kAThreads) k_sk_scatter(const uint64_t *__restrict__ packed, ItemSrc src,
                                                          SkParams P, uint4 *__restrict__ l1_data,
                                                          const uint64_t *__restrict__ l1_base,
                                                          const uint64_t *__restrict__ l1_cap,
                                                          unsigned long long *l1_cursor, uint16_t *__restrict__ l1_sub,
                                                          unsigned long long *prof, unsigned long long *rstate, int rmode) {
    __shared__ uint64_t stage[kStage];
    __shared__ uint8_t stage_l1[kStage];
    __shared__ uint16_t perm[kStage];         // stage entries in bucket order
    __shared__ uint64_t sbase[kAWaves][2][64];  // item first base per (wave, batch parity, lane)
    __shared__ uint32_t hist[256];            // entries per bucket in this flush
    __shared__ uint32_t boff[256];            // exclusive scan of hist
    __shared__ uint32_t bcur[256];            // rank cursors
    __shared__ unsigned long long rpos[256];  // next free slot of this workgroup's reservation (absolute)
    __shared__ unsigned long long rlim[256];  // end of the bucket's region (absolute)
    __shared__ uint32_t rleft[256];           // slots left in it
    __shared__ uint32_t wtot[kAWaves];
    __shared__ int more_flag[2];  // alternating per flush: set, barrier, read; reset a flush later

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tb = threadIdx.x;  // threads < 256 own bucket tb through every flush
    // each bucket holds its current reservation and, in a register of its owner thread,
    // the next one, requested a flush ahead so the cursor atomic's latency is hidden
    // (the atomic's result stays unused until the next flush, so its latency is hidden)
    unsigned long long my_next = 0, my_base = 0;
    uint32_t prev_need = 0;  // applied to rpos/rleft at the next flush (after its barrier)
    // rmode (one launch per part of a streamed input, nc_ahead_*): 0 a single launch; 1 the
    // first of several, 2 a middle one, 3 the last. After 1 and 2 every workgroup leaves its
    // reservations in rstate (no inert fill) and the next launch (same grid) takes them up
    unsigned long long *rs = rstate ? rstate + ((uint64_t)blockIdx.x * 256 + (tb & 255)) * 3 : nullptr;
    if (tb < 256) {
        hist[tb] = 0;
        bcur[tb] = 0;
        my_base = l1_base[tb];
        rlim[tb] = my_base + l1_cap[tb];
        if (rmode >= 2) {
            rpos[tb] = rs[0];
            rleft[tb] = (uint32_t)rs[1];
            my_next = rs[2];
        } else {
            rleft[tb] = 0;
            my_next = atomicAdd(&l1_cursor[tb], (unsigned long long)P.mini);
        }
    }
    if (threadIdx.x == 0) more_flag[0] = more_flag[1] = 0;
    __syncthreads();
    uint64_t *seg = stage + __builtin_amdgcn_readfirstlane(wave * kSeg);  // wave-uniform: a scalar base
    uint8_t *seg_l1 = stage_l1 + wave * kSeg;
    uint32_t nflush = 0;

    // absolute slot; a bucket whose region is exhausted drops the write (its cursor keeps
    // counting, so the host re-sizes and re-runs). Beside each descriptor goes its fine
    // sub-partition (kDeadSub for padding), so pass B's counting passes read 2 bytes, not 16.
    const int sub_shift = kHShift + kHBits - P.l2_bits;
    auto put = [&](int b, uint64_t pos, const uint4 &d) {
        if (pos < rlim[b]) {
            l1_data[pos] = d;
            const uint64_t hi = (uint64_t)d.w << 32;
            l1_sub[pos] = ((d.w >> (kNShift - 32)) & 63) ? (uint16_t)(sub_shift < 64 ? hi >> sub_shift : 0) : kDeadSub;
        }
    };

    const uint64_t n_items = src.fixed_len ? src.n_reads * src.ipr : src.n_items;
    const uint64_t n_batches = (n_items + 63) / 64;
    const uint64_t bstride = (uint64_t)gridDim.x * kAWaves;
    uint64_t batch = (uint64_t)blockIdx.x * kAWaves + wave;
    constexpr bool kFull = FULL;  // m == 16: the m-mers need no mask
    const uint32_t mmask = (uint32_t)mask_bits(2 * P.m);
    const uint32_t salt32 = (uint32_t)P.salt;
    const int nmax = P.nmax;

    // per-lane scan state (wave-uniform: active, c, ph, nck, fill, par, bsf)
    uint32_t H[3 * kCk];  // ring of three 8-hash groups; step c reads groups c, c+1, c+2 (mod 3)
    uint64_t cw[3], pa = 0, pb = 0;  // the item's first words; the next step's window words
    uint64_t qa = 0, qb = 0;         // kAPF == 2: the step after next's
    uint64_t s = 0;
    int np = 0, c = 0, ph = 0, nck = 0;
    uint32_t prev_hm = 0, h_open = 0, p7 = 0, ihc = 0, fill = 0, par = 1, bsf = 0;
    bool active = false;
    auto fetch = [&](uint64_t bt, uint64_t &sb, int &n, uint64_t *w) {
        const uint64_t item = bt * 64 + lane;
        sb = 0;
        n = 0;
        if (bt < n_batches && item < n_items) get_item(src, P.E, item, sb, n);
#pragma unroll
        for (int k = 0; k < 3; ++k) w[k] = packed[(sb >> 5) + k];
    };

    // one step: positions 8c .. 8c+7 of the lane's item; the window's bases start at 8c+16.
    // G = c mod 3 names the ring group holding positions 8c.. (compile time, so the ring
    // never moves). Positions are wave-uniform, so the close test is four compares.
    auto step = [&](auto Gc) {
        constexpr int G = decltype(Gc)::value;
        c = __builtin_amdgcn_readfirstlane(c);
        const int rb = kCk * c + 2 * kCk;
        const uint64_t win = win32(pa, pb, s + rb);
        if constexpr (kAPF == 2) {  // the step after next's window words; the next step's were loaded a step ago
            pa = qa;
            pb = qb;
            const u64x2 nx = *(const u64x2 *)(packed + ((s + rb + 2 * kCk) >> 5));
            qa = nx.a;
            qb = nx.b;
        } else {
            const u64x2 nx = *(const u64x2 *)(packed + ((s + rb + kCk) >> 5));  // next step's window words
            pa = nx.a;
            pb = nx.b;
        }
        hash_step<kFull>(win, P.m, mmask, salt32, H + ((G + 2) % 3) * kCk);
        uint32_t hm[kCk];
        window_min<W, G>(H, hm);
        if (c == 0) {
            prev_hm = hm[0];
            h_open = hm[0];
            p7 = 0;
        }
#if MCAAT_CLOSEMASK
        // the close test as four compares straight into lane masks (no bool materialised
        // between the ballot and the branch), the closing lanes' region entered on the mask
        // itself; the entry's hash is the previous position's (a super-k-mer's minimizer hash
        // is constant from its open to its close), so no open hash is carried. The fill count
        // is wave-uniform: kept in a scalar register, its additions are scalar
        fill = __builtin_amdgcn_readfirstlane(fill);
#pragma unroll
        for (int t = 0; t < kCk; ++t) {
            const int i = kCk * c + t;
            const uint32_t prv = t ? hm[t - 1] : prev_hm;
            const unsigned long long bm = __builtin_amdgcn_ballot_w64((uint32_t)(i - 1) < (uint32_t)np) &
                                          (__builtin_amdgcn_ballot_w64(i == np) |
                                           __builtin_amdgcn_ballot_w64(hm[t] != prv) |
                                           __builtin_amdgcn_ballot_w64((int)p7 <= (i - nmax) * 128));
            if (bm) {
                if (__builtin_amdgcn_inverse_ballot_w64(bm)) {
                    const uint32_t idx =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
                    seg[fill + idx] = ((uint64_t)(p7 + ihc + (uint32_t)i) << 32) | prv;
                    p7 = (uint32_t)i << kPeP;
                }
                fill += (uint32_t)__popcll(bm);
            }
        }
        (void)h_open;
#else
#pragma unroll
        for (int t = 0; t < kCk; ++t) {
            const int i = kCk * c + t;
            const uint32_t prv = t ? hm[t - 1] : prev_hm;
            const bool cl = ((uint32_t)(i - 1) < (uint32_t)np) &
                            ((i == np) | (hm[t] != prv) | ((int)p7 <= (i - nmax) * 128));
            const unsigned long long bm = __builtin_amdgcn_ballot_w64(cl);
            if (bm) {
                if (cl) {
                    const uint32_t idx =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, fill));
                    // one 8-B LDS store per close (two 4-B stores at a 2-word stride were 2-way
                    // bank conflicts for consecutive lanes)
                    seg[idx] = ((uint64_t)(p7 + ihc + (uint32_t)i) << 32) | h_open;
                    p7 = (uint32_t)i << kPeP;
                    h_open = hm[t];
                }
                fill += (uint32_t)__popcll(bm);
            }
        }
#endif
        prev_hm = hm[kCk - 1];
    };

    // MCAAT_PROF_A=1: 100-MHz real-time ticks per phase, summed over waves
    unsigned long long tp[5] = {0, 0, 0, 0, 0}, t0 = prof ? __builtin_amdgcn_s_memrealtime() : 0;
    auto tick = [&](int phase) {
        if (prof) {
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            tp[phase] += t1 - t0;
            t0 = t1;
        }
    };

    // a new item hashes its first two groups into the ring groups G, G+1
    auto start_item = [&](auto Gc) {
        constexpr int G = decltype(Gc)::value;
        fetch(batch, s, np, cw);
        par ^= 1u;
        ++bsf;
        sbase[wave][par][lane] = s;
        ihc = (par << kPePar) | ((uint32_t)lane << kPeLane);
        {
            const u64x2 nx = *(const u64x2 *)(packed + ((s + 2 * kCk) >> 5));
            pa = nx.a;
            pb = nx.b;
        }
        if constexpr (kAPF == 2) {
            const u64x2 nx = *(const u64x2 *)(packed + ((s + 3 * kCk) >> 5));
            qa = nx.a;
            qb = nx.b;
        }
        int mx = np;
#pragma unroll
        for (int o = 32; o; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
        nck = mx / kCk + 1;  // steps covering positions 0..max np (the last close)
        const int o8 = (int)(s & 31) + kCk;
        hash_step<kFull>(win32(cw[0], cw[1], s), P.m, mmask, salt32, H + G * kCk);
        hash_step<kFull>(o8 >= 32 ? win32(cw[1], cw[2], s + kCk) : win32(cw[0], cw[1], s + kCk), P.m, mmask,
                         salt32, H + ((G + 1) % 3) * kCk);
        c = 0;
        active = true;
    };
    // false: the wave goes to the flush with its ring at phase G
    auto run = [&](auto Gc) -> bool {
        constexpr int G = decltype(Gc)::value;
        if (!active) {
            // no more items, or the segment already references two batches (the sbase slots)
            if (batch >= n_batches || bsf >= 2) {
                ph = G;
                return false;
            }
            start_item(Gc);
        }
        // a wave short of room for a worst-case step goes to the flush
        if (fill + 64 * kCk > (uint32_t)kSeg) {
            ph = G;
            return false;
        }
        step(Gc);
        if (++c == nck) {
            active = false;
            batch += bstride;
        }
        return true;
    };

    for (;;) {
        // the scan is unrolled over the three ring phases; a flush may interrupt it at any
        // phase, so the ring is rotated back to phase 0 first (once per flush)
        ph = __builtin_amdgcn_readfirstlane(ph);
        if (ph != 0) {
            uint32_t T[3 * kCk];
#pragma unroll
            for (int u = 0; u < 3 * kCk; ++u) T[u] = H[u];
            if (ph == 1) {
#pragma unroll
                for (int u = 0; u < 3 * kCk; ++u) H[u] = T[(u + kCk) % (3 * kCk)];
            } else {
#pragma unroll
                for (int u = 0; u < 3 * kCk; ++u) H[u] = T[(u + 2 * kCk) % (3 * kCk)];
            }
            ph = 0;
        }
        for (;;) {
            if (!run(std::integral_constant<int, 0>())) break;
            if (!run(std::integral_constant<int, 1>())) break;
            if (!run(std::integral_constant<int, 2>())) break;
        }
        tick(0);
        // bucket of each entry: the minimum hash is biased towards 0, so buckets come from
        // a re-hash of it (a bijection)
        for (uint32_t e = lane; e < fill; e += 64) {
            const uint32_t l1 = part_mix((uint32_t)seg[e]) >> 24;
            seg_l1[e] = (uint8_t)l1;
            atomicAdd(&hist[l1], 1u);
        }
        tick(1);
        if (lane == 0) wtot[wave] = fill;
        if (lane == 0 && (active || batch < n_batches)) more_flag[nflush & 1] = 1;
        lds_barrier();  // A: stage, hist, wtot complete
        const int more = more_flag[nflush & 1];
        if (threadIdx.x == 0) more_flag[(nflush + 1) & 1] = 0;
        ++nflush;
        tick(2);
        // reservations (threads < 256, one bucket each) and the bucket offsets (wave 0)
        if (tb < 256) {
            rpos[tb] += prev_need;
            rleft[tb] -= prev_need;
            const uint32_t need = hist[tb];
            if (need > rleft[tb]) {
                for (uint32_t z = 0; z < rleft[tb]; ++z) put(tb, rpos[tb] + z, make_uint4(0, 0, 0, 0));
                if (need <= P.mini) {
                    rpos[tb] = my_base + my_next;
                    rleft[tb] = P.mini;
                    my_next = atomicAdd(&l1_cursor[tb], (unsigned long long)P.mini);
                } else {  // more than a reservation in one flush: grab synchronously
                    const uint32_t grab = ((need + P.mini - 1) / P.mini) * P.mini;
                    rpos[tb] = my_base + atomicAdd(&l1_cursor[tb], (unsigned long long)grab);
                    rleft[tb] = grab;
                }
            }
            prev_need = need;
        }
        if (wave == 0) {
            const uint4 hv = *(const uint4 *)&hist[4 * lane];
            const uint32_t sum4 = hv.x + hv.y + hv.z + hv.w;
            uint32_t incl = sum4;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = __shfl_up(incl, o);
                if (lane >= o) incl += v;
            }
            const uint32_t ex = incl - sum4;
            *(uint4 *)&boff[4 * lane] = make_uint4(ex, ex + hv.x, ex + hv.x + hv.y, ex + hv.x + hv.y + hv.z);
        }
        lds_barrier();  // B: boff, rpos ready; hist consumed
        if (tb < 256) hist[tb] = 0;
        tick(3);
        for (uint32_t e = lane; e < fill; e += 64) {
            const int b = seg_l1[e];
            perm[boff[b] + atomicAdd(&bcur[b], 1u)] = (uint16_t)(wave * kSeg + e);
        }
        lds_barrier();  // C: perm ready
        // consecutive threads write consecutive slots of a bucket's run; each entry's bases
        // are fetched here (kWB entries per thread per round, their loads in flight together)
        uint32_t total = 0;
#pragma unroll
        for (int w = 0; w < kAWaves; ++w) total += wtot[w];
        // a batch of kWB entries per thread: first its stage reads and base loads, then the
        // descriptors; with kWPipe the next batch's loads are issued before this batch's
        // descriptors are built (two batches of registers, slots fixed at compile time)
        uint64_t q[2][kWB], B0[2][kWB], x[2][kWB][3];
        auto load_batch = [&](auto Sc, uint32_t j0) {
            constexpr int S = decltype(Sc)::value;
#pragma unroll
            for (int k = 0; k < kWB; ++k) {
                const uint32_t j = j0 + k * kAThreads;
                q[S][k] = 0;
                B0[S][k] = 0;
                if (j < total) {
                    const uint32_t i = perm[j];
                    q[S][k] = stage[i];
                    const uint32_t hi = (uint32_t)(q[S][k] >> 32);
                    const uint32_t ln = (hi >> kPeLane) & 63, pr = (hi >> kPePar) & 1;
                    B0[S][k] = sbase[i / kSeg][pr][ln] + ((hi >> kPeP) & 127);
                }
                // the first two words in one 16-B load; the third only when the bases reach
                // it (these loads are uncoalesced, so the vector L1 pays per lane and line)
                const int L = (int)(((uint32_t)(q[S][k] >> 32) & 127) - (((uint32_t)(q[S][k] >> 32) >> kPeP) & 127)) + P.E - 1;
                const u64x2 x01 = *(const u64x2 *)(packed + (B0[S][k] >> 5));
                x[S][k][0] = x01.a;
                x[S][k][1] = x01.b;
                x[S][k][2] = j < total && 2 * (int)(B0[S][k] & 31) + 2 * L > 128 ? packed[(B0[S][k] >> 5) + 2] : 0;
            }
        };
        auto store_batch = [&](auto Sc, uint32_t j0) {
            constexpr int S = decltype(Sc)::value;
#pragma unroll
            for (int k = 0; k < kWB; ++k) {
                const uint32_t j = j0 + k * kAThreads;
                if (j >= total) continue;
                const uint32_t i = perm[j];
                const int b = stage_l1[i];
                const uint32_t hi = (uint32_t)(q[S][k] >> 32);
                const uint32_t n = (hi & 127) - ((hi >> kPeP) & 127);
                const int sh = 2 * (int)(B0[S][k] & 31);
                // bases past the last edge are zeroed, so every copy of a super-k-mer is the
                // same 128-bit descriptor whatever follows it in its read
                const int L = (int)n + P.E - 1;
                const uint64_t w0 = (sh ? (x[S][k][0] >> sh) | (x[S][k][1] << (64 - sh)) : x[S][k][0]) & mask_bits(2 * L);
                uint64_t w1 = (sh ? (x[S][k][1] >> sh) | (x[S][k][2] << (64 - sh)) : x[S][k][1]) &
                              mask_bits(L > 32 ? 2 * (L - 32) : 0);
                const uint32_t h = part_mix((uint32_t)q[S][k]);
                w1 |= ((uint64_t)n << kNShift) | ((uint64_t)((h >> (24 - kHBits)) & ((1u << kHBits) - 1)) << kHShift);
                put(b, rpos[b] + (j - boff[b]),
                    make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)));
            }
        };
        constexpr uint32_t kStep = kWB * kAThreads;
        using S0 = std::integral_constant<int, 0>;
        using S1 = std::integral_constant<int, 1>;
        if constexpr (kWPipe) {
            uint32_t j0 = threadIdx.x;
            if (j0 < total) load_batch(S0(), j0);
            for (; j0 < total; j0 += 2 * kStep) {
                if (j0 + kStep < total) load_batch(S1(), j0 + kStep);
                store_batch(S0(), j0);
                if (j0 + kStep >= total) break;
                if (j0 + 2 * kStep < total) load_batch(S0(), j0 + 2 * kStep);
                store_batch(S1(), j0 + kStep);
            }
        } else {
            for (uint32_t j0 = threadIdx.x; j0 < total; j0 += kStep) {
                load_batch(S0(), j0);
                store_batch(S0(), j0);
            }
        }
        if (tb < 256) bcur[tb] = 0;
        fill = 0;
        bsf = active ? 1u : 0u;  // the batch in progress keeps its sbase slot
        lds_barrier();  // D: stage free again
        tick(4);
        if (!more) break;
    }
    // zero-fill what is left of this workgroup's reservations, the current and the
    // prefetched one (n = 0 descriptors are inert)
    if (tb < 256) {
        rpos[tb] += prev_need;
        rleft[tb] -= prev_need;
    }
    if (rmode == 1 || rmode == 2) {  // the next launch continues these reservations
        if (tb < 256) {
            rs[0] = rpos[tb];
            rs[1] = rleft[tb];
            rs[2] = my_next;
        }
        return;
    }
    __syncthreads();
    for (int pass = 0; pass < 2; ++pass) {
        for (int b = 0; b < 256; ++b)
            for (uint32_t z = threadIdx.x; z < rleft[b]; z += kAThreads) put(b, rpos[b] + z, make_uint4(0, 0, 0, 0));
        __syncthreads();
        if (tb < 256) {
            rpos[tb] = my_base + my_next;
            rleft[tb] = P.mini;
        }
        __syncthreads();
    }
    if (prof && lane == 0)
        for (int i = 0; i < 5; ++i) atomicAdd(&prof[i], tp[i]);
}

typedef void (*SkKernel)(const uint64_t *, ItemSrc, SkParams, uint4 *, const uint64_t *, const uint64_t *,
                         unsigned long long *, uint16_t *, unsigned long long *, unsigned long long *, int);
SkKernel sk_kernel(int w, bool full) {
    if (full) {
        switch (w) {
#define MCAAT_SK(W) \
    case W:         \
        return k_sk_scatter<W, true>;
            MCAAT_SK(9) MCAAT_SK(10) MCAAT_SK(11) MCAAT_SK(12) MCAAT_SK(13) MCAAT_SK(14) MCAAT_SK(15) MCAAT_SK(16)
#undef MCAAT_SK
        }
    } else {
        switch (w) {
#define MCAAT_SK(W) \
    case W:         \
        return k_sk_scatter<W, false>;
            MCAAT_SK(1) MCAAT_SK(2) MCAAT_SK(3) MCAAT_SK(4) MCAAT_SK(5) MCAAT_SK(6) MCAAT_SK(7) MCAAT_SK(8)
            MCAAT_SK(9) MCAAT_SK(10) MCAAT_SK(11) MCAAT_SK(12) MCAAT_SK(13) MCAAT_SK(14) MCAAT_SK(15) MCAAT_SK(16)
#undef MCAAT_SK
        }
    }
    throw Error(MCAAT_E_INVALID, "node_counter: minimizer window out of range");
}

// ---- B: radix pass on the next l2_bits hash bits, per L1 bucket -----------------------------
// k_l2_hist adds each workgroup's LDS histogram into the per-(bucket, sub) totals; after an
// exclusive scan those are the fine-partition bases, and k_l2_scatter reserves space per
// (workgroup, sub) with one atomic on the fine cursor and ranks inside the workgroup in LDS.
constexpr int kBThreads = 1024;
constexpr uint32_t kChunk = 65536;


// Every (chunk, sub) run is rounded up to a multiple of 4 descriptors (64 B) and padded
// with inert ones, so each 64-B line of the fine partitions is written by one workgroup.
#ifndef MCAAT_BLG
#define MCAAT_BLG 4
#endif
constexpr int kLG = MCAAT_BLG;  // descriptors per buffered line (4: 64 B)
static_assert(kLG == 2 || kLG == 4, "32-B or 64-B lines");
__device__ __forceinline__ uint32_t round4(uint32_t x) { return (x + kLG - 1) & ~(uint32_t)(kLG - 1); }

// LDS histogram of one chunk's sub rows (16-B aligned: 8 rows per load, all loads of a
// thread in flight together)
__device__ __forceinline__ void chunk_hist(const uint16_t *__restrict__ sub, uint64_t s0, uint32_t n, uint32_t *lh) {
    const uint4 *v = (const uint4 *)(sub + s0);
    const uint32_t n8 = n / 8;
    for (uint32_t i0 = threadIdx.x; i0 < n8; i0 += 4 * kBThreads) {
        uint4 q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = i0 + k * kBThreads < n8 ? v[i0 + k * kBThreads] : make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t w[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if ((w[j] & 0xffff) != kDeadSub) atomicAdd(&lh[w[j] & 0xffff], 1u);
                if ((w[j] >> 16) != kDeadSub) atomicAdd(&lh[w[j] >> 16], 1u);
            }
        }
    }
    for (uint32_t i = 8 * n8 + threadIdx.x; i < n; i += kBThreads) {
        const uint32_t x = sub[s0 + i];
        if (x != kDeadSub) atomicAdd(&lh[x], 1u);
    }
}

// (round 3) each chunk's sub counts are also kept (cc[c][i]); k_chunk_runs turns them into the
// chunk's run start per sub, so k_l2_scatter needs neither a counting pass over the chunk's sub
// rows nor one cursor atomic per (chunk, sub)
__global__ void __launch_bounds__(kBThreads) k_l2_hist(const uint16_t *__restrict__ sub, const uint64_t *chunk_start,
                                                       const uint32_t *chunk_len, const uint32_t *chunk_bucket,
                                                       int l2_bits, unsigned long long *tot, uint32_t *cc) {
    extern __shared__ uint32_t lh[];
    const uint32_t S = 1u << l2_bits;
    const uint64_t c = blockIdx.x;
    for (uint32_t i = threadIdx.x; i < S; i += kBThreads) lh[i] = 0;
    __syncthreads();
    chunk_hist(sub, chunk_start[c], chunk_len[c], lh);
    __syncthreads();
    const uint64_t fb = (uint64_t)chunk_bucket[c] * S;
    for (uint32_t i = threadIdx.x; i < S; i += kBThreads) {
        cc[c * S + i] = lh[i];
        if (lh[i]) atomicAdd(&tot[fb + i], (unsigned long long)round4(lh[i]));
    }
}

// chunk run starts in lines, in place of the chunk counts: one thread per (L1 bucket, sub) walks
// the bucket's chunks from the sub's fine-partition base
__global__ void __launch_bounds__(256) k_chunk_runs(uint32_t *cc, const uint64_t *bchunk, const uint64_t *fine,
                                                    uint32_t S) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 256ull * S) return;
    const uint64_t b = t / S, i = t % S;
    uint64_t run = fine[t] / kLG;
    for (uint64_t c = bchunk[b]; c < bchunk[b + 1]; ++c) {
        const uint32_t x = cc[c * S + i];
        cc[c * S + i] = (uint32_t)run;
        run += round4(x) / kLG;
    }
}

// Each sub keeps one 64-B line (4 descriptors) of its run in LDS; the lane that completes
// the line writes it out whole, so HBM sees full-line writes instead of 16-B pieces. Runs
// start on line boundaries (round4), so no line is shared by two workgroups. A sub that gets
// more descriptors in one round than its buffered line holds writes the excess directly
// (rare), and copies the ones that belong to its new partial line into the buffer once the
// old line has been written.
constexpr int kMaxSub = 2048;   // l2_bits <= 11: 128 KB of line buffers
#ifndef MCAAT_BPF
#define MCAAT_BPF 2
#endif
constexpr int kBPF = MCAAT_BPF;  // rounds of descriptor loads in flight
#ifndef MCAAT_BCOOP
#define MCAAT_BCOOP 1
#endif
constexpr bool kCoopFlush = MCAAT_BCOOP != 0;  // completed lines written by the whole wave

__global__ void __launch_bounds__(kBThreads) k_l2_scatter(const uint4 *__restrict__ data,
                                                          const uint16_t *__restrict__ sub,
                                                          const uint64_t *chunk_start, const uint32_t *chunk_len,
                                                          const uint32_t *runs, int l2_bits,
                                                          uint4 *__restrict__ out, uint64_t gbase) {
    __shared__ uint4 buf[kMaxSub * kLG];
    __shared__ uint32_t lb[kMaxSub];  // this workgroup's run of each sub, in lines
    __shared__ uint32_t lc[kMaxSub];  // descriptors per sub placed so far
    __shared__ uint32_t bl[kMaxSub];  // line of the run held in buf
    const uint32_t S = 1u << l2_bits;
    const uint64_t c = blockIdx.x;  // (chunk index relative to the launch's first chunk: runs is offset to match)
    for (uint32_t i = threadIdx.x; i < S; i += kBThreads) {
        lb[i] = runs[c * S + i];
        lc[i] = 0;
        bl[i] = 0;
    }
    __syncthreads();
    const uint64_t s0 = chunk_start[c];
    const uint32_t n = chunk_len[c];
    // one descriptor per thread per round, the next kBPF rounds' already in flight
    uint32_t v[kBPF];
    uint4 d[kBPF];
#pragma unroll
    for (int j = 0; j < kBPF; ++j) {
        const uint32_t i = j * kBThreads + threadIdx.x;
        v[j] = i < n ? sub[s0 + i] : kDeadSub;
        d[j] = i < n ? data[s0 + i] : make_uint4(0, 0, 0, 0);
    }
    for (uint32_t i00 = 0; i00 < n; i00 += kBPF * kBThreads)
#pragma unroll
    for (int j = 0; j < kBPF; ++j) {
        const uint32_t i0 = i00 + j * kBThreads;
        if (i0 >= n) break;  // uniform: every thread reaches the same barriers
        const uint32_t cv = v[j];
        const uint4 cd = d[j];
        const uint32_t ni = i0 + kBPF * kBThreads + threadIdx.x;
        v[j] = ni < n ? sub[s0 + ni] : kDeadSub;
        if (ni < n) d[j] = data[s0 + ni];
        const bool live = cv != kDeadSub;
        uint32_t r = 0, line = 0;
        bool buffered = false;
        if (live) {
            r = atomicAdd(&lc[cv], 1u);
            line = bl[cv];
            buffered = r / kLG == line;
            if (buffered) buf[cv * kLG + (r & (kLG - 1))] = cd;
            else out[(uint64_t)lb[cv] * kLG + r - gbase] = cd;
        }
        lds_barrier();
        uint32_t nline = 0;
        if (kCoopFlush) {
            // the lines completed this round leave the wave kLG lanes per line, each lane one
            // 16-B piece: one store instruction writes 64/kLG whole lines (one lane per line
            // with kLG stores before), and the LDS reads are kLG-lane contiguous runs
            const bool done = live && buffered && (r & (kLG - 1)) == kLG - 1;
            const unsigned long long dm = __ballot(done);
            const uint32_t lane = threadIdx.x & 63;
            const uint64_t dst = done ? ((uint64_t)lb[cv] + line) * kLG - gbase : 0;
            const uint32_t src = done ? cv * kLG : 0;
            const int nd = __popcll(dm);
            for (int b0 = 0; b0 < nd; b0 += 64 / kLG) {
                const int j = b0 + (int)(lane / kLG);  // the line this lane helps write
                // lane holding the j-th set bit of dm (binary search on prefix popcounts)
                int pos = 0;
                if (j < nd) {
#pragma unroll
                    for (int step = 32; step; step >>= 1) {
                        const unsigned long long below = dm & ((pos + step >= 64) ? ~0ull : ((1ull << (pos + step)) - 1));
                        if (__popcll(below) <= j) pos += step;
                    }
                }
                const uint64_t d = __shfl(dst, pos);
                const uint32_t sidx = __shfl(src, pos);
                if (j < nd) out[d + (lane & (kLG - 1))] = buf[sidx + (lane & (kLG - 1))];
            }
            if (live) {
                nline = lc[cv] / kLG;
                bl[cv] = nline;  // every writer stores the same value
            }
        } else if (live) {
            if (buffered && (r & (kLG - 1)) == kLG - 1) {
                uint4 *o = out + (((uint64_t)lb[cv] + line) * kLG - gbase);
#pragma unroll
                for (int z = 0; z < kLG; ++z) o[z] = buf[cv * kLG + z];
            }
            nline = lc[cv] / kLG;
            bl[cv] = nline;  // every writer stores the same value
        }
        lds_barrier();
        if (live && !buffered && r / kLG == nline) buf[cv * kLG + (r & (kLG - 1))] = cd;
    }
    lds_barrier();
    // the last, partly filled line of each run, padded with inert descriptors
    for (uint32_t i = threadIdx.x; i < S; i += kBThreads) {
        const uint32_t k = lc[i];
        if (k & (kLG - 1)) {
            uint4 *o = out + (((uint64_t)lb[i] + k / kLG) * kLG - gbase);
#pragma unroll
            for (uint32_t z = 0; z < kLG; ++z) o[z] = z < (k & (kLG - 1)) ? buf[i * kLG + z] : make_uint4(0, 0, 0, 0);
        }
    }
}

// ---- C: per-partition LDS counting ----------------------------------------------------
// Deep coverage repeats every interior super-k-mer of a locus once per covering read, so a
// partition first collapses identical descriptors (LDS table keyed by all 128 bits), then
// expands each distinct one once, adding its multiplicity to every edge it holds. A
// partition with too many distinct descriptors (shallow data) is expanded from the raw
// descriptor stream instead; one with too many distinct edges for LDS goes to the
// global-table fallback.
#ifndef MCAAT_CTHREADS
#define MCAAT_CTHREADS 1024
#endif
constexpr int kCThreads = MCAAT_CTHREADS;
constexpr int kCWaves = kCThreads / 64;
constexpr int kCap = 4096;                                 // edge slots
constexpr int kCapMax = kCap * 85 / 100 - kCWaves * 64;    // distinct edges before giving up
constexpr int kDCap = 2048;                                // descriptor slots
constexpr int kDMax = kDCap * 3 / 4;                       // distinct descriptors before going raw
constexpr int kDProbe = 128;                               // probe bound of the descriptor table
#ifndef MCAAT_CB
#define MCAAT_CB 1
#endif
constexpr int kCB = MCAAT_CB;                              // descriptor loads in flight per thread
#ifndef MCAAT_CPF
#define MCAAT_CPF 1
#endif
constexpr bool kCPF = MCAAT_CPF != 0;                      // next round's loads issued before the probes
constexpr int kDefer = 64;                                 // descriptors with w0 == kEmpty before going raw
#ifndef MCAAT_CPERCU
#define MCAAT_CPERCU 2
#endif
constexpr int kCPerCu = MCAAT_CPERCU;                      // resident workgroups per CU (LDS, VGPR <= 64)
#ifndef MCAAT_CSPLIT
#define MCAAT_CSPLIT 2
#endif
constexpr uint32_t kSplitLg = MCAAT_CSPLIT;                // log2 classes of an overflowing partition (<= 3 spare hash bits)
static_assert(kSplitLg <= 3, "the sub-partition takes the top 11 of the 14 stored hash bits");
constexpr uint32_t kSplitMax = 3;                          // spare hash bits: deepest class split
#ifndef MCAAT_CRING
#define MCAAT_CRING 0
#endif
// collapse rounds in flight in an LDS-DMA ring (0: the register prefetch below). Measured and
// rejected (round 3, C3): a 2-round ring, 74.8 KB of LDS per workgroup, took pass C 56.4 -> 62.6 ms
constexpr int kCRing = MCAAT_CRING;
// one 16-B LDS-DMA per lane: lds is the wave-uniform base, lane i lands at lds + 16 i
// (inline asm: the compiler's own wait bookkeeping would otherwise drain every DMA before the
// next LDS access, vmcnt(0); the callers count their DMAs with wait_vm0 / wait_vm1)
__device__ __forceinline__ void dma16(const uint4 *src, uint4 *lds) {
    const uint32_t dst = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)lds);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_vm1() { asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); }
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// the deferred list only overflows on pathological T runs: those partitions go raw at once
__device__ __forceinline__ bool n_deferred_over(uint32_t n) { return n > (uint32_t)kDefer; }

// overflow-list entry: partition (24 bits), class (4), log2 class count (4)
__device__ __forceinline__ uint32_t ovf_part(uint32_t e) { return e & 0xFFFFFFu; }
__device__ __forceinline__ bool ovf_in_class(uint32_t e, uint32_t dw) {  // dw: descriptor word 3
    const uint32_t lgn = e >> 28, cls = (e >> 24) & 15;
    return ((dw >> (kHShift - 32)) & ((1u << lgn) - 1)) == cls;
}

// LG = log2 of the edge-table size
template <int LG>
__device__ __forceinline__ uint32_t edge_slot(uint64_t c) {
    return (((uint32_t)c ^ (uint32_t)(c >> 32)) * 0x9E3779B1u) >> (32 - LG);
}
// the error-rich variant (C2, C5: most partitions hold more distinct edges than kCapMax): an
// edge table twice the size, one 1024-thread workgroup per CU (96 KB of LDS)
constexpr int kCapBig = 8192;
constexpr int kCapMaxBig = kCapBig * 85 / 100 - kCWaves * 64;
// (round 4) the middle tier: 6144 slots (72 KB), still two 1024-thread workgroups per CU, for
// partitions of ~3-4K distinct edges (C5: ~3700) that overflow 4096 slots; slots are taken by a
// multiply-high of the hash (not a power of two)
constexpr int kCapMid = 6144;
constexpr int kCapMaxMid = kCapMid * 85 / 100 - kCWaves * 64;
constexpr int cap_lg(int cap) { return cap == 4096 ? 12 : cap == 8192 ? 13 : cap == kCapMid ? 0 : -1; }
template <int CAP>
__device__ __forceinline__ uint32_t edge_slot_n(uint64_t c) {
    if constexpr ((CAP & (CAP - 1)) == 0) {
        return edge_slot<cap_lg(CAP)>(c);
    } else {
        const uint32_t h = ((uint32_t)c ^ (uint32_t)(c >> 32)) * 0x9E3779B1u;
        return (uint32_t)(((uint64_t)h * (uint64_t)CAP) >> 32);
    }
}
// descriptor-table slots of an edge-table tier: the 8192-slot tier's 96-KB region holds a
// 4096-slot descriptor table (80 KB), so error-rich partitions (C5: ~2000 distinct descriptors)
// collapse in one pass instead of being re-read as four classes
constexpr int dcap_for(int cap) { return cap == kCapBig ? 2 * kDCap : kDCap; }
template <int DCAP>
__device__ __forceinline__ uint32_t desc_slot(uint64_t w0, uint64_t w1) {
    static_assert(DCAP == 2048 || DCAP == 4096, "11 or 12 slot bits");
    const uint64_t x = (w0 ^ (w1 * 0x9E3779B97F4A7C15ULL)) * 0xD6E8FEB86659FD93ULL;
    return (uint32_t)(x >> (64 - (DCAP == 4096 ? 12 : 11)));
}

template <bool PROF, int kCap, int PERCU>
__global__ void __launch_bounds__(kCThreads, PERCU * kCThreads / 256) k_lds_count(const uint4 *__restrict__ data, uint64_t gbase,
                                                         const uint64_t *__restrict__ fine_base, uint64_t p0,
                                                         uint64_t F, int E,
                                                         uint64_t *out_keys, uint32_t *out_cnt, uint64_t out_cap,
                                                         unsigned long long *out_cursor, uint32_t *ovf_list,
                                                         unsigned long long *ovf_n, uint32_t cap_max, uint32_t dmax,
                                                         unsigned long long *split_n, uint32_t split_first,
                                                         uint32_t split_max, unsigned long long *prof) {
    static_assert(cap_lg(kCap) >= 0, "edge table of 4096, 6144 or 8192 slots");
    constexpr int kDCap = dcap_for(kCap);  // descriptor slots of this tier
    // The descriptor table (phase 1) and the edge table (phases 2-3) share one LDS region:
    // between the phases each thread keeps its two descriptor slots in registers. 48 KB per
    // workgroup, so two 1024-thread workgroups share a CU and one's loads overlap the other's
    // LDS work.
    // With kCRing > 0 the collapse streams the partition through a ring of kCRing rounds of
    // descriptors placed after the descriptor table, filled by LDS-DMA (global_load_lds): the
    // loads of the next kCRing rounds are in flight without holding registers.
    constexpr int kEdgeBytes = kCap * 12, kDescBytes = kDCap * 20, kRingBytes = kCRing * kCThreads * 16;
    constexpr int kCollBytes = kDescBytes + kRingBytes;
    __shared__ __attribute__((aligned(16))) unsigned char region[kEdgeBytes > kCollBytes ? kEdgeBytes : kCollBytes];
    unsigned long long *const keys = (unsigned long long *)region;
    uint32_t *const cnt = (uint32_t *)(keys + kCap);
    unsigned long long *const dk0 = (unsigned long long *)region, *const dk1 = dk0 + kDCap;
    uint32_t *const dcnt = (uint32_t *)(dk1 + kDCap);  // > 0: the slot holds a descriptor
    // descriptors whose first word equals the empty marker (a run of >= 32 T) cannot be
    // keyed in the descriptor table; they wait here and are expanded with weight 1
    __shared__ uint4 deferred[kDefer];
    __shared__ uint32_t n_deferred;
    __shared__ uint32_t n_distinct, n_ddistinct;
    __shared__ int ovf, dovf;
    __shared__ uint32_t todo[16];
    __shared__ int ntodo;
    __shared__ uint32_t wsum[kCWaves];
    __shared__ unsigned long long obase;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // MCAAT_PROF_C=1: 100-MHz ticks per phase (clear, collapse, expand, emit) and counts of
    // partitions expanded raw
    unsigned long long tp[5] = {0, 0, 0, 0, 0}, t0 = PROF ? __builtin_amdgcn_s_memrealtime() : 0;
    auto tick = [&](int phase) {
        if (PROF) {
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            tp[phase] += t1 - t0;
            t0 = t1;
        }
    };

    // add weight to canonical edge c; false once the table has overflowed
    auto insert = [&](uint64_t c, uint32_t weight) {
        uint32_t h = edge_slot_n<kCap>(c);
        for (int probe = 0; probe < kCap; ++probe) {
            const unsigned long long cur = keys[h];
            if (cur == c) {
                atomicAdd(&cnt[h], weight);
                return;
            }
            if (cur == kEmpty) {
                const unsigned long long prev = atomicCAS(&keys[h], kEmpty, (unsigned long long)c);
                if (prev == kEmpty) {
                    atomicAdd(&cnt[h], weight);
                    if (atomicAdd(&n_distinct, 1u) + 1 > cap_max) ovf = 1;
                    return;
                }
                if (prev == c) {
                    atomicAdd(&cnt[h], weight);
                    return;
                }
            }
            h = h + 1 == (uint32_t)kCap ? 0 : h + 1;
        }
        ovf = 1;  // defensive: never spin on a full table
    };

    for (uint64_t p = p0 + blockIdx.x; p < F; p += gridDim.x) {
      // a partition whose distinct descriptors or edges overflow a table is counted again as
      // edge-disjoint classes (spare minimizer-hash bits: every occurrence of a canonical edge
      // carries the same minimizer), each collapsed, expanded and emitted alone
      // (round 4) the classes still to count, a stack of (cls | lgn << 4): a class that
      // overflows either table is split on its next spare hash bits — split_first bits the
      // first time, one bit after that — until split_max bits, past which an edge overflow goes to
      // the fallback and a descriptor overflow expands raw. Round 3 split once, 2^kSplitLg ways.
      if (threadIdx.x == 0) {
          todo[0] = 0;
          ntodo = 1;
      }
      __syncthreads();
      for (;;) {
        const int nt = ntodo;
        const uint32_t item = nt ? todo[nt - 1] : 0u;
        // every thread has read the top before thread 0 pops it (or, on an empty stack, before it
        // starts the next partition's)
        __syncthreads();
        if (nt == 0) break;
        const uint32_t cls = item & 15, lgn = item >> 4;
        const uint32_t cmask = (1u << lgn) - 1;
        // children of this class, pushed by thread 0 when it overflows (every thread has read
        // ntodo/todo: the clear below ends with a barrier before any push)
        auto split = [&]() {
            if (threadIdx.x == 0) {
                atomicAdd(split_n, 1ull);
                const uint32_t b = lgn == 0 ? split_first : 1u;
                for (uint32_t j = (1u << b); j-- > 0;) todo[ntodo++] = (cls + (j << lgn)) | ((lgn + b) << 4);
            }
        };
        for (int i = threadIdx.x; i < kDCap; i += kCThreads) {
            dk0[i] = dk1[i] = kEmpty;
            dcnt[i] = 0;
        }
        if (threadIdx.x == 0) {
            n_distinct = n_ddistinct = n_deferred = 0;
            ovf = dovf = 0;
            ntodo = nt - 1;  // popped
        }
        __syncthreads();
        tick(0);
        const uint64_t beg = fine_base[p] - gbase, end = fine_base[p + 1] - gbase;

        // ---- 1: collapse identical descriptors ----
        // wait-free: the two key words are claimed separately, each by a CAS from empty; a
        // lane moves on as soon as either word holds another value, so no lane ever waits on
        // another (a descriptor whose first word is the empty marker is deferred)
        auto collapse = [&](uint64_t w0, uint64_t w1) {
            if (((w1 >> kNShift) & 63) == 0) return;  // padding
            if (((uint32_t)(w1 >> kHShift) & cmask) != cls) return;  // another class
            if (w0 == kEmpty) {
                const uint32_t j = atomicAdd(&n_deferred, 1u);
                if (j < (uint32_t)kDefer)
                    deferred[j] = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
                else
                    dovf = 1;
                return;
            }
            uint32_t h = desc_slot<kDCap>(w0, w1);
            for (int probe = 0; probe < kDProbe; ++probe, h = (h + 1) & (kDCap - 1)) {
                unsigned long long k1 = dk1[h];
                if (k1 == kEmpty) {
                    k1 = atomicCAS(&dk1[h], kEmpty, (unsigned long long)w1);
                    if (k1 == kEmpty) {
                        k1 = w1;
                        if (atomicAdd(&n_ddistinct, 1u) + 1 > dmax) dovf = 1;
                    }
                }
                if (k1 != w1) continue;
                unsigned long long k0 = dk0[h];
                if (k0 == kEmpty) {
                    k0 = atomicCAS(&dk0[h], kEmpty, (unsigned long long)w0);
                    if (k0 == kEmpty) k0 = w0;
                }
                if (k0 != w0) continue;
                atomicAdd(&dcnt[h], 1u);
                return;
            }
            dovf = 1;
            if (PROF) atomicAdd(&prof[5], 1ull);
        };
        if constexpr (kCRing > 0) {
            // LDS-DMA ring: wave w's 64 lanes land round r's descriptors d0 + 64w .. in slot
            // r % kCRing (one 1-KB global_load_lds per wave); a lane reads back only its own
            // entry, so no barrier orders the waves, and each wave counts its own DMAs (vmcnt)
            uint4 *const ring = (uint4 *)(region + kDescBytes);
            auto issue = [&](uint64_t d0, int slot) {
                const uint64_t d = d0 + threadIdx.x;
                const uint4 *src = data + (d < end ? d : beg);  // in bounds; masked when read
                dma16(src, ring + slot * kCThreads + wave * 64);
            };
#pragma unroll
            for (int r = 0; r < kCRing; ++r)
                if (beg + (uint64_t)r * kCThreads < end) issue(beg + (uint64_t)r * kCThreads, r);
            int slot = 0;
            for (uint64_t d0 = beg; d0 < end; d0 += kCThreads) {
                if (__hip_atomic_load(&dovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                // DMAs issued after this round's (uniform): rounds d0+1 .. min(d0+kCRing-1, last)
                const uint64_t left = (end - d0 - 1) / kCThreads;  // rounds after this one
                if (left >= 1 && kCRing >= 2) wait_vm1(); else wait_vm0();
                const uint4 cq = ring[slot * kCThreads + threadIdx.x];
                const uint64_t d = d0 + threadIdx.x;
                if (left >= (uint64_t)kCRing) {
                    wait_lgkm0();  // the read has landed before the DMA may overwrite the slot
                    issue(d0 + (uint64_t)kCRing * kCThreads, slot);
                }
                if (d < end)
                    collapse((uint64_t)cq.x | ((uint64_t)cq.y << 32), (uint64_t)cq.z | ((uint64_t)cq.w << 32));
                slot = slot + 1 == kCRing ? 0 : slot + 1;
            }
            wait_vm0();  // no DMA may land in the region once it becomes the edge table
        } else {
        // kCB descriptors per thread per round: their loads are all in flight together, and
        // with kCPF the next round's are issued before this round's probes
        uint4 q[kCB];
        if (kCPF) {
#pragma unroll
            for (int k = 0; k < kCB; ++k) {
                const uint64_t d = beg + threadIdx.x + (uint64_t)k * kCThreads;
                q[k] = d < end ? data[d] : make_uint4(0, 0, 0, 0);
            }
        }
        for (uint64_t d0 = beg + threadIdx.x; d0 < end; d0 += (uint64_t)kCThreads * kCB) {
            if (__hip_atomic_load(&dovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
            uint4 cq[kCB];
#pragma unroll
            for (int k = 0; k < kCB; ++k) {
                if (kCPF) {
                    cq[k] = q[k];
                    const uint64_t d = d0 + (uint64_t)(k + kCB) * kCThreads;
                    q[k] = d < end ? data[d] : make_uint4(0, 0, 0, 0);
                } else {
                    const uint64_t d = d0 + (uint64_t)k * kCThreads;
                    cq[k] = d < end ? data[d] : make_uint4(0, 0, 0, 0);
                }
            }
#pragma unroll
            for (int k = 0; k < kCB; ++k)
                if (d0 + (uint64_t)k * kCThreads < end)
                    collapse((uint64_t)cq[k].x | ((uint64_t)cq[k].y << 32), (uint64_t)cq[k].z | ((uint64_t)cq[k].w << 32));
        }
        }
        __syncthreads();
        tick(1);
        if (dovf && lgn + (lgn == 0 ? split_first : 1u) <= split_max && !n_deferred_over(n_deferred)) {
            split();
            __syncthreads();  // every thread has read dovf and the stack before the next clear
            continue;
        }
        if (PROF && threadIdx.x == 0) {
            if (dovf) tp[4]++;
            atomicAdd(&prof[6], (unsigned long long)n_ddistinct);
            atomicAdd(&prof[7], (unsigned long long)(end - beg));
        }

        // ---- 2: expand into canonical edges ----
        // wave-level: the edges of the wave's 64 descriptors are spread over its lanes, each
        // added with its descriptor's multiplicity
        auto spread = [&](uint64_t w0, uint64_t w1, int n, uint32_t wgt) {
            int incl = n;
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(incl, o);
                if (lane >= o) incl += v;
            }
            const int total = __shfl(incl, 63);
            // all 64 lanes stay active through the shuffles (an inactive source lane reads 0)
            for (int b0 = 0; b0 < total; b0 += 64) {
                // checked every 64 edges (wave-uniform): after the flag is raised each wave
                // inserts at most 64 more keys, so the table (kCapMax + kCThreads < kCap)
                // always keeps a free slot and every probe terminates
                if (__hip_atomic_load(&ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                const int idx = b0 + lane;
                // owner lane: first lane whose inclusive prefix exceeds idx (6 uniform steps)
                int lo = 0;
#pragma unroll
                for (int step = 32; step > 0; step >>= 1)
                    if (__shfl(incl, lo + step - 1) <= idx) lo += step;
                const int src = lo > 63 ? 63 : lo;
                const int i = idx - (__shfl(incl, src) - __shfl(n, src));
                const uint64_t a0 = __shfl(w0, src), a1 = __shfl(w1, src);
                const uint32_t wt = __shfl(wgt, src);
                if (idx >= total) continue;
                insert(canon_edge(desc_window(a0, a1, i, E), E), wt);
            }
        };
        // the distinct descriptors move to registers (slots threadIdx.x + j * kCThreads), then
        // the region becomes the edge table
        constexpr int kSlots = kDCap / kCThreads;
        static_assert(kDCap % kCThreads == 0, "whole descriptor slots per thread");
        const bool raw = dovf;
        uint64_t r0[kSlots] = {}, r1[kSlots] = {};
        uint32_t rc[kSlots] = {};
        if (!raw) {
#pragma unroll
            for (int j = 0; j < kSlots; ++j) {
                const int i = threadIdx.x + j * kCThreads;
                rc[j] = dcnt[i];
                if (rc[j]) {
                    r0[j] = dk0[i];
                    r1[j] = dk1[i];
                }
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < kCap; i += kCThreads) {
            keys[i] = kEmpty;
            cnt[i] = 0;
        }
        __syncthreads();
        if (PROF && !raw) {  // expansion inserts: the distinct descriptors' edges
            unsigned long long ins = 0;
#pragma unroll
            for (int j = 0; j < kSlots; ++j) ins += rc[j] ? (r1[j] >> kNShift) & 63 : 0;
            for (int o = 32; o; o >>= 1) ins += __shfl_down(ins, o);
            if (lane == 0 && ins) atomicAdd(&prof[8], ins);
        }
        if (!raw) {
#pragma unroll
            for (int j = 0; j < kSlots; ++j) spread(r0[j], r1[j], (int)((r1[j] >> kNShift) & 63), rc[j]);
            if (wave == 0) {
                // n_deferred <= kDefer here (more sends the partition raw)
                const bool live = (uint32_t)lane < n_deferred;
                const uint4 q = live ? deferred[lane] : make_uint4(0, 0, 0, 0);
                const uint64_t w0 = (uint64_t)q.x | ((uint64_t)q.y << 32), w1 = (uint64_t)q.z | ((uint64_t)q.w << 32);
                spread(w0, w1, (int)((w1 >> kNShift) & 63), 1u);
            }
        } else {
            for (uint64_t d0 = beg + (uint64_t)wave * 64; d0 < end; d0 += kCThreads) {
                if (__hip_atomic_load(&ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                const uint64_t d = d0 + lane;
                uint64_t w0 = 0, w1 = 0;
                if (d < end) {
                    const uint4 q = data[d];
                    w0 = (uint64_t)q.x | ((uint64_t)q.y << 32);
                    w1 = (uint64_t)q.z | ((uint64_t)q.w << 32);
                    if (((uint32_t)(w1 >> kHShift) & cmask) != cls) w0 = w1 = 0;
                }
                spread(w0, w1, (int)((w1 >> kNShift) & 63), 1u);
            }
        }
        __syncthreads();
        tick(2);
        if (ovf) {
            // too many distinct edges for the LDS table: count the partition again as
            // edge-disjoint classes (shallow or error-rich data); a class that still overflows
            // goes to the global-table fallback
            if (lgn + (lgn == 0 ? split_first : 1u) <= split_max) {
                split();
            } else if (threadIdx.x == 0) {
                ovf_list[atomicAdd(ovf_n, 1ull)] = (uint32_t)p | (cls << 24) | (lgn << 28);
            }
            __syncthreads();
            continue;
        }
        if (PROF && threadIdx.x == 0) atomicAdd(&prof[9], (unsigned long long)n_distinct);
        // ---- 3: block-wide compaction of the occupied slots ----
        constexpr int per = kCap / kCThreads;
        int mine = 0;
        for (int j = 0; j < per; ++j) mine += keys[threadIdx.x * per + j] != kEmpty;
        int incl = mine;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (int w = 0; w < kCWaves; ++w) {
                const uint32_t v = wsum[w];
                wsum[w] = t;
                t += v;
            }
            obase = t ? atomicAdd(out_cursor, (unsigned long long)t) : 0;
        }
        __syncthreads();
        uint64_t o = obase + wsum[wave] + incl - mine;
        for (int j = 0; j < per; ++j) {
            const int s = threadIdx.x * per + j;
            const unsigned long long kk = keys[s];
            if (kk != kEmpty) {
                if (o < out_cap) {
                    out_keys[o] = kk;
                    out_cnt[o] = cnt[s];
                }
                ++o;
            }
        }
        __syncthreads();
        tick(3);
      }
    }
    if (PROF && (threadIdx.x & 63) == 0)
        for (int i = 0; i < 5; ++i) atomicAdd(&prof[i], tp[i]);
}

// ---- fallback: global open-addressing table for overflowing partitions ------------------
constexpr uint32_t kMaxProbe = 1u << 14;

struct __attribute__((aligned(16))) Slot {
    unsigned long long key1;  // key + 1 (0 = empty)
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

__global__ void __launch_bounds__(kBlock) k_part_occ(const uint4 *data, uint64_t gbase, const uint64_t *fine_base,
                                                     const uint32_t *parts, uint64_t np, uint64_t *occ) {
    for (uint64_t q = blockIdx.x; q < np; q += gridDim.x) {
        const uint32_t e = parts[q];
        const uint64_t p = ovf_part(e);
        unsigned long long acc = 0;
        for (uint64_t d = fine_base[p] - gbase + threadIdx.x; d < fine_base[p + 1] - gbase; d += blockDim.x) {
            const uint32_t dw = data[d].w;
            if (ovf_in_class(e, dw)) acc += (dw >> (kNShift - 32)) & 63;
        }
        __shared__ unsigned long long s;
        if (threadIdx.x == 0) s = 0;
        __syncthreads();
        block_add(&s, acc);
        __syncthreads();
        if (threadIdx.x == 0) occ[q] = s;
        __syncthreads();
    }
}

__global__ void __launch_bounds__(kBlock) k_fallback(const uint4 *data, uint64_t gbase, const uint64_t *fine_base,
                                                     const uint32_t *parts, uint64_t np, int E, Slot *tab,
                                                     uint64_t mask, unsigned long long *n_new, int *overflow) {
    for (uint64_t q = blockIdx.x; q < np; q += gridDim.x) {
        const uint32_t e = parts[q];
        const uint64_t p = ovf_part(e);
        for (uint64_t d = fine_base[p] - gbase + threadIdx.x; d < fine_base[p + 1] - gbase; d += blockDim.x) {
            const uint4 x = data[d];
            if (!ovf_in_class(e, x.w)) continue;
            const uint64_t w0 = (uint64_t)x.x | ((uint64_t)x.y << 32);
            const uint64_t w1 = (uint64_t)x.z | ((uint64_t)x.w << 32);
            const int n = (int)((w1 >> kNShift) & 63);
            for (int i = 0; i < n; ++i) table_insert(canon_edge(desc_window(w0, w1, i, E), E), tab, mask, n_new, overflow);
        }
    }
}

__global__ void __launch_bounds__(kBlock) k_fallback_emit(const Slot *tab, uint64_t cap, uint64_t *out_keys,
                                                          uint32_t *out_cnt, uint64_t out_cap,
                                                          unsigned long long *out_cursor) {
    const int lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < cap; base += stride) {
        const uint64_t i = base + threadIdx.x;
        const bool occ = i < cap && tab[i].key1 != 0;
        const unsigned long long m = __ballot(occ);
        unsigned long long off = 0;
        if (lane == 0 && m) off = atomicAdd(out_cursor, (unsigned long long)__popcll(m));
        off = __shfl(off, 0);
        if (occ) {
            const uint64_t o = off + __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
            if (o < out_cap) {
                out_keys[o] = tab[i].key1 - 1;
                out_cnt[o] = tab[i].cnt;
            }
        }
    }
}

__global__ void k_items_count(const uint64_t *offsets, uint64_t n_reads, int E, uint64_t *cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_reads; r += stride) {
        const uint64_t len = offsets[r + 1] - offsets[r];
        cnt[r] = len >= (uint64_t)E ? (len - E + 1 + kItem - 1) / kItem : 0;
    }
}

__global__ void k_items_fill(const uint64_t *offsets, uint64_t n_reads, int E, const uint64_t *start,
                             uint64_t *item_base, uint32_t *item_np) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_reads; r += stride) {
        const uint64_t len = offsets[r + 1] - offsets[r];
        if (len < (uint64_t)E) continue;
        const uint64_t npos = len - E + 1;
        uint64_t s = start[r];
        for (uint64_t c = 0; c * kItem < npos; ++c, ++s) {
            item_base[s] = offsets[r] + c * kItem;
            const uint64_t rem = npos - c * kItem;
            item_np[s] = (uint32_t)(rem < (uint64_t)kItem ? rem : kItem);
        }
    }
}

__global__ void k_sum_u32(const uint32_t *v, uint64_t n, unsigned long long *sum) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) acc += v[i];
    block_add(sum, acc);
}

template <class T>
void exclusive_scan(mcaat_ctx *ctx, const T *in, T *out, uint64_t n) {
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, (size_t)n, ctx->stream));
    DevBuf<uint8_t> t(tmp);
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(t.p, tmp, in, out, (size_t)n, ctx->stream));
}

}  // namespace

// MCAAT_VERBOSE=1: host wall-clock marks of the sub-stages on stderr (stream-synchronised)
void verbose_mark(mcaat_ctx *ctx, const char *what) {
    static const bool on = getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1';
    static double last = 0;
    if (!on) return;
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    const double pre = ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
    (void)hipStreamSynchronize(ctx->stream);
    clock_gettime(CLOCK_MONOTONIC, &ts);
    const double now = ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
    fprintf(stderr, "[mcaat] %-28s %10.2f ms (sync %.2f)\n", what, last ? now - last : 0.0, now - pre);
    last = now;
}

// fine partitions: ~8K edge occurrences each (8 L1 bits + l2_bits), so that even at ~5x
// coverage (a rank's share of a sharded dataset) a partition's distinct edges fit the LDS
// table; deep data reaches the 2^19 cap long before (C3: 70K occurrences each, ~1K distinct
// descriptors after the collapse)
int nc_fine_bits(mcaat_ctx *ctx, uint64_t n_occ) {
    int fine_bits = 0;
    while ((1ULL << (fine_bits + 1)) * 8192ULL <= n_occ) ++fine_bits;
    fine_bits = (int)knob(ctx, "nc.fine_bits", fine_bits);
    return std::max(8, std::min(19, fine_bits));  // l2_bits <= 11: k_l2_scatter's line buffers
}

// pass A's minimizer parameters for k (every pass A launch for k uses the same)
SkParams sk_params(int k) {
    const int E = k + 1;
    SkParams P;
    P.E = E;
    // long minimizers (near-unique per genome locus) keep the per-partition load uniform;
    // short ones (m=11) concentrate thousands of distinct edges on small-hash m-mers
    P.m = std::max(3, std::min(16, E - 8));  // <= 16: the m-mer machinery is 32-bit
    // longer windows mean longer super-k-mers (fewer descriptors to write, partition and
    // collapse); m >= 14 keeps minimizers near-unique per locus. k=27: W 13 -> 15 (m 14)
    // took node_counter 201 -> 194 ms at C3 (pass C splits the partitions that then overflow
    // the descriptor table into edge-disjoint classes)
    if (E >= 22) P.m = std::max(14, std::min(16, E - 14));
    if (const char *e = getenv("MCAAT_MINI_W")) {  // A/B knob: minimizer window (m-mers per edge)
        const int wt = atoi(e);
        if (wt >= 1 && wt <= 16) P.m = std::max(3, std::min(16, E - wt + 1));
    }
    if (P.m > E) P.m = E;
    P.w = E - P.m + 1;
    if (P.w > 16) throw Error(MCAAT_E_INVALID, "node_counter: minimizer window above 16");
    P.nmax = kDescBases - E + 1;
    P.salt = 0x6d696e696d697aULL;
    P.mini = kMiniOne;

    return P;
}

void node_counter(mcaat_ctx *ctx, const mcaat_reads *r, int k, CountResult &out) {
    NcBuckets b;
    if (r->ahead && r->ahead_k == k) {  // pass A ran while the input was read (nc_ahead_*)
        b = std::move(*r->ahead);
        r->ahead.reset();
        verbose_mark(ctx, "node_counter.A_ahead");
    } else {
        node_counter_a(ctx, r, k, nullptr, b);
    }
    node_counter_bc(ctx, b, k, out);
}

// pass A: the reads' super-k-mer descriptors in 256 L1 buckets. The fine-partition bits come
// from the reads' edge occurrences (nc_fine_bits), or from pick(occurrences) when given: a
// sharded build derives them from the sum over its ranks (pick is collective, called once on
// every rank), because the sub rows written here depend on them.
void node_counter_a(mcaat_ctx *ctx, const mcaat_reads *r, int k, const std::function<int(uint64_t)> &pick,
                    NcBuckets &bk) {
    verbose_mark(ctx, "node_counter.begin");
    const int E = k + 1;
    hipStream_t st = ctx->stream;
    SkParams P = sk_params(k);
    // work items (<= kItem edge positions each)
    ItemSrc src{};
    src.offsets = r->offsets.p;
    src.n_reads = r->n_reads;
    DevBuf<uint64_t> item_base;
    DevBuf<uint32_t> item_np;
    uint64_t n_occ = 0, n_items = 0;
    if (r->fixed_len) {
        src.fixed_len = r->fixed_len;
        const uint64_t npos = r->fixed_len >= (uint64_t)E ? r->fixed_len - E + 1 : 0;
        src.ipr = (npos + kItem - 1) / kItem;
        n_items = r->n_reads * src.ipr;
        n_occ = r->n_reads * npos;
        if (!npos) {
            src.fixed_len = 0;
            src.n_items = 0;
        }
    } else if (r->n_reads) {
        DevBuf<uint64_t> cnt(r->n_reads + 1), start(r->n_reads + 1);
        HIP_OK(hipMemsetAsync(cnt.p, 0, cnt.bytes(), st));
        hipLaunchKernelGGL(k_items_count, dim3(grid_for(r->n_reads, kBlock)), dim3(kBlock), 0, st, r->offsets.p,
                           r->n_reads, E, cnt.p);
        LAUNCH_OK();
        exclusive_scan(ctx, cnt.p, start.p, r->n_reads + 1);
        HIP_OK(hipMemcpyAsync(&n_items, start.p + r->n_reads, 8, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        item_base.alloc(n_items);
        item_np.alloc(n_items);
        hipLaunchKernelGGL(k_items_fill, dim3(grid_for(r->n_reads, kBlock)), dim3(kBlock), 0, st, r->offsets.p,
                           r->n_reads, E, start.p, item_base.p, item_np.p);
        LAUNCH_OK();
        {  // occurrences = sum of the items' positions (reduced on the device)
            DevBuf<unsigned long long> socc(1);
            HIP_OK(hipMemsetAsync(socc.p, 0, 8, st));
            hipLaunchKernelGGL(k_sum_u32, dim3(grid_for(n_items, kBlock, (unsigned)ctx->n_cu * 8)), dim3(kBlock), 0, st,
                               item_np.p, n_items, socc.p);
            LAUNCH_OK();
            unsigned long long h = 0;
            HIP_OK(hipMemcpyAsync(&h, socc.p, 8, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            n_occ = h;
        }
        src.item_base = item_base.p;
        src.item_np = item_np.p;
        src.n_items = n_items;
    }
    const int fine_bits = pick ? pick(n_occ) : nc_fine_bits(ctx, n_occ);
    P.l2_bits = fine_bits - 8;
    if (pick) P.mini = kMiniShard;  // a rank of a sharded build
    if (knob_set(ctx, "nc.a_mini")) P.mini = (uint32_t)std::max<int64_t>(8, knob(ctx, "nc.a_mini", 1024)) & ~7u;
    bk.l2_bits = P.l2_bits;
    bk.n_occ = n_occ;
    bk.regions.assign(256, {});
    if (n_occ == 0) {
        bk.data.alloc(1);
        bk.sub.alloc(8);
        return;
    }

    // ---- A ----
    // expected descriptors: density 2/(w+1) per edge + one per item, with headroom
    const double dens = 2.0 / (P.w + 1);
    uint64_t est = (uint64_t)(1.08 * (dens * (double)n_occ + (double)n_items)) + 4096;
    std::vector<uint64_t> cap(256), base(257);
    // + one partially used reservation per (workgroup, bucket)
    const uint64_t a_grid = (uint64_t)kAPerCu * ctx->n_cu;
    for (int b = 0; b < 256; ++b) cap[b] = (est / 256 + 2 * a_grid * P.mini + 7) & ~7ull;  // 16-B aligned sub rows
    if (const int64_t fixed = knob(ctx, "nc.l1_slots", 0))  // test knob: undersize -> resize and re-run
        for (int b = 0; b < 256; ++b) cap[b] = ((uint64_t)fixed + 7) & ~7ull;
    DevBuf<uint64_t> dcap(256), dbase(257);
    DevBuf<unsigned long long> dcur(256);
    DevBuf<uint4> &l1 = bk.data;
    DevBuf<uint16_t> &l1s = bk.sub;
    std::vector<unsigned long long> tot(256);
    static const bool prof_a = getenv("MCAAT_PROF_A") && getenv("MCAAT_PROF_A")[0] == '1';
    DevBuf<unsigned long long> dprof(8);
    if (prof_a) HIP_OK(hipMemsetAsync(dprof.p, 0, dprof.bytes(), st));
    for (int attempt = 0;; ++attempt) {
        base[0] = 0;
        for (int b = 0; b < 256; ++b) base[b + 1] = base[b] + cap[b];
        l1.alloc(base[256]);
        l1s.alloc(base[256]);
        HIP_OK(hipMemcpyAsync(dcap.p, cap.data(), 8 * 256, hipMemcpyHostToDevice, st));
        HIP_OK(hipMemcpyAsync(dbase.p, base.data(), 8 * 257, hipMemcpyHostToDevice, st));
        HIP_OK(hipMemsetAsync(dcur.p, 0, dcur.bytes(), st));
        {
            KernelTimer kt(ctx, "sk_scatter", 0.0);  // bytes added below, once the descriptor count is known
            hipLaunchKernelGGL(sk_kernel(P.w, P.m == 16), dim3((unsigned)a_grid), dim3(kAThreads), 0, st, r->packed.p, src, P, l1.p,
                               dbase.p, dcap.p, dcur.p, l1s.p, prof_a ? dprof.p : nullptr, nullptr, 0);
            LAUNCH_OK();
            kt.stop();
        }
        HIP_OK(hipMemcpyAsync(tot.data(), dcur.p, 8 * 256, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        bool ok = true;
        for (int b = 0; b < 256; ++b)
            if (tot[b] > cap[b]) ok = false;
        if (ok) break;
        if (attempt > 0) throw Error(MCAAT_E_CAPACITY, "node_counter: L1 bucket sizing failed");
        for (int b = 0; b < 256; ++b) cap[b] = (tot[b] + 8) & ~7ull;  // exact on the second run (cursors count every grab)
    }
    uint64_t n_desc = 0;
    bk.base = base;
    for (int b = 0; b < 256; ++b) {
        n_desc += tot[b];
        if (tot[b]) bk.regions[b].push_back({base[b], tot[b]});  // tot: whole reservations
    }
    // algorithmic bytes of the launch: the 2-bit stream read once, a 16-B descriptor and its
    // 2-B sub row written per reserved slot (the tail slots of a reservation are written inert)
    ctx->kstats["sk_scatter"].total_bytes += 0.25 * (double)r->n_bases + 18.0 * (double)n_desc;
    if (prof_a) {
        unsigned long long hp[8];
        HIP_OK(hipMemcpy(hp, dprof.p, 64, hipMemcpyDeviceToHost));
        const double waves = (double)a_grid * kAWaves;
        fprintf(stderr, "[mcaat] pass A per-wave ms (100 MHz clock): scan %.1f bucket %.1f wait %.1f reserve %.1f write %.1f\n",
                hp[0] / waves / 1e5, hp[1] / waves / 1e5, hp[2] / waves / 1e5, hp[3] / waves / 1e5, hp[4] / waves / 1e5);
    }
    verbose_mark(ctx, "node_counter.A");
}

// ---- pass A on a streamed input (mcaat_count_ahead) -------------------------------------
// The host FASTQ packer uploads its parts one by one while it reads; pass A runs on each part
// as soon as it is in HBM, on the side stream, so by the time the last part lands only that
// part's pass A is left. Every launch has the same grid and keeps its workgroups' L1
// reservations in `state` for the next one (k_sk_scatter rmode), so the parts fill the
// buckets as one launch over the whole input would (no inert slots between launches). The
// buckets are sized from an estimate of the input's edge occurrences made before the read; if
// one overflows (or a part's reads are not all of the sampled length) the result is dropped
// and the count runs pass A on the concatenated reads as usual.
struct NcAhead {
    mcaat_ctx *ctx = nullptr;
    int k = 0;
    SkParams P{};
    uint64_t a_grid = 0;
    std::vector<uint64_t> cap, base;
    DevBuf<uint64_t> dcap, dbase;
    DevBuf<unsigned long long> dcur, state;
    std::shared_ptr<NcBuckets> bk;
    std::mutex mu;
    int launches = 0;
    bool failed = false, ended = false;
    uint64_t n_occ = 0;
    ~NcAhead() {
        if (ctx && !ended) (void)hipStreamSynchronize(ctx->side);  // launches may still read the parts
    }
};

static_assert(kItem == kNcItem, "the packer's item estimate uses pass A's item length");

std::shared_ptr<NcAhead> nc_ahead_begin(mcaat_ctx *ctx, int k, uint64_t n_occ_est, uint64_t n_items_est) {
    auto a = std::make_shared<NcAhead>();
    a->ctx = ctx;
    a->k = k;
    a->P = sk_params(k);
    a->P.l2_bits = nc_fine_bits(ctx, n_occ_est) - 8;
    if (knob_set(ctx, "nc.a_mini")) a->P.mini = (uint32_t)std::max<int64_t>(8, knob(ctx, "nc.a_mini", 1024)) & ~7u;
    a->bk = std::make_shared<NcBuckets>();
    a->bk->l2_bits = a->P.l2_bits;
    a->a_grid = (uint64_t)kAPerCu * ctx->n_cu;
    // node_counter_a's sizing, with more headroom for the estimate
    const double dens = 2.0 / (a->P.w + 1);
    const uint64_t est = (uint64_t)(1.12 * (dens * (double)n_occ_est + (double)n_items_est)) + 4096;
    a->cap.assign(256, 0);
    a->base.assign(257, 0);
    for (int b = 0; b < 256; ++b) {
        a->cap[b] = (est / 256 + 2 * a->a_grid * a->P.mini + 7) & ~7ull;
        if (const int64_t fixed = knob(ctx, "nc.l1_slots", 0)) a->cap[b] = ((uint64_t)fixed + 7) & ~7ull;
        a->base[b + 1] = a->base[b] + a->cap[b];
    }
    a->bk->data.alloc(a->base[256]);
    a->bk->sub.alloc(a->base[256]);
    a->dcap.alloc(256);
    a->dbase.alloc(257);
    a->dcur.alloc(256);
    a->state.alloc(a->a_grid * 256 * 3);
    h2d(ctx, a->dcap.p, a->cap.data(), 8 * 256);
    h2d(ctx, a->dbase.p, a->base.data(), 8 * 257);
    HIP_OK(hipMemsetAsync(a->dcur.p, 0, a->dcur.bytes(), ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));  // the side stream's launches read these
    return a;
}

// pass A over one uploaded part: n_reads reads of L bases from word 0 of `packed`
void nc_ahead_part(NcAhead &a, const uint64_t *packed, uint64_t n_reads, uint64_t L) {
    const int E = a.k + 1;
    std::lock_guard<std::mutex> g(a.mu);
    if (a.failed || !n_reads || L < (uint64_t)E) return;
    ItemSrc src{};
    src.n_reads = n_reads;
    src.fixed_len = L;
    const uint64_t npos = L - E + 1;
    src.ipr = (npos + kItem - 1) / kItem;
    a.n_occ += n_reads * npos;
    hipLaunchKernelGGL(sk_kernel(a.P.w, a.P.m == 16), dim3((unsigned)a.a_grid), dim3(kAThreads), 0, a.ctx->side, packed,
                       src, a.P, a.bk->data.p, (const uint64_t *)a.dbase.p, (const uint64_t *)a.dcap.p, a.dcur.p,
                       a.bk->sub.p, nullptr, a.state.p, a.launches ? 2 : 1);
    LAUNCH_OK();
    ++a.launches;
}

void nc_ahead_fail(NcAhead &a) {
    std::lock_guard<std::mutex> g(a.mu);
    a.failed = true;
}

// the last launch (no reads: it fills what is left of the reservations), then the buckets, or
// null when the run failed
std::shared_ptr<NcBuckets> nc_ahead_end(NcAhead &a) {
    std::lock_guard<std::mutex> g(a.mu);
    mcaat_ctx *ctx = a.ctx;
    std::vector<unsigned long long> tot(256, 0);
    if (!a.failed) {
        ItemSrc src{};
        hipLaunchKernelGGL(sk_kernel(a.P.w, a.P.m == 16), dim3((unsigned)a.a_grid), dim3(kAThreads), 0, ctx->side,
                           (const uint64_t *)a.bk->data.p, src, a.P, a.bk->data.p, (const uint64_t *)a.dbase.p,
                           (const uint64_t *)a.dcap.p, a.dcur.p, a.bk->sub.p, nullptr, a.state.p, a.launches ? 3 : 0);
        LAUNCH_OK();
        HIP_OK(hipMemcpyAsync(tot.data(), a.dcur.p, 8 * 256, hipMemcpyDeviceToHost, ctx->side));
    }
    HIP_OK(hipStreamSynchronize(ctx->side));
    a.ended = true;
    for (int b = 0; b < 256 && !a.failed; ++b)
        if (tot[b] > a.cap[b]) a.failed = true;
    if (a.failed) return nullptr;
    NcBuckets &bk = *a.bk;
    bk.n_occ = a.n_occ;
    bk.base = a.base;
    bk.regions.assign(256, {});
    uint64_t n_desc = 0;
    for (int b = 0; b < 256; ++b) {
        n_desc += tot[b];
        if (tot[b]) bk.regions[b].push_back({a.base[b], tot[b]});
    }
    ctx->kstats["sk_scatter_ahead"].launches += a.launches + 1;
    ctx->kstats["sk_scatter_ahead"].total_bytes += 18.0 * (double)n_desc;
    if (!a.n_occ) {  // node_counter_a's empty-input buckets
        bk.data.alloc(1);
        bk.sub.alloc(8);
    }
    return a.bk;
}

// passes B and C over the L1 buckets' regions (a bucket may hold several, e.g. one per rank
// after a sharded build's descriptor exchange): final canonical counts of their edges
void node_counter_bc(mcaat_ctx *ctx, NcBuckets &bk, int k, CountResult &out) {
    const int E = k + 1;
    hipStream_t st = ctx->stream;
    out.n = 0;
    uint64_t n_desc = 0;
    for (const auto &v : bk.regions)
        for (const auto &rg : v) n_desc += rg.second;
    if (n_desc == 0) {
        out.keys.alloc(1);
        out.counts.alloc(1);
        return;
    }
    const uint64_t n_occ = bk.n_occ;
    DevBuf<uint4> &l1 = bk.data;
    DevBuf<uint16_t> &l1s = bk.sub;
    SkParams P;
    P.l2_bits = bk.l2_bits;
    const uint32_t S = 1u << P.l2_bits;
    const uint64_t F = 256ull * S;
    DevBuf<unsigned long long> dprof(10);

    // ---- B + C, over groups of L1 buckets whose fine partitions fit a memory budget ----
    // The sub histogram of every chunk gives all fine-partition offsets at once; each group
    // then scatters its buckets into a buffer of its own and counts them, so the peak
    // footprint is the L1 buckets plus one group's fine partitions.
    std::vector<uint64_t> cstart;
    std::vector<uint32_t> clen, cbucket;
    std::vector<uint64_t> bchunk(257, 0);  // first chunk of each bucket
    for (int b = 0; b < 256; ++b) {
        bchunk[b] = cstart.size();
        for (const auto &rg : bk.regions[b])
            for (uint64_t o = 0; o < rg.second; o += kChunk) {
                cstart.push_back(rg.first + o);
                clen.push_back((uint32_t)std::min<uint64_t>(kChunk, rg.second - o));
                cbucket.push_back((uint32_t)b);
            }
    }
    bchunk[256] = cstart.size();
    const uint64_t nch = cstart.size();
    DevBuf<uint64_t> dcs(nch ? nch : 1), dfine(F + 1);
    DevBuf<unsigned long long> dtot(F + 1);
    DevBuf<uint32_t> dcl(nch ? nch : 1), dcb(nch ? nch : 1);
    HIP_OK(hipMemcpyAsync(dcs.p, cstart.data(), 8 * nch, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(dcl.p, clen.data(), 4 * nch, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(dcb.p, cbucket.data(), 4 * nch, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(dtot.p, 0, dtot.bytes(), st));
    std::vector<uint64_t> hfine(F + 1);
    DevBuf<uint32_t> druns(nch * S ? nch * S : 1);  // per chunk and sub: count, then run start (lines)
    {
        KernelTimer kt(ctx, "l2_hist", 2.0 * (double)n_desc);
        if (nch) {
            hipLaunchKernelGGL(k_l2_hist, dim3((unsigned)nch), dim3(kBThreads), 4 * S, st, l1s.p, dcs.p, dcl.p, dcb.p,
                               P.l2_bits, dtot.p, druns.p);
            LAUNCH_OK();
        }
        exclusive_scan(ctx, (const uint64_t *)dtot.p, dfine.p, F + 1);
        d2h(ctx, hfine.data(), dfine.p, 8 * (F + 1));
        if (hfine[F] / kLG >= (1ull << 32)) throw Error(MCAAT_E_CAPACITY, "node_counter: 2^32 or more fine-partition lines");
        if (nch) {
            DevBuf<uint64_t> dbch(257);
            HIP_OK(hipMemcpyAsync(dbch.p, bchunk.data(), 8 * 257, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_chunk_runs, dim3(grid_for(256ull * S, 256)), dim3(256), 0, st, druns.p,
                               (const uint64_t *)dbch.p, (const uint64_t *)dfine.p, S);
            LAUNCH_OK();
            HIP_OK(hipStreamSynchronize(st));  // dbch is freed on scope exit
        }
        kt.stop();
    }
    const uint64_t n_live = hfine[F];
    verbose_mark(ctx, "node_counter.B_hist");

    uint64_t out_cap = (uint64_t)knob(ctx, "nc.out_cap", (int64_t)std::max<uint64_t>(n_occ / 32, 1u << 20));
    if (out_cap < 1) out_cap = 1;
    out.keys.alloc(out_cap);
    out.counts.alloc(out_cap);
    DevBuf<unsigned long long> dcnt(4);
    HIP_OK(hipMemsetAsync(dcnt.p, 0, dcnt.bytes(), st));
    DevBuf<uint32_t> ovf_list(F << kSplitMax);  // one entry per (partition, class)
    static const bool prof_c = getenv("MCAAT_PROF_C") && getenv("MCAAT_PROF_C")[0] == '1';
    if (prof_c) HIP_OK(hipMemsetAsync(dprof.p, 0, dprof.bytes(), st));
    const uint64_t group_budget =
        (uint64_t)knob(ctx, "nc.group_budget", (int64_t)std::max<uint64_t>(n_live / 4 + 1, 1ULL << 28));  // descriptors per group
    const uint32_t cap_max = (uint32_t)std::min<int64_t>(kCapMax, std::max<int64_t>(1, knob(ctx, "nc.edge_cap", kCapMax)));
    const uint32_t cap_max_big = (uint32_t)std::min<int64_t>(kCapMaxBig, std::max<int64_t>(1, knob(ctx, "nc.edge_cap", kCapMaxBig)));
    const uint32_t cap_max_mid = (uint32_t)std::min<int64_t>(kCapMaxMid, std::max<int64_t>(1, knob(ctx, "nc.edge_cap", kCapMaxMid)));
    // larger edge tables: tier 0 = 4096 slots, 1 = 6144 (two workgroups per CU), 2 = 8192 (one).
    // knob nc.big_table fixes the tier (0, 1 = 8192 as in round 3, 2 = 6144); default: from the
    // next group on, 8192 slots once a group split more than 1 in 8 of its partitions into
    // classes (error-rich data)
    const int64_t big_knob = knob(ctx, "nc.big_table", -1);
    int tier = big_knob == 1 ? 2 : big_knob == 2 ? 1 : 0;
    const uint32_t dmax = (uint32_t)std::min<int64_t>(kDMax, std::max<int64_t>(1, knob(ctx, "nc.desc_cap", kDMax)));
    constexpr int kDMaxBig = dcap_for(kCapBig) * 3 / 4;
    // bits of a partition's first class split: round 3's four-way split in the 4096-slot tier (C2:
    // partitions far over it); two-way in the 8192-slot tier, whose overflowing partitions (C5)
    // are mostly just over it, so halves fit and each re-read is half as many passes
    const uint32_t split_first = (uint32_t)std::min<int64_t>(kSplitMax, std::max<int64_t>(1, knob(ctx, "nc.split_first", kSplitLg)));
    const uint32_t split_big = (uint32_t)std::min<int64_t>(kSplitMax, std::max<int64_t>(1, knob(ctx, "nc.split_first", 1)));
    const uint32_t split_max = (uint32_t)std::min<int64_t>(kSplitMax, std::max<int64_t>(1, knob(ctx, "nc.split_max", kSplitMax)));
    const uint32_t dmax_big = (uint32_t)std::min<int64_t>(kDMaxBig, std::max<int64_t>(1, knob(ctx, "nc.desc_cap", kDMaxBig)));
    // groups of L1 buckets; with the overlap knob (default on) group g+1's pass B runs on the
    // side stream while group g's pass C counts on the main stream (two groups' fine
    // partitions alive at once, so groups are half the size)
    const bool overlap = knob(ctx, "nc.overlap", 1) != 0;
    const bool free_sync = knob(ctx, "nc.free_sync", 0) != 0;
    struct Group {
        int b0, b1;
        DevBuf<uint4> fine;
        hipEvent_t done = nullptr;
    };
    std::vector<Group> groups;
    for (int b0 = 0; b0 < 256;) {
        int b1 = b0 + 1;
        uint64_t gb = overlap && !knob_set(ctx, "nc.group_budget") ? group_budget / 2 + 1 : group_budget;
        // the first group is a small probe: the edge-table tier is chosen from its class splits,
        // so on error-rich data only 1/16 of the descriptors take the re-read of a split
        if (b0 == 0 && big_knob < 0 && !knob_set(ctx, "nc.group_budget")) gb = gb / 8 + 1;
        while (b1 < 256 && hfine[(uint64_t)(b1 + 1) * S] - hfine[(uint64_t)b0 * S] <= gb) ++b1;
        groups.push_back(Group{b0, b1, {}, nullptr});
        b0 = b1;
    }
    if (overlap && !ctx->side) HIP_OK(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
    hipStream_t sb = overlap ? ctx->side : st;
    if (overlap) {  // the side stream starts after everything queued so far (pass A, offsets)
        hipEvent_t ev = event_get(ctx);
        HIP_OK(hipEventRecord(ev, st));
        HIP_OK(hipStreamWaitEvent(sb, ev, 0));
        event_put(ctx, ev);
    }
    std::vector<KernelTimer *> btimers;
    auto launch_b = [&](Group &g) {
        const uint64_t p0 = (uint64_t)g.b0 * S, p1 = (uint64_t)g.b1 * S;
        const uint64_t gbase = hfine[p0], gn = hfine[p1] - gbase;
        const uint64_t c0 = bchunk[g.b0], c1 = bchunk[g.b1];
        {
            AllocStreamScope scope(sb);  // written by pass B on the side stream
            g.fine.alloc(gn ? gn : 1);
        }
        auto *kt = new KernelTimer(ctx, "l2_partition", 34.0 * (double)gn, sb);  // sub rows + descriptors read, descriptors written
        if (c1 > c0) {
            hipLaunchKernelGGL(k_l2_scatter, dim3((unsigned)(c1 - c0)), dim3(kBThreads), 0, sb, l1.p, l1s.p,
                               dcs.p + c0, dcl.p + c0, (const uint32_t *)druns.p + c0 * S, P.l2_bits, g.fine.p, gbase);
            LAUNCH_OK();
        }
        kt->mark();
        g.done = event_get(ctx);
        HIP_OK(hipEventRecord(g.done, sb));
        btimers.push_back(kt);
    };
    struct TimerGuard {  // timers of launched B passes, freed on every exit
        std::vector<KernelTimer *> &v;
        ~TimerGuard() { for (auto *t : v) delete t; }
    } tguard{btimers};
    uint64_t n_out = 0;
    if (!groups.empty()) launch_b(groups[0]);
    for (size_t gi = 0; gi < groups.size(); ++gi) {
        Group &grp = groups[gi];
        const int b0 = grp.b0, b1 = grp.b1;
        const uint64_t p0 = (uint64_t)b0 * S, p1 = (uint64_t)b1 * S;
        const uint64_t gbase = hfine[p0], gn = hfine[p1] - gbase;
        HIP_OK(hipStreamWaitEvent(st, grp.done, 0));
        // the next group's partitioning overlaps this group's counting
        if (overlap && gi + 1 < groups.size()) launch_b(groups[gi + 1]);
        DevBuf<uint4> &fine = grp.fine;
        // C; a group whose output overflows the key buffers is counted again after they grow
        for (int attempt = 0;; ++attempt) {
            HIP_OK(hipMemsetAsync(dcnt.p + 1, 0, 16, st));
            {
                KernelTimer kt(ctx, "lds_count", 16.0 * (double)gn);
                const unsigned wg = (unsigned)std::min<uint64_t>(p1 - p0, (uint64_t)(tier == 2 ? 1 : kCPerCu) * ctx->n_cu);
                auto kern = tier == 2 ? (prof_c ? k_lds_count<true, kCapBig, 1> : k_lds_count<false, kCapBig, 1>)
                          : tier == 1 ? (prof_c ? k_lds_count<true, kCapMid, kCPerCu> : k_lds_count<false, kCapMid, kCPerCu>)
                                : (prof_c ? k_lds_count<true, kCap, kCPerCu> : k_lds_count<false, kCap, kCPerCu>);
                hipLaunchKernelGGL(kern, dim3(wg), dim3(kCThreads), 0, st, fine.p, gbase, dfine.p, p0, p1, E, out.keys.p,
                                   out.counts.p, out_cap, dcnt.p, ovf_list.p, dcnt.p + 1,
                                   tier == 2 ? cap_max_big : tier == 1 ? cap_max_mid : cap_max, tier == 2 ? dmax_big : dmax,
                                   dcnt.p + 2, tier == 2 ? split_big : split_first, split_max, prof_c ? dprof.p : nullptr);
                LAUNCH_OK();
                kt.stop();
            }
            unsigned long long hc[3];
            HIP_OK(hipMemcpyAsync(hc, dcnt.p, 24, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            const uint64_t n_ovf = hc[1];
            ctx->kstats["lds_count_split_partitions"].launches += hc[2];
            // measured at C5: the 6144-slot tier still splits more than 1 in 8 partitions (183.6 ms
            // of pass C either way), so the default goes straight to 8192 slots
            if (big_knob < 0 && tier < 2 && hc[2] * 8 > p1 - p0) tier = 2;
            ctx->kstats["lds_count_overflow_partitions"].launches += n_ovf;
            if (n_ovf) {
                // global-table fallback for the partitions whose distinct edges overflowed LDS,
                // in batches whose table fits a fixed memory budget
                DevBuf<uint64_t> occ(n_ovf);
                hipLaunchKernelGGL(k_part_occ, dim3((unsigned)std::min<uint64_t>(n_ovf, 65536)), dim3(kBlock), 0, st,
                                   fine.p, gbase, dfine.p, ovf_list.p, n_ovf, occ.p);
                LAUNCH_OK();
                std::vector<uint64_t> occ_h(n_ovf);
                std::vector<uint32_t> parts_h(n_ovf);
                d2h(ctx, occ_h.data(), occ.p, 8 * n_ovf);
                d2h(ctx, parts_h.data(), ovf_list.p, 4 * n_ovf);
                const uint64_t budget =
                    (uint64_t)std::max<int64_t>(1, knob(ctx, "nc.fallback_budget", 1LL << 30));  // occurrences per batch (table <= 32 GB)
                DevBuf<unsigned long long> nn(1);
                DevBuf<int> dover(1);
                DevBuf<uint32_t> dparts(n_ovf);
                for (uint64_t q0 = 0; q0 < n_ovf;) {
                    uint64_t q1 = q0, occ_b = 0;
                    while (q1 < n_ovf && (q1 == q0 || occ_b + occ_h[q1] <= budget)) occ_b += occ_h[q1++];
                    HIP_OK(hipMemcpyAsync(dparts.p, parts_h.data() + q0, 4 * (q1 - q0), hipMemcpyHostToDevice, st));
                    uint64_t tcap = next_pow2(occ_b + occ_b / 2 + 1024);
                    for (;;) {
                        DevBuf<Slot> tab(tcap);
                        HIP_OK(hipMemsetAsync(tab.p, 0, tab.bytes(), st));
                        HIP_OK(hipMemsetAsync(nn.p, 0, 8, st));
                        HIP_OK(hipMemsetAsync(dover.p, 0, 4, st));
                        hipLaunchKernelGGL(k_fallback, dim3((unsigned)std::min<uint64_t>(q1 - q0, 65536)), dim3(kBlock),
                                           0, st, fine.p, gbase, dfine.p, dparts.p, q1 - q0, E, tab.p, tcap - 1, nn.p,
                                           dover.p);
                        LAUNCH_OK();
                        int over = 0;
                        HIP_OK(hipMemcpyAsync(&over, dover.p, 4, hipMemcpyDeviceToHost, st));
                        HIP_OK(hipStreamSynchronize(st));
                        if (over) {
                            tcap <<= 1;
                            continue;
                        }
                        hipLaunchKernelGGL(k_fallback_emit, dim3(grid_for(tcap, kBlock, 65536)), dim3(kBlock), 0, st,
                                           tab.p, tcap, out.keys.p, out.counts.p, out_cap, dcnt.p);
                        LAUNCH_OK();
                        HIP_OK(hipStreamSynchronize(st));
                        break;
                    }
                    q0 = q1;
                }
                HIP_OK(hipMemcpyAsync(hc, dcnt.p, 8, hipMemcpyDeviceToHost, st));
                HIP_OK(hipStreamSynchronize(st));
            }
            const uint64_t total = hc[0];
            ctx->kstats["lds_count"].total_bytes += 12.0 * (double)(std::min(total, out_cap) - std::min(n_out, out_cap));
            if (total <= out_cap) {
                n_out = total;
                break;
            }
            if (attempt > 0) throw Error(MCAAT_E_CAPACITY, "node_counter: output sizing failed");
            if (getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1')
                fprintf(stderr, "[mcaat] node_counter: group %zu overflowed the output (%llu > %llu): re-count\n", gi,
                        (unsigned long long)total, (unsigned long long)out_cap);
            // grow (keeping the groups already counted) and count this group again
            const uint64_t ncap = total + (total - n_out) * (uint64_t)(256 - b1) / (uint64_t)(b1 - b0) + (1u << 20);
            DevBuf<uint64_t> k2(ncap);
            DevBuf<uint32_t> c2(ncap);
            HIP_OK(hipMemcpyAsync(k2.p, out.keys.p, 8 * n_out, hipMemcpyDeviceToDevice, st));
            HIP_OK(hipMemcpyAsync(c2.p, out.counts.p, 4 * n_out, hipMemcpyDeviceToDevice, st));
            out.keys = std::move(k2);
            out.counts = std::move(c2);
            out_cap = ncap;
            // the counter restarts at n_out (two 32-bit device writes: no host buffer to keep alive)
            HIP_OK(hipMemsetD32Async((hipDeviceptr_t)dcnt.p, (int)(uint32_t)n_out, 1, st));
            HIP_OK(hipMemsetD32Async((hipDeviceptr_t)((uint32_t *)dcnt.p + 1), (int)(uint32_t)(n_out >> 32), 1, st));
            // (round 4 placed a synchronise here before the old buffers went back to the arena;
            // the arena's fences order their reuse now, nc.free_sync=1 restores it for A/B)
            if (free_sync) HIP_OK(hipStreamSynchronize(st));
        }
        // (round 4) the output is sized from n_occ / 32 (C3: 0.53 G distinct of 1.15 G); an
        // error-rich input (C5: ~2 G) used to overflow it mid-run, re-count a whole group and copy
        // everything counted so far. The groups are hash ranges, so the first (the small probe)
        // already tells the total: grow once, early, while little is copied.
        if (gi + 1 < groups.size() && (!knob_set(ctx, "nc.out_cap") || knob(ctx, "nc.grow_early", 0)) && hfine[p1] > 0) {
            const double frac = (double)hfine[p1] / (double)std::max<uint64_t>(n_live, 1);
            // grown with 8 % headroom, and again only when the plain extrapolation passes that
            // (C5's estimate moved 2.1194 -> 2.1201 G over the groups: three copies of up to 9 GB)
            const double need = (double)n_out / frac;
            const uint64_t est = (uint64_t)(need * 1.08) + (1u << 20);
            if (need > (double)out_cap) {
                if (getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1')
                    fprintf(stderr, "[mcaat] node_counter: output grown after group %zu (%llu distinct, %.4f of the descriptors): %llu -> %llu\n",
                            gi, (unsigned long long)n_out, frac, (unsigned long long)out_cap, (unsigned long long)est);
                DevBuf<uint64_t> k2(est);
                DevBuf<uint32_t> c2(est);
                HIP_OK(hipMemcpyAsync(k2.p, out.keys.p, 8 * n_out, hipMemcpyDeviceToDevice, st));
                HIP_OK(hipMemcpyAsync(c2.p, out.counts.p, 4 * n_out, hipMemcpyDeviceToDevice, st));
                // the next group's pass B (side stream) may be handed the old buffers: the arena
                // makes it wait for these copies (round 4 synchronised here: nc.free_sync=1)
                if (free_sync) HIP_OK(hipStreamSynchronize(st));
                out.keys = std::move(k2);
                out.counts = std::move(c2);
                out_cap = est;
            }
        }
        if (!overlap && gi + 1 < groups.size()) launch_b(groups[gi + 1]);
        fine.release();
        event_put(ctx, grp.done);
        grp.done = nullptr;
    }
    for (auto *t : btimers) t->finish();
    if (prof_c) {
        unsigned long long hp[10];
        HIP_OK(hipMemcpy(hp, dprof.p, 80, hipMemcpyDeviceToHost));
        const double waves = (double)ctx->n_cu * kCWaves;
        fprintf(stderr, "[mcaat] pass C per-wave ms: clear %.1f collapse %.1f expand %.1f emit %.1f; raw partitions %.0f (probe fails %llu), distinct descriptors %llu of %llu\n",
                hp[0] / waves / 1e5, hp[1] / waves / 1e5, hp[2] / waves / 1e5, hp[3] / waves / 1e5, (double)hp[4], hp[5], hp[6], hp[7]);
        // edges inserted by the expansion (each distinct descriptor's n) against the distinct edges
        fprintf(stderr, "[mcaat] pass C expansion: %llu edge inserts for %llu distinct edges (%.2f per edge)\n", hp[8], hp[9],
                hp[9] ? (double)hp[8] / (double)hp[9] : 0.0);
    }
    l1.release();
    l1s.release();
    bk.regions.assign(256, {});
    out.n = n_out;
    verbose_mark(ctx, "node_counter.C");
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

// loads this file's code object now (HIP defers it to the first launch of one of its kernels)
void preload_node_counter() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, (const void *)k_l2_hist);
}

}  // namespace mcaat
