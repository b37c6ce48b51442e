// common.h — shared host/device definitions for the MI355X mcaat hot path.
//
// Encoding (DESIGN.md "SDBG conventions"):
//   base codes A=0 C=1 G=2 T=3. Reads are one packed 2-bit stream: base j lives at
//   word j>>5, bits 2*(j&31) (LSB-first), so the E-symbol window starting at j is a
//   funnel shift of two words and equals lsb(e) = sum s[i] << 2i directly.
//   Edge e = s[0..k]; BOSS key K = ((lsb & mask_2k) << 2) | s[k]  (colex label, then W).
//   Edge id = rank of K in the sorted array of distinct oriented edges.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MCAAT_HD __host__ __device__ __forceinline__

namespace mcaat {

constexpr uint64_t kEmpty = ~0ULL;
constexpr int kMaxK = 30;           // (k+1)-mer keys use 2(k+1) <= 62 bits; bit 2E is a sort sentinel
constexpr int kIdxBits = 40;        // edge ids < 2^40 in packed adjacency words
constexpr uint64_t kIdxMask = (1ULL << kIdxBits) - 1;

MCAAT_HD uint64_t mask_bits(int n) { return n >= 64 ? ~0ULL : ((1ULL << n) - 1); }

// splitmix64 finaliser: the counter-based RNG and the table hash
MCAAT_HD uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
MCAAT_HD uint64_t hash3(uint64_t a, uint64_t b, uint64_t c) {
    return mix64(a ^ mix64(b ^ mix64(c)));
}

// reverse the order of the 2-bit groups in a 64-bit word
MCAAT_HD uint64_t rev2_64(uint64_t x) {
    x = ((x >> 2) & 0x3333333333333333ULL) | ((x & 0x3333333333333333ULL) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0FULL) | ((x & 0x0F0F0F0F0F0F0F0FULL) << 4);
    x = ((x >> 8) & 0x00FF00FF00FF00FFULL) | ((x & 0x00FF00FF00FF00FFULL) << 8);
    x = ((x >> 16) & 0x0000FFFF0000FFFFULL) | ((x & 0x0000FFFF0000FFFFULL) << 16);
    return (x >> 32) | (x << 32);
}
// lsb of the reverse complement of an E-symbol edge given its lsb
MCAAT_HD uint64_t lsb_rc(uint64_t lsb, int E) {
    return (rev2_64(lsb) >> (64 - 2 * E)) ^ mask_bits(2 * E);
}
MCAAT_HD uint64_t boss_key(uint64_t lsb, int k) {
    return ((lsb & mask_bits(2 * k)) << 2) | (lsb >> (2 * k));
}
MCAAT_HD uint64_t boss_to_lsb(uint64_t K, int k) {
    return (K >> 2) | ((K & 3) << (2 * k));
}
// window of E symbols starting at base j of a packed stream
MCAAT_HD uint64_t window_at(const uint64_t *packed, uint64_t j, int E) {
    const uint64_t w = j >> 5;
    const int s = 2 * (int)(j & 31);
    uint64_t v = packed[w] >> s;
    if (s + 2 * E > 64) v |= packed[w + 1] << (64 - s);
    return v & mask_bits(2 * E);
}

// ---------------------------------------------------------------------------
// Device-resident SDBG (structure of arrays, all in HBM).
//   out_info[e]: bits 0..39 first edge of target node, bits 40..43 mask of the W
//                symbols present at the target node (out-edges are consecutive).
//   in_info[e] : bits 0..39 first edge of the (k-1)-suffix group holding e's
//                predecessors, bits 40..55 positions (relative) of edges in that
//                group whose W == last label symbol of e.
//   valid      : one bit per edge, 64 edges per word (ballot-packed).
// ---------------------------------------------------------------------------
struct GraphView {
    int k;
    uint64_t D;
    const uint64_t *key;
    const uint16_t *mult;
    const uint64_t *out_info;
    const uint64_t *in_info;
    uint64_t *valid;
    // search-region replicas of a sharded graph (round 5): compact id -> edge id; null: ids are
    // edge ids. Only FindCycle's frame order (the libstdc++ bucket, id mod 13) reads it.
    const uint64_t *gid = nullptr;
};

__device__ __forceinline__ bool bit_get(const uint64_t *bm, uint64_t i) { return (bm[i >> 6] >> (i & 63)) & 1; }


// valid in-edges of e in ASCENDING id order; returns count
__device__ __forceinline__ int dev_incoming(const GraphView &g, uint64_t e, uint64_t *in) {
    const uint64_t ii = g.in_info[e];
    const uint64_t lo = ii & kIdxMask;
    unsigned m = (unsigned)(ii >> kIdxBits) & 0xFFFF;
    int n = 0;
    while (m) {
        const int j = __ffs(m) - 1;
        m &= m - 1;
        const uint64_t id = lo + j;
        if (bit_get(g.valid, id)) in[n++] = id;
    }
    return n;
}
// bits [lo, lo + 16) of a bitmap from its words lo/64 and lo/64 + 1
__device__ __forceinline__ uint32_t bits16(uint64_t w0, uint64_t w1, uint64_t lo) {
    const int sh = (int)(lo & 63);
    return (uint32_t)(((w0 >> sh) | (sh ? w1 << (64 - sh) : 0)) & 0xFFFFu);
}
// index of lo's word and of the word after it, clamped to the bitmap (an edge without
// neighbours may carry any lo: the loads stay in bounds, the mask discards their bits)
__device__ __forceinline__ uint64_t this_word(uint64_t lo, uint64_t nw) {
    const uint64_t w = lo >> 6;
    return w < nw ? w : nw - 1;
}
__device__ __forceinline__ uint64_t next_word(uint64_t lo, uint64_t nw) {
    const uint64_t w = (lo >> 6) + 1;
    return w < nw ? w : nw - 1;
}
// the two bitmap words at lo/64 (clamped like this_word) in one 16-B load: bitmaps are
// allocated with a padding word after the last (mcaat_graph::bitmap_words), so the pair always
// lies inside the allocation. Scans are bound by how many distinct addresses their gathers
// issue, not by bytes: one load instead of two.
struct __attribute__((aligned(8))) WordPair {
    uint64_t a, b;
};
__device__ __forceinline__ WordPair word_pair(const uint64_t *bm, uint64_t lo, uint64_t nw) {
    return *(const WordPair *)(bm + this_word(lo, nw));
}
// multiplicities of edges lo .. lo+3 from the three dwords holding them (one 12-B load; mult is
// allocated 8 entries past D, mcaat_graph::mult_entries); entries past D are garbage the
// caller masks
struct __attribute__((aligned(4))) Dword3 {
    uint32_t x, y, z;
};
__device__ __forceinline__ void mult4(const uint16_t *mult, uint64_t lo, uint32_t *m) {
    const Dword3 d = *(const Dword3 *)(mult + (lo & ~1ull));
    const uint64_t w = (uint64_t)d.x | ((uint64_t)d.y << 32);
    if (lo & 1) {
        const uint64_t v = (w >> 16) | ((uint64_t)d.z << 48);
        m[0] = (uint32_t)v & 0xFFFF, m[1] = (uint32_t)(v >> 16) & 0xFFFF, m[2] = (uint32_t)(v >> 32) & 0xFFFF, m[3] = (uint32_t)(v >> 48);
    } else {
        m[0] = (uint32_t)w & 0xFFFF, m[1] = (uint32_t)(w >> 16) & 0xFFFF, m[2] = (uint32_t)(w >> 32) & 0xFFFF, m[3] = (uint32_t)(w >> 48);
    }
}
// valid out-edges of e in DESCENDING id order (DESIGN.md convention); returns count. The
// out-edges are the consecutive ids [lo, lo + cnt): their valid bits are one bitmap window.
__device__ __forceinline__ int dev_outgoing(const GraphView &g, uint64_t e, uint64_t *out) {
    const uint64_t oi = g.out_info[e];
    const uint64_t lo = oi & kIdxMask;
    const unsigned m = (unsigned)(oi >> kIdxBits) & 0xF;
    const int cnt = __popc(m);
    const WordPair w = word_pair(g.valid, lo, (g.D + 63) / 64);
    const uint32_t vb = bits16(w.a, w.b, lo);
    int n = 0;
    for (int i = cnt - 1; i >= 0; --i)
        if ((vb >> i) & 1) out[n++] = lo + i;
    return n;
}
__device__ __forceinline__ int dev_outdeg(const GraphView &g, uint64_t e) {
    uint64_t t[4];
    return dev_outgoing(g, e, t);
}
__device__ __forceinline__ int dev_indeg(const GraphView &g, uint64_t e) {
    uint64_t t[4];
    return dev_incoming(g, e, t);
}

// block-wide sum, one atomic per block (blockDim.x must be a multiple of 64, <= 1024)
__device__ __forceinline__ void block_add(unsigned long long *counter, unsigned long long v) {
    __shared__ unsigned long long part[16];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) part[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += part[i];
        if (t) atomicAdd(counter, t);
    }
    __syncthreads();  // part[] is reused by the next call in the same kernel
}

// workgroup barrier for LDS hand-offs only: __syncthreads() also drains every outstanding
// global store and atomic (vmcnt(0))
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace mcaat
