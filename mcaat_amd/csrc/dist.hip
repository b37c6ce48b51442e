// dist.hip — the hash-range sharded graph build of a multi-GPU run, natively over a Comm
// (RCCL or shared memory; comm.hip); SURVEY.md §8e, DESIGN.md §7. Default route (round 4):
//   1. every rank runs pass A of the counter (node_counter_a) on its reads: super-k-mer
//      descriptors in 256 L1 buckets (hash ranges of the minimizer);
//   2. the buckets are cut into `world` contiguous owner ranges of equal descriptor weight and
//      each bucket's descriptors go to its owner (exchange_descriptors; round 5: straight from
//      pass A's buffers, one segment per bucket); every occurrence of a canonical edge has the
//      same minimizer, so the owner's passes B and C give final counts;
//   3. the ranks sum a histogram of the top BOSS-key bits and cut it into owner ranges,
//      contiguous in BOSS order; the counted canonical edges expand to their oriented edges and
//      go to their BOSS-range owners (route_oriented, one all-to-all), which sort their ranges;
//   4. round 5 (default, dist.shard_cf): each rank keeps its range as a sharded graph and builds
//      its adjacency from its four target key ranges (sdbg_finish_sharded, shard_cf.hip); the
//      per-shard CycleFinder runs on it. dist.shard_cf=0: an exact-size all-gather in rank order
//      concatenates the ranges into the single-GPU edge array (edge ids bit-identical), and every
//      rank builds the whole adjacency (sdbg_finish), round 4's form.
// dist.desc=0 keeps round 3's route (each rank counts its own reads, partial counts to the owner
// of the smaller BOSS key, summed there: canon_reduce), dist.oriented=1 round 2's (both
// orientations with 32-bit partial counts).
// Replaces: Read2SdbgS2::Run driven from sdbg_build.cpp:171-187, for reads split over ranks.
#include <algorithm>
#include <vector>

#include "comm.h"

namespace mcaat {

namespace {

constexpr int kHistBits = 12;

// world-1 ascending split points at histogram-bin edges with equal weight (owner o takes
// keys in [splits[o-1], splits[o])); the same rule as shard.choose_splits
std::vector<uint64_t> choose_splits(const std::vector<uint64_t> &hist, int world, int key_bits) {
    const int nb = (int)hist.size();
    int bits = 0;
    while ((1 << bits) < nb) ++bits;
    const int shift = key_bits - bits;
    std::vector<double> cum(nb);
    double acc = 0;
    for (int i = 0; i < nb; ++i) cum[i] = acc += (double)hist[i];
    const double total = nb ? cum[nb - 1] : 0.0;
    std::vector<uint64_t> out;
    int prev = 0;
    for (int o = 1; o < world; ++o) {
        int b = nb;
        if (total > 0) b = (int)(std::lower_bound(cum.begin(), cum.end(), total * o / world) - cum.begin()) + 1;
        b = std::min(std::max(b, prev), nb);
        out.push_back((uint64_t)b << shift);
        prev = b;
    }
    return out;
}

}  // namespace

// Round 4 (default; knob dist.desc=0 keeps the count exchange below): pass A's super-k-mer
// descriptors go to the owner of their L1 bucket. Every occurrence of a canonical edge has
// the same minimizer and so the same L1 bucket, so each owner's passes B and C over all ranks'
// descriptors of its buckets give final counts, each canonical edge on exactly one rank: no
// partial sums, no owner-side sort of ~D_c pairs whatever N (the count exchange's canon_reduce).
// The owners are contiguous bucket ranges of equal descriptor weight; a rank sends bucket b's
// reservations (whole reservation runs, inert padding included) to b's owner, which keeps one
// region per (bucket, source rank) for pass B.
// Replaces: the S2 counting of Read2SdbgS2::Run (sdbg_build.cpp:171-187) over reads split by rank.
// Round 5: the buckets go out from where pass A wrote them (one segment per bucket, grouped per
// owner: Comm::alltoallv_dev_segs), with no full-size send buffer; one rank keeps its buckets.
static void exchange_descriptors(mcaat_ctx *ctx, Comm &comm, NcBuckets &bk, NcBuckets &own, uint64_t occ_total) {
    const int N = comm.world, R = comm.rank;
    std::vector<uint64_t> mine(256, 0);
    for (int b = 0; b < 256; ++b) {
        if (bk.regions[b].size() > 1) throw Error(MCAAT_E_INVALID, "descriptor exchange: one region per bucket expected");
        for (const auto &rg : bk.regions[b]) mine[b] += rg.second;
    }
    // dist.segs_at_one=1 (tests): one rank runs the exchange too (its segments are the
    // transport's self-copies), so the segment all-to-all is exercised on a one-GPU box
    if (N == 1 && !knob(ctx, "dist.segs_at_one", 0)) {  // every bucket is this rank's: nothing moves
        own = std::move(bk);
        own.n_occ = occ_total;
        return;
    }
    const std::vector<uint64_t> all = comm.allgather_vec(mine);  // [rank][bucket]
    std::vector<double> cum(256);
    double acc = 0;
    for (int b = 0; b < 256; ++b) {
        for (int q = 0; q < N; ++q) acc += (double)all[(uint64_t)q * 256 + b];
        cum[b] = acc;
    }
    // owner o takes buckets [lo[o], lo[o+1])
    std::vector<int> lo(N + 1, 0);
    lo[N] = 256;
    for (int o = 1; o < N; ++o) {
        int b = acc > 0 ? (int)(std::lower_bound(cum.begin(), cum.end(), acc * o / N) - cum.begin()) + 1 : 256;
        lo[o] = std::min(std::max(b, lo[o - 1]), 256);
    }
    // to owner q: one segment per non-empty bucket of its range, descriptors and sub rows
    std::vector<std::vector<Comm::Seg>> s16(N), s2(N);
    for (int q = 0; q < N; ++q)
        for (int b = lo[q]; b < lo[q + 1]; ++b)
            for (const auto &rg : bk.regions[b]) {
                s16[q].push_back({bk.data.p + rg.first, 16 * rg.second});
                s2[q].push_back({bk.sub.p + rg.first, 2 * rg.second});
            }
    // from source q: its non-empty buckets of [lo[R], lo[R+1]), in bucket order
    std::vector<std::vector<uint64_t>> r16(N), r2(N);
    uint64_t n_recv = 0;
    own.regions.assign(256, {});
    for (int q = 0; q < N; ++q)
        for (int b = lo[R]; b < lo[R + 1]; ++b) {
            const uint64_t n = all[(uint64_t)q * 256 + b];
            if (!n) continue;
            r16[q].push_back(16 * n);
            r2[q].push_back(2 * n);
            own.regions[b].push_back({n_recv, n});
            n_recv += n;
        }
    own.data.alloc(n_recv ? n_recv : 1);
    own.sub.alloc(n_recv ? n_recv : 8);
    HIP_OK(hipStreamSynchronize(ctx->stream));
    comm.alltoallv_dev_segs(s16, own.data.p, r16);
    comm.alltoallv_dev_segs(s2, own.sub.p, r2);
    bk.data.release();
    bk.sub.release();
    own.l2_bits = bk.l2_bits;
    // occurrences behind this owner's descriptors (sizes its output buffer), by its share
    own.n_occ = acc > 0 ? (uint64_t)((double)occ_total * (double)n_recv / acc) + 1 : 0;
}

void build_graph_sharded(mcaat_ctx *ctx, Comm &comm, const mcaat_reads *r, int k, mcaat_graph *g) {
    hipStream_t st = ctx->stream;
    const int N = comm.world, R = comm.rank;
    StageTimer timer(ctx);
    const uint64_t xr0 = comm.n_coll, xq0 = comm.n_queued;  // the build's collectives (kstats "xr_build", queued "xq_build")
    CountResult c;
    const bool desc_route = knob(ctx, "dist.desc", 1) != 0 && !knob(ctx, "dist.oriented", 0);
    if (desc_route) {
        NcBuckets bk, own;
        uint64_t occ_total = 0;
        node_counter_a(ctx, r, k,
                       [&](uint64_t occ) {
                           for (uint64_t x : comm.allgather_one(occ)) occ_total += x;
                           return nc_fine_bits(ctx, occ_total);
                       },
                       bk);
        timer.mark("node_counter_a");
        exchange_descriptors(ctx, comm, bk, own, occ_total);
        timer.mark("shard_desc_all_to_all");
        node_counter_bc(ctx, own, k, c);
        timer.mark("node_counter_bc");
    } else {
        node_counter(ctx, r, k, c);
        timer.mark("node_counter");
    }

    std::vector<uint64_t> hist(1u << kHistBits);
    counts_histogram(ctx, c, k, kHistBits, hist.data());
    {
        const std::vector<uint64_t> all = comm.allgather_vec(hist);
        std::fill(hist.begin(), hist.end(), 0);
        for (size_t i = 0; i < all.size(); ++i) hist[i % hist.size()] += all[i];
    }
    const std::vector<uint64_t> splits = choose_splits(hist, N, 2 * (k + 1));
    DevBuf<uint64_t> uk;
    DevBuf<uint16_t> um;
    uint64_t u = 0;
    auto exchange = [&](const std::vector<uint64_t> &out_sizes, const uint64_t *skeys, const uint16_t *svals,
                        DevBuf<uint64_t> &rkeys, DevBuf<uint16_t> &rvals) {
        const std::vector<uint64_t> mat = comm.allgather_vec(out_sizes);
        std::vector<uint64_t> in(N), sb(N), rb(N);
        uint64_t n_in = 0;
        for (int s = 0; s < N; ++s) n_in += in[s] = mat[(uint64_t)s * N + R];
        rkeys.alloc(n_in ? n_in : 1);
        rvals.alloc(n_in ? n_in : 1);
        for (int p = 0; p < N; ++p) sb[p] = 8 * out_sizes[p], rb[p] = 8 * in[p];
        comm.alltoallv_dev(skeys, sb.data(), rkeys.p, rb.data());
        for (int p = 0; p < N; ++p) sb[p] = 2 * out_sizes[p], rb[p] = 2 * in[p];
        comm.alltoallv_dev(svals, sb.data(), rvals.p, rb.data());
        return n_in;
    };
    if (desc_route) {
        // final counts: expand each canonical edge to its oriented edges and route them to their
        // BOSS-range owners, which sort their ranges
        const uint64_t cap2 = std::max<uint64_t>(1, 2 * c.n);
        DevBuf<uint64_t> qk(cap2);
        DevBuf<uint16_t> qm(cap2);
        std::vector<uint64_t> sizes2(N);
        route_oriented(ctx, k, c.keys.p, c.counts.p, c.n, N, splits.data(), sizes2.data(), qk.p, qm.p, cap2);
        c = CountResult{};
        timer.mark("shard_partition");
        DevBuf<uint64_t> sk2;
        DevBuf<uint16_t> sm2;
        u = exchange(sizes2, qk.p, qm.p, sk2, sm2);
        qk.release();
        qm.release();
        timer.mark("shard_all_to_all");
        uk.alloc(u ? u : 1);
        um.alloc(u ? u : 1);
        sort_oriented(ctx, k, sk2.p, sm2.p, u, uk.p, um.p);
        timer.mark("shard_reduce");
    } else if (knob(ctx, "dist.oriented", 0)) {
        const uint64_t cap = std::max<uint64_t>(1, 2 * c.n);
        DevBuf<uint64_t> okeys(cap);
        DevBuf<uint32_t> ocnt(cap);
        std::vector<uint64_t> sizes(N);
        counts_partition(ctx, c, k, N, splits.data(), sizes.data(), okeys.p, ocnt.p, cap);
        c = CountResult{};
        timer.mark("shard_partition");

        // sizes[s][d] of every rank s -> what this rank receives
        const std::vector<uint64_t> mat = comm.allgather_vec(sizes);
        std::vector<uint64_t> in(N), sb(N), rb(N);
        uint64_t n_in = 0;
        for (int s = 0; s < N; ++s) n_in += in[s] = mat[(uint64_t)s * N + R];
        DevBuf<uint64_t> rk(n_in);
        DevBuf<uint32_t> rc(n_in);
        for (int p = 0; p < N; ++p) sb[p] = 8 * sizes[p], rb[p] = 8 * in[p];
        comm.alltoallv_dev(okeys.p, sb.data(), rk.p, rb.data());
        for (int p = 0; p < N; ++p) sb[p] = 4 * sizes[p], rb[p] = 4 * in[p];
        comm.alltoallv_dev(ocnt.p, sb.data(), rc.p, rb.data());
        okeys.release();
        ocnt.release();
        timer.mark("shard_all_to_all");

        uk.alloc(n_in ? n_in : 1);
        um.alloc(n_in ? n_in : 1);
        u = edges_reduce(ctx, k, rk.p, rc.p, n_in, uk.p, um.p);
        timer.mark("shard_reduce");
    } else {
        // step 3: canonical edges to the owner of their smaller BOSS key
        const uint64_t cap = std::max<uint64_t>(1, c.n);
        DevBuf<uint64_t> okeys(cap);
        DevBuf<uint16_t> ocnt(cap);
        std::vector<uint64_t> sizes(N);
        counts_partition_canon(ctx, c, k, N, splits.data(), sizes.data(), okeys.p, ocnt.p, cap);
        c = CountResult{};
        timer.mark("shard_partition");
        DevBuf<uint64_t> rk;
        DevBuf<uint16_t> rc;
        const uint64_t n_in = exchange(sizes, okeys.p, ocnt.p, rk, rc);
        okeys.release();
        ocnt.release();
        timer.mark("shard_all_to_all");
        // step 4: sum, expand, route the oriented edges to their range owners, sort
        DevBuf<uint64_t> ck(n_in ? n_in : 1);
        DevBuf<uint32_t> ct(n_in ? n_in : 1);
        const uint64_t nc = canon_reduce(ctx, k, rk.p, rc.p, n_in, ck.p, ct.p);
        rk.release();
        rc.release();
        const uint64_t cap2 = std::max<uint64_t>(1, 2 * nc);
        DevBuf<uint64_t> qk(cap2);
        DevBuf<uint16_t> qm(cap2);
        std::vector<uint64_t> sizes2(N);
        route_oriented(ctx, k, ck.p, ct.p, nc, N, splits.data(), sizes2.data(), qk.p, qm.p, cap2);
        ck.release();
        ct.release();
        DevBuf<uint64_t> sk2;
        DevBuf<uint16_t> sm2;
        u = exchange(sizes2, qk.p, qm.p, sk2, sm2);
        qk.release();
        qm.release();
        uk.alloc(u ? u : 1);
        um.alloc(u ? u : 1);
        sort_oriented(ctx, k, sk2.p, sm2.p, u, uk.p, um.p);
        timer.mark("shard_reduce");
    }

    const std::vector<uint64_t> ns = comm.allgather_one(u);
    uint64_t D = 0;
    for (uint64_t x : ns) D += x;
    g->ctx = ctx;
    g->k = k;
    g->D = D;
    // (round 5, default) the graph stays sharded: this rank keeps its range, builds its edges'
    // adjacency by one exchange with the target owners, and CycleFinder runs per shard
    // (shard_cf.hip). dist.shard_cf=0: the exact-size all-gather below, every rank the whole graph.
    if (knob(ctx, "dist.shard_cf", 1) != 0 && desc_route) {
        g->sharded = true;
        g->rank_lo.assign(N + 1, 0);
        for (int r = 0; r < N; ++r) g->rank_lo[r + 1] = g->rank_lo[r] + ns[r];
        g->key_split = splits;
        g->id_lo = g->rank_lo[R];
        g->D_local = u;
        g->key = std::move(uk);
        g->mult.alloc(mcaat_graph::mult_entries(u));
        HIP_OK(hipMemcpyAsync(g->mult.p, um.p, 2 * u, hipMemcpyDeviceToDevice, st));
        HIP_OK(hipStreamSynchronize(st));
        um.release();
        timer.mark("shard_all_gather");
        sdbg_finish_sharded(ctx, comm, g);
        timer.mark("sdbg_build");
        HIP_OK(hipStreamSynchronize(st));
        timer.finish();
        ctx->kstats["xr_build"].launches += comm.n_coll - xr0;
        ctx->kstats["xq_build"].launches += comm.n_queued - xq0;
        return;
    }
    g->key.alloc(D ? D : 1);
    g->mult.alloc(mcaat_graph::mult_entries(D));
    std::vector<uint64_t> b8(N), b2(N);
    for (int p = 0; p < N; ++p) b8[p] = 8 * ns[p], b2[p] = 2 * ns[p];
    HIP_OK(hipStreamSynchronize(st));
    comm.allgatherv_dev(uk.p, g->key.p, b8.data());
    comm.allgatherv_dev(um.p, g->mult.p, b2.data());
    uk.release();
    um.release();
    timer.mark("shard_all_gather");
    sdbg_finish(ctx, g);
    timer.mark("sdbg_build");
    HIP_OK(hipStreamSynchronize(st));
    timer.finish();
    ctx->kstats["xr_build"].launches += comm.n_coll - xr0;
    ctx->kstats["xq_build"].launches += comm.n_queued - xq0;
}

}  // namespace mcaat
