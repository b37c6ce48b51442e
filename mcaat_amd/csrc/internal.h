// internal.h — library-private structures of libmcaat_gpu.so
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <functional>
#include <vector>
#include <sys/mman.h>
#include <cstring>
#include <cstdlib>
#include <new>

#include "../../include/mcaat_gpu.h"
#include "common.h"

namespace mcaat {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};
// input the 4-line GPU FASTQ parser does not take (the host kseq-style reader does)
struct FormatError : Error {
    explicit FormatError(const std::string &m) : Error(MCAAT_E_IO, m) {}
};

#define HIP_OK(expr)                                                                              \
    do {                                                                                          \
        hipError_t e__ = (expr);                                                                  \
        if (e__ != hipSuccess)                                                                    \
            throw ::mcaat::Error(MCAAT_E_HIP, std::string(#expr " failed: ") + hipGetErrorString(e__) + \
                                                  " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
    } while (0)

#define LAUNCH_OK() HIP_OK(hipGetLastError())

// Caching device allocator: the hot path allocates the same multi-GB buffers every
// step; hipMalloc/hipFree of such buffers costs 10-100s of ms each, so freed blocks are
// kept per device and reused (best fit within 2x); on an allocation failure the cache
// is trimmed and the allocation retried.
void *dev_alloc(size_t bytes);
void dev_free(void *p, size_t bytes, int device);
int current_device();
void dev_trim();
// stream-ordered reuse (alloc.hip): frees fence the watched streams that still have work queued,
// and an allocation waits (on its stream) for the fences of the other streams
void watch_stream(int device, hipStream_t s);
void unwatch_stream(int device, hipStream_t s);
hipStream_t alloc_stream();  // this thread's allocation stream (null: the host waits)
void set_alloc_stream(hipStream_t s);
void arena_stats(uint64_t *fences, uint64_t *waits);
// device bytes handed out now, the most since the last reset, and the chunks held (this device)
void arena_usage(uint64_t *in_use, uint64_t *peak, uint64_t *reserved, bool reset_peak);
void arena_check(::mcaat_ctx *ctx, int64_t *out);  // mcaat_arena_check
// allocations inside the scope are for work queued on stream s
struct AllocStreamScope {
    hipStream_t prev;
    explicit AllocStreamScope(hipStream_t s) : prev(alloc_stream()) { set_alloc_stream(s); }
    ~AllocStreamScope() { set_alloc_stream(prev); }
    AllocStreamScope(const AllocStreamScope &) = delete;
    AllocStreamScope &operator=(const AllocStreamScope &) = delete;
};
void preload_node_counter();
void preload_sdbg_build();
void preload_cycle_finder();
void preload_fastq_pack();
void preload_read_mapping();
void preload_shard();  // the multi-GPU build, per-shard CycleFinder and succinct view modules
void preload_shard_cf();
void preload_sdbg_succinct();

// owning device buffer
template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    size_t cap_bytes = 0;
    int dev = 0;  // arena the block came from (freed there whatever device is current)
    DevBuf() = default;
    explicit DevBuf(size_t count) { alloc(count); }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    DevBuf(DevBuf &&o) noexcept : p(o.p), n(o.n), cap_bytes(o.cap_bytes), dev(o.dev) { o.p = nullptr; o.n = 0; o.cap_bytes = 0; }
    DevBuf &operator=(DevBuf &&o) noexcept {
        if (this != &o) {
            release();
            p = o.p; n = o.n; cap_bytes = o.cap_bytes; dev = o.dev;
            o.p = nullptr; o.n = 0; o.cap_bytes = 0;
        }
        return *this;
    }
    ~DevBuf() { release(); }
    void alloc(size_t count) {
        release();
        if (count == 0) count = 1;
        cap_bytes = (count * sizeof(T) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
        dev = current_device();
        p = (T *)dev_alloc(cap_bytes);
        n = count;
    }
    void release() {
        if (p) dev_free(p, cap_bytes, dev);
        p = nullptr;
        n = 0;
        cap_bytes = 0;
    }
    size_t bytes() const { return n * sizeof(T); }
};

struct KernelStat {
    double total_ms = 0;
    uint64_t launches = 0;
    double total_bytes = 0;  // algorithmic bytes over all launches
};

struct HostPool {
    uint64_t *p = nullptr;
    size_t n = 0;  // words
    HostPool() = default;
    HostPool(const HostPool &) = delete;
    HostPool &operator=(const HostPool &) = delete;
    ~HostPool() { free(p); }
    void ensure(size_t words) {
        if (words <= n) return;
        free(p);
        p = nullptr;
        n = 0;
        const size_t huge = 2u << 20, bytes = (words * 8 + huge - 1) / huge * huge;
        void *q = nullptr;
        if (posix_memalign(&q, huge, bytes) != 0) throw std::bad_alloc();
        madvise(q, bytes, MADV_HUGEPAGE);
        memset(q, 0, bytes);
        p = (uint64_t *)q;
        n = bytes / 8;
    }
};

}  // namespace mcaat

struct mcaat_ctx {
    int device = 0;
    int n_cu = 256;  // compute units (persistent-grid sizing)
    hipStream_t stream = nullptr;
    // second stream (created on first use): node_counter partitions the next group of L1
    // buckets (pass B) on it while pass C counts the current group
    hipStream_t side = nullptr;
    std::vector<std::pair<const char *, double>> stages;
    std::map<std::string, mcaat::KernelStat> kstats;
    bool timing = true;
    // host bitmap pool reused by every CycleFinder call: 2-MB aligned and advised for huge
    // pages (random bit probes over ~D/8 bytes), faulted in once; each call zeroes only the
    // words it touched
    mcaat::HostPool host_bits;
    // pinned staging chunks of the FASTQ reader, kept between calls (hipHostMalloc of a few
    // hundred MB costs more than parsing a small file); freed by mcaat_finalize
    uint8_t *pinned[2] = {nullptr, nullptr};
    size_t pinned_bytes = 0;
    // tuning/test knobs (mcaat_set_knob): size limits that decide which code path a stage
    // takes, so small parity inputs can drive the branches that only large inputs reach
    std::map<std::string, int64_t> knobs;
    // timing events reused across calls (stage and kernel timers take them from here)
    std::vector<hipEvent_t> events;
    // pinned bounce buffer for device-to-host result copies (mcaat::d2h). A copy straight into
    // a large pageable vector pins it for the transfer, and freeing it afterwards (munmap) makes
    // the driver evict and later restore the process's queues: the next step's first
    // submission then waited ~20-28 ms on an idle GPU.
    uint8_t *bounce = nullptr;
    size_t bounce_bytes = 0;
    // pinned staging of the host FASTQ packer (two buffers per packing thread), kept
    uint8_t *pack_pinned = nullptr;
    size_t pack_pinned_bytes = 0;
    // mcaat_count_ahead: the next host-packed FASTQ read runs node_counter's pass A for this k
    // on its parts as they land (0: off; one read takes it)
    int ahead_k = 0;
    // per-shard region BFS (shard_cf.hip): the request-block size the last forward / backward BFS
    // ended with, so the next step starts there instead of rerunning after an overflow (every
    // rank learns the same size: it is agreed over all ranks)
    uint64_t bfs_block[2] = {0, 0};
};

namespace mcaat {
// a C-ABI entry's context: its device, and its main stream as this thread's allocation stream
inline void bind(mcaat_ctx *ctx) {
    HIP_OK(hipSetDevice(ctx->device));
    set_alloc_stream(ctx->stream);
}
}  // namespace mcaat

namespace mcaat {
struct NcBuckets;
}
struct mcaat_reads {
    mcaat_ctx *ctx = nullptr;
    // (round 5) node_counter's pass A, run while the input was read (mcaat_count_ahead): the
    // first count for ahead_k takes it over
    mutable std::shared_ptr<mcaat::NcBuckets> ahead;
    int ahead_k = 0;
    mcaat::DevBuf<uint64_t> packed;
    mcaat::DevBuf<uint64_t> offsets;
    uint64_t n_reads = 0, n_bases = 0, n_words = 0;
    uint64_t fixed_len = 0;  // >0 when every read has this length (offsets[i] = i*len)
    // Mapping view (reads.cpp:88-130): one entry per input record, second-file records
    // reversed and complemented, A/C/G -> 0/1/2 and any other symbol -> 3. Empty when it
    // equals the counting view above (one file, ACGT only).
    mcaat::DevBuf<uint64_t> rec_packed;
    mcaat::DevBuf<uint64_t> rec_offsets;
    uint64_t n_records = 0;
    bool has_records = false;
    std::vector<uint64_t> file_records;  // mapping-view records per input file (file order)
};

struct mcaat_mapped {  // relevant reads: node-id chains in reference order
    std::vector<uint64_t> ids;
    std::vector<uint64_t> offsets{0};
    std::vector<uint64_t> records;  // index of each relevant read in the mapping view
};

struct mcaat_graph {
    mcaat_ctx *ctx = nullptr;
    int k = 0;
    uint64_t D = 0;
    mcaat::DevBuf<uint64_t> key;
    mcaat::DevBuf<uint16_t> mult;
    mcaat::DevBuf<uint64_t> out_info;
    mcaat::DevBuf<uint64_t> in_info;
    mcaat::DevBuf<uint64_t> valid;
    // every edge still valid, as the build leaves the graph (round 4): CycleFinder's tips pass
    // then reads no bitmap windows before the filter; cleared by anything that clears a bit
    bool all_valid = false;
    // radix directory over the top bits of the BOSS key (label lookups after the build)
    mcaat::DevBuf<uint64_t> dir;
    int dir_shift = 0;
    // (round 5) a sharded graph (mcaat_build_graph_sharded, knob dist.shard_cf): this rank holds
    // the edges [id_lo, id_lo + D_local) of the D edges, its BOSS-key range; key, mult, out_info,
    // in_info (global ids) and valid are indexed by local position; rank_lo holds every rank's
    // first id (N + 1 entries), key_split the N - 1 BOSS-key splits (owner of a key: the number of
    // splits at or below it). CycleFinder runs per shard (shard_cf.hip); mcaat_graph_unshard
    // gathers the whole graph for the host steps after it.
    bool sharded = false;
    uint64_t id_lo = 0, D_local = 0;
    std::vector<uint64_t> rank_lo, key_split;
    uint64_t dir_base = 0;  // sharded: the local directory's prefixes are (key - dir_base) >> dir_shift
    uint64_t dir_n = 0;     // sharded: its prefix count
    // sharded: every rank's four target ranges O_W(r) (shard_cf.hip target_ranges), 4 (N + 1) ids
    std::vector<uint64_t> tgt_lo;
    // search-region replicas (shard_cf.hip): compact id -> edge id, read for FindCycle's frame
    // order (the libstdc++ bucket of an id) and to name results
    mcaat::DevBuf<uint64_t> gid;
    mcaat::GraphView view() const {
        return mcaat::GraphView{k, sharded ? D_local : D, key.p, mult.p, out_info.p, in_info.p, valid.p,
                                gid.n ? gid.p : nullptr};
    }
    uint64_t n_words() const { return ((sharded ? D_local : D) + 63) / 64; }
    // allocation sizes: a valid/visited bitmap keeps one word past its last, and mult 8
    // entries past its last, so a neighbour window is one 16-B / 12-B load (common.h win16,
    // mult4) even at the end of the graph
    static uint64_t bitmap_words(uint64_t d) { return (d + 63) / 64 + 1; }
    static uint64_t mult_entries(uint64_t d) { return d + 8; }
};

struct mcaat_cycles {
    std::vector<uint64_t> starts;
    std::vector<std::vector<uint64_t>> flat;
    std::vector<std::vector<uint64_t>> offsets;
    std::vector<uint64_t> cand_ids;
    std::vector<int32_t> cand_bucket;
    uint64_t stats[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};

namespace mcaat {

inline hipEvent_t event_get(mcaat_ctx *ctx) {
    if (!ctx->events.empty()) {
        hipEvent_t e = ctx->events.back();
        ctx->events.pop_back();
        return e;
    }
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    return e;
}
inline void event_put(mcaat_ctx *ctx, hipEvent_t e) {
    if (e) ctx->events.push_back(e);
}

// device -> host copy of n bytes through the ctx's pinned bounce buffer (stream-synchronous)
inline void d2h(mcaat_ctx *ctx, void *dst, const void *src, size_t n) {
    if (!n) return;
    if (ctx->bounce_bytes < n) {
        if (ctx->bounce) {
            HIP_OK(hipStreamSynchronize(ctx->stream));
            HIP_OK(hipHostFree(ctx->bounce));
            ctx->bounce = nullptr;
            ctx->bounce_bytes = 0;
        }
        const size_t want = std::max<size_t>(n, 4u << 20);
        HIP_OK(hipHostMalloc((void **)&ctx->bounce, want, hipHostMallocDefault));
        ctx->bounce_bytes = want;
    }
    HIP_OK(hipMemcpyAsync(ctx->bounce, src, n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    memcpy(dst, ctx->bounce, n);
}

// host -> device copy of n bytes through the same bounce buffer (stream-synchronous)
inline void h2d(mcaat_ctx *ctx, void *dst, const void *src, size_t n) {
    if (!n) return;
    if (ctx->bounce_bytes < n) {
        if (ctx->bounce) {
            HIP_OK(hipStreamSynchronize(ctx->stream));
            HIP_OK(hipHostFree(ctx->bounce));
            ctx->bounce = nullptr;
            ctx->bounce_bytes = 0;
        }
        const size_t want = std::max<size_t>(n, 4u << 20);
        HIP_OK(hipHostMalloc((void **)&ctx->bounce, want, hipHostMallocDefault));
        ctx->bounce_bytes = want;
    }
    HIP_OK(hipStreamSynchronize(ctx->stream));  // an earlier copy out of the bounce buffer is done
    memcpy(ctx->bounce, src, n);
    HIP_OK(hipMemcpyAsync(dst, ctx->bounce, n, hipMemcpyHostToDevice, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
}

// event-bracketed stage timer on the ctx stream
struct StageTimer {
    mcaat_ctx *ctx;
    std::vector<std::pair<const char *, hipEvent_t>> marks;
    explicit StageTimer(mcaat_ctx *c) : ctx(c) { ctx->stages.clear(); mark("begin"); }
    void mark(const char *name) {
        hipEvent_t e = event_get(ctx);
        HIP_OK(hipEventRecord(e, ctx->stream));
        marks.push_back({name, e});
    }
    // call after the stream is synchronised
    void finish() {
        if (!marks.empty()) HIP_OK(hipEventSynchronize(marks.back().second));
        for (size_t i = 1; i < marks.size(); ++i) {
            float ms = 0;
            HIP_OK(hipEventElapsedTime(&ms, marks[i - 1].second, marks[i].second));
            ctx->stages.push_back({marks[i].first, (double)ms});
        }
        for (auto &m : marks) event_put(ctx, m.second);
        marks.clear();
    }
    ~StageTimer() {
        // an unfinished timer (an error unwinding): its events may still be pending
        for (auto &m : marks) (void)hipEventDestroy(m.second);
    }
};

// HIP-event timing of one kernel launch on the ctx stream
struct KernelTimer {
    mcaat_ctx *ctx;
    const char *name;
    double bytes;
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t s = nullptr;
    KernelTimer(mcaat_ctx *c, const char *n, double algorithmic_bytes, hipStream_t on = nullptr)
        : ctx(c), name(n), bytes(algorithmic_bytes), s(on ? on : c->stream) {
        a = event_get(ctx);
        b = event_get(ctx);
        HIP_OK(hipEventRecord(a, s));
    }
    void stop() {
        mark();
        finish();
    }
    // mark() closes the timed span on the stream; finish() waits for it, so work launched on
    // other streams in between is not held up by the host
    void mark() { HIP_OK(hipEventRecord(b, s)); }
    void finish() {
        HIP_OK(hipEventSynchronize(b));
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, a, b));
        auto &s = ctx->kstats[name];
        s.total_ms += ms;
        s.launches += 1;
        s.total_bytes += bytes;
        event_put(ctx, a);
        event_put(ctx, b);
        a = b = nullptr;
    }
    ~KernelTimer() {  // not stopped (an error unwinding)
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
};

// value of a knob set with mcaat_set_knob, or the default
inline int64_t knob(const mcaat_ctx *ctx, const char *name, int64_t dflt) {
    auto it = ctx->knobs.find(name);
    return it == ctx->knobs.end() ? dflt : it->second;
}

inline bool knob_set(const mcaat_ctx *ctx, const char *name) { return ctx->knobs.count(name) != 0; }

inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap = 65535u * 16) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

inline uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// stage entry points (implemented in the .hip files)
struct CountResult {
    DevBuf<uint64_t> keys;   // canonical lsb (k+1)-mers, unsorted unless requested
    DevBuf<uint32_t> counts;
    uint64_t n = 0;
};
void node_counter(mcaat_ctx *ctx, const mcaat_reads *r, int k, CountResult &out);
// node_counter in its two halves (a sharded build exchanges the L1 buckets between them)
struct NcBuckets {
    DevBuf<uint4> data;     // 16-B super-k-mer descriptors
    DevBuf<uint16_t> sub;   // each one's fine sub-partition row (same slots)
    // per L1 bucket: its regions (first slot, slots) in data/sub, each a whole number of
    // kMini-slot reservations (256 slots: every region starts 16-B aligned in sub)
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> regions;
    // pass A's layout: bucket b's slots start at base[b] (257 entries; a bucket's reserved but
    // unused tail is not part of its region). Empty when the regions came from an exchange.
    std::vector<uint64_t> base;
    int l2_bits = 0;        // fine partitions = 256 << l2_bits
    uint64_t n_occ = 0;     // edge occurrences behind the descriptors (sizes the output)
};
int nc_fine_bits(mcaat_ctx *ctx, uint64_t n_occ);
void node_counter_a(mcaat_ctx *ctx, const mcaat_reads *r, int k, const std::function<int(uint64_t)> &pick, NcBuckets &b);
void node_counter_bc(mcaat_ctx *ctx, NcBuckets &b, int k, CountResult &out);
// pass A on a streamed input, part by part (node_counter.hip; used by the FASTQ packer)
struct NcAhead;
std::shared_ptr<NcAhead> nc_ahead_begin(mcaat_ctx *ctx, int k, uint64_t n_occ_est, uint64_t n_items_est);
void nc_ahead_part(NcAhead &a, const uint64_t *packed, uint64_t n_reads, uint64_t L);
void nc_ahead_fail(NcAhead &a);
std::shared_ptr<NcBuckets> nc_ahead_end(NcAhead &a);
constexpr int kNcItem = 127;  // pass A's edge positions per work item (node_counter.hip kItem)
void verbose_mark(mcaat_ctx *ctx, const char *what);
void sort_counts(mcaat_ctx *ctx, CountResult &c, int k);
void sdbg_build(mcaat_ctx *ctx, CountResult &c, int k, mcaat_graph *g);
void sdbg_finish(mcaat_ctx *ctx, mcaat_graph *g);
// the succinct (BOSS) view of a built graph, checked and timed beside its arrays
// (sdbg_succinct.hip, mcaat_graph_succinct_check)
void graph_succinct_check(mcaat_graph *g, bool check, uint64_t *out, double *ms);
// multi-GPU build pieces (shard.hip)
void counts_histogram(mcaat_ctx *ctx, const CountResult &c, int k, int bits, uint64_t *hist_host);
void counts_partition(mcaat_ctx *ctx, const CountResult &c, int k, int n_owners, const uint64_t *splits_host,
                      uint64_t *sizes_host, uint64_t *okeys, uint32_t *ocnt, uint64_t cap);
uint64_t edges_reduce(mcaat_ctx *ctx, int k, const uint64_t *keys, const uint32_t *cnt, uint64_t n, uint64_t *keys_out,
                      uint16_t *mult_out);
void graph_from_sorted(mcaat_ctx *ctx, int k, const uint64_t *keys, const uint16_t *mult, uint64_t D, mcaat_graph *g);
// the native multi-GPU build's canonical-pair exchange (shard.hip): canonical edges routed to the
// owner of their smaller BOSS key with 16-bit partial counts; the owner sums them
// (canon_reduce), routes the oriented edges to their range owners (route_oriented), and each
// owner sorts what it received (sort_oriented)
uint64_t counts_partition_canon(mcaat_ctx *ctx, const CountResult &c, int k, int n_owners, const uint64_t *splits_host,
                                uint64_t *sizes_host, uint64_t *okeys, uint16_t *ocnt, uint64_t cap);
uint64_t canon_reduce(mcaat_ctx *ctx, int k, const uint64_t *keys, const uint16_t *cnt16, uint64_t n, uint64_t *keys_out,
                      uint32_t *tot_out);
uint64_t route_oriented(mcaat_ctx *ctx, int k, const uint64_t *keys, const uint32_t *tot, uint64_t n, int n_owners,
                        const uint64_t *splits_host, uint64_t *sizes_host, uint64_t *okeys, uint16_t *omult, uint64_t cap);
void sort_oriented(mcaat_ctx *ctx, int k, const uint64_t *keys, const uint16_t *mult, uint64_t n, uint64_t *keys_out,
                   uint16_t *mult_out);
struct Comm;  // comm.h
// comm: the ranks of a multi-GPU run that each hold this graph (null: one GPU); every rank
// gets the same results
void cycle_finder(mcaat_graph *g, const mcaat_cf_params &p, mcaat_cycles *out, Comm *comm = nullptr);
// CycleFinder's searches over a search graph (cycle_finder.hip; the whole graph, or a region
// replica of a sharded one): DepthLevelSearch of the ascending candidate ids, split over the
// ranks (returns the passing ids, ascending, on every rank) ...
std::vector<uint64_t> cf_depth_level_search(mcaat_graph *g, const std::vector<uint64_t> &cand, int limit, Comm *comm);
// ... and the bucket loop of FindCycle over the starts in the reference's order (out->starts,
// flat, offsets, stats[5..7])
void cf_find_cycles(mcaat_graph *g, const mcaat_cf_params &p, const std::vector<uint64_t> &starts, mcaat_cycles *out,
                    Comm *comm);
// (round 5) the per-shard CycleFinder over a sharded graph (shard_cf.hip)
void cycle_finder_sharded(mcaat_graph *g, const mcaat_cf_params &p, mcaat_cycles *out, Comm &comm);
// the sharded build's adjacency: every rank its range's out_info / in_info by one request /
// response exchange with the owners of the targets (shard_cf.hip)
void sdbg_finish_sharded(mcaat_ctx *ctx, Comm &comm, mcaat_graph *g);
// a sharded graph -> the whole graph on every rank (valid bits kept)
void graph_unshard(mcaat_graph *g, Comm &comm);
void synth_reads(mcaat_ctx *ctx, const mcaat_synth_spec &s, mcaat_reads *out, uint64_t first, uint64_t count);
void synth_genome_host(const mcaat_synth_spec &s, std::vector<uint64_t> &genome);
void graph_neighbors(const mcaat_graph *g, const uint64_t *ids, size_t n, int incoming, uint64_t *out,
                     int32_t *counts);
void graph_set_valid(mcaat_graph *g, const uint64_t *ids, size_t n, int valid);
void graph_gather(const mcaat_graph *g, const uint64_t *ids, size_t n, uint64_t *keys, uint16_t *mult);
void graph_download_valid(const mcaat_graph *g, uint8_t *valid);
void graph_keep_only(mcaat_graph *g, const uint64_t *ids, size_t n);
void graph_keep_region(mcaat_graph *g, const uint64_t *seeds, size_t n, uint64_t hops);
// valid edge ids (ascending) and each one's valid out-neighbours as ranks among them; null ids:
// only the count
uint64_t graph_valid_out_ranks(const mcaat_graph *g, uint64_t *ids, uint32_t *nbr, uint8_t *cnt);
// FASTQ(.gz) inputs parsed on the GPU (fastq_ingest.hip)
// ranges: per file, the byte range [first, second) to read (a rank's part; null: whole files)
void ingest_fastq(mcaat_ctx *ctx, const char *const *files, int n_files, mcaat_reads *r,
                  const std::vector<std::pair<uint64_t, uint64_t>> *ranges = nullptr);
// Decompressed sequential bytes of an input file (instream.hip): gzip (zlib), bzip2 (libbz2,
// opened at run time) or plain; concatenated members / streams are read in sequence.
class InStream {
   public:
    enum class Kind { Plain, Gzip, Bzip2 };
    explicit InStream(const char *path);
    ~InStream();
    InStream(const InStream &) = delete;
    InStream &operator=(const InStream &) = delete;
    size_t read(uint8_t *dst, size_t n);  // < n only at the end of the input
    Kind kind() const { return kind_; }

   private:
    struct Impl;
    Impl *impl_;
    Kind kind_ = Kind::Plain;
};
// plain 4-line FASTQ with upper-case ACGT sequences packed by host threads (fastq_pack.hip);
// false (nothing changed) when an input is outside that form: the GPU text parser takes it
bool fastq_hostpack(mcaat_ctx *ctx, const char *const *files, int n_files,
                    const std::vector<std::pair<uint64_t, uint64_t>> *ranges, mcaat_reads *r);
// first 4-line FASTQ record start at or after byte pos of a plain file (its size if none)
uint64_t fastq_record_start(const char *path, uint64_t pos);
bool is_compressed_file(const char *path);  // gzip or bzip2: read whole, never split
void write_fastq(const mcaat_reads *r, const char *path, int threads);
void graph_save(const mcaat_graph *g, const char *path);
void graph_load(mcaat_ctx *ctx, const char *path, mcaat_graph *g);
void map_reads(const mcaat_graph *g, const mcaat_reads *r, const uint64_t *nodes, size_t n_nodes,
               uint64_t max_batch_ids, mcaat_mapped *out);

}  // namespace mcaat

struct mcaat_counts {  // device-resident canonical counts of one rank
    mcaat_ctx *ctx = nullptr;
    int k = 0;
    mcaat::CountResult c;
};

