// alloc.hip — device memory arena behind DevBuf (see internal.h).
//
// The hot path allocates tens of multi-GB buffers per step with a fixed pattern. hipMalloc /
// hipFree of such buffers costs 10-100s of ms each, and an exact-size cache cannot reuse a
// freed 100 GB partition buffer for the next stage's 10 GB arrays, which at ~200 GB peak on
// a 288 GB device forces trims and re-allocation every step. This arena keeps every
// hipMalloc'd chunk, serves requests best-fit from free segments (splitting them) and
// coalesces neighbouring free segments of a chunk on free, so after the first step the whole
// pipeline runs inside memory it already owns. On an allocation failure, wholly free chunks
// are released and the request retried.
//
// Stream order (round 5). A block is freed by the host while kernels queued on some stream may
// still read or write it. Reusing it at once is safe only for work queued later on that same
// stream. So a free records a fence (an event) on every watched stream that still has work
// queued (the context's main and side streams, watch_stream), and the segment carries those
// fences; when the segment is handed out again for work on stream S (the thread's allocation
// stream, AllocStreamScope / bind: the context's main stream by default), S waits on the device
// for the fences of every other stream that have not completed (hipStreamWaitEvent, no host
// wait). An allocation with no stream named waits for them on the host. Round 4's race (the
// count output's early growth freeing buffers a queued copy still read, handed to the next pass
// B on the side stream) is thereby excluded by the allocator, not by a synchronise at the site.
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <map>
#include <mutex>
#include <set>

#include "internal.h"

namespace mcaat {

namespace {

constexpr size_t kAlign = 256;
constexpr size_t kMinChunk = 256ull << 20;  // grow by at least 256 MiB

// one fence: stream slot (Arena::streams) and serial of the event recorded there at a free
struct Fence {
    int slot;
    uint64_t serial;
};

struct Arena {
    struct Seg {
        size_t size;
        bool free;
        char *chunk;  // base of the hipMalloc'd chunk this segment belongs to
        std::vector<Fence> fences;  // free segments: per watched stream, its last fence
    };
    std::map<char *, Seg> segs;                       // by address
    std::set<std::pair<size_t, char *>> free_by_size;  // best fit
    std::map<char *, size_t> chunks;                  // chunk base -> size
    // watched streams; each keeps its recorded fence events in serial order until they complete
    struct Watched {
        hipStream_t s = nullptr;
        int users = 0;
        std::deque<std::pair<uint64_t, hipEvent_t>> pending;
    };
    std::vector<Watched> streams;
    std::vector<hipEvent_t> event_pool;
    uint64_t serial = 0;
    uint64_t in_use = 0, peak = 0;  // bytes handed out now / most since the last reset
    uint64_t fences_recorded = 0, waits = 0;

    hipEvent_t new_event() {
        if (!event_pool.empty()) {
            hipEvent_t e = event_pool.back();
            event_pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        return e;
    }
    // completed fences leave the front of each stream's queue (events complete in stream order)
    void retire() {
        for (auto &w : streams)
            while (!w.pending.empty() && hipEventQuery(w.pending.front().second) == hipSuccess) {
                event_pool.push_back(w.pending.front().second);
                w.pending.pop_front();
            }
        (void)hipGetLastError();  // hipErrorNotReady from the queries
    }
    // the event of fence f while it may be pending, else null (completed, or its stream unwatched)
    hipEvent_t pending_event(const Fence &f) const {
        if (f.slot < 0 || (size_t)f.slot >= streams.size()) return nullptr;
        for (const auto &pe : streams[f.slot].pending)
            if (pe.first == f.serial) return pe.second;
        return nullptr;
    }
    // fences for a block freed now: one per watched stream with work still queued
    std::vector<Fence> fence_now() {
        std::vector<Fence> out;
        for (size_t i = 0; i < streams.size(); ++i) {
            auto &w = streams[i];
            if (!w.s) continue;
            const hipError_t q = hipStreamQuery(w.s);
            if (q == hipSuccess) continue;
            (void)hipGetLastError();
            hipEvent_t e = new_event();
            HIP_OK(hipEventRecord(e, w.s));
            w.pending.push_back({++serial, e});
            out.push_back(Fence{(int)i, serial});
            ++fences_recorded;
        }
        return out;
    }
    static void merge_fences(std::vector<Fence> &a, const std::vector<Fence> &b) {
        for (const Fence &f : b) {
            bool hit = false;
            for (Fence &x : a)
                if (x.slot == f.slot) {
                    x.serial = std::max(x.serial, f.serial);  // later on the same stream: completes later
                    hit = true;
                }
            if (!hit) a.push_back(f);
        }
    }
    // make work on stream `on` (null: the host) wait for the fences of the other streams
    void wait_fences(const std::vector<Fence> &fs, hipStream_t on) {
        for (const Fence &f : fs) {
            if (on && (size_t)f.slot < streams.size() && streams[f.slot].s == on) continue;  // stream order
            hipEvent_t e = pending_event(f);
            if (!e) continue;
            if (hipEventQuery(e) == hipSuccess) continue;
            (void)hipGetLastError();
            ++waits;
            if (on) HIP_OK(hipStreamWaitEvent(on, e, 0));
            else HIP_OK(hipEventSynchronize(e));
        }
    }

    void add_free(char *p, size_t sz, char *chunk, std::vector<Fence> fences = {}) {
        segs[p] = Seg{sz, true, chunk, std::move(fences)};
        free_by_size.insert({sz, p});
    }
    void *take(size_t bytes, hipStream_t on) {
        auto it = free_by_size.lower_bound({bytes, nullptr});
        if (it == free_by_size.end()) return nullptr;
        char *p = it->second;
        const size_t sz = it->first;
        free_by_size.erase(it);
        Seg &s = segs[p];
        s.free = false;
        std::vector<Fence> fences = std::move(s.fences);
        s.fences.clear();
        if (sz - bytes >= kAlign) {
            s.size = bytes;
            add_free(p + bytes, sz - bytes, s.chunk, fences);  // the rest keeps the fences
        }
        in_use += segs[p].size;
        peak = std::max(peak, in_use);
        wait_fences(fences, on);
        return p;
    }
    void give(char *p, std::vector<Fence> fences) {
        auto it = segs.find(p);
        if (it == segs.end()) return;
        it->second.free = true;
        in_use -= it->second.size;
        it->second.fences = std::move(fences);
        // coalesce with the next segment of the same chunk
        auto nx = std::next(it);
        if (nx != segs.end() && nx->second.free && nx->second.chunk == it->second.chunk &&
            it->first + it->second.size == nx->first) {
            free_by_size.erase({nx->second.size, nx->first});
            it->second.size += nx->second.size;
            merge_fences(it->second.fences, nx->second.fences);
            segs.erase(nx);
        }
        // and with the previous one
        if (it != segs.begin()) {
            auto pv = std::prev(it);
            if (pv->second.free && pv->second.chunk == it->second.chunk && pv->first + pv->second.size == it->first) {
                free_by_size.erase({pv->second.size, pv->first});
                pv->second.size += it->second.size;
                merge_fences(pv->second.fences, it->second.fences);
                segs.erase(it);
                it = pv;
            }
        }
        free_by_size.insert({it->second.size, it->first});
    }
    // release chunks that are entirely free (the caller has synchronised the device)
    void trim() {
        for (auto c = chunks.begin(); c != chunks.end();) {
            auto s = segs.find(c->first);
            if (s != segs.end() && s->second.free && s->second.size == c->second) {
                free_by_size.erase({s->second.size, s->first});
                segs.erase(s);
                (void)hipFree(c->first);
                c = chunks.erase(c);
            } else {
                ++c;
            }
        }
    }
};

struct Pools {
    std::mutex mu;
    std::map<int, Arena> by_device;
};
Pools &pools() {
    static Pools *p = new Pools;  // intentionally leaked: outlives static destructors
    return *p;
}
}  // namespace

thread_local hipStream_t tl_alloc_stream = nullptr;

int current_device() {
    int d = 0;
    (void)hipGetDevice(&d);
    return d;
}

hipStream_t alloc_stream() { return tl_alloc_stream; }
void set_alloc_stream(hipStream_t s) { tl_alloc_stream = s; }

void watch_stream(int device, hipStream_t s) {
    if (!s) return;
    std::lock_guard<std::mutex> lk(pools().mu);
    Arena &a = pools().by_device[device];
    for (auto &w : a.streams)
        if (w.s == s) {
            ++w.users;
            return;
        }
    for (auto &w : a.streams)
        if (!w.s) {  // a free slot (its old fences read as complete: pending is empty)
            w.s = s;
            w.users = 1;
            return;
        }
    a.streams.push_back({});
    a.streams.back().s = s;
    a.streams.back().users = 1;
}

void unwatch_stream(int device, hipStream_t s) {
    if (!s) return;
    std::lock_guard<std::mutex> lk(pools().mu);
    Arena &a = pools().by_device[device];
    for (auto &w : a.streams)
        if (w.s == s && --w.users <= 0) {
            (void)hipStreamSynchronize(s);  // its fences complete before the slot can be reused
            for (auto &pe : w.pending) a.event_pool.push_back(pe.second);
            w.pending.clear();
            w.s = nullptr;
            w.users = 0;
        }
}

void *dev_alloc(size_t bytes) {
    bytes = (bytes + kAlign - 1) & ~(kAlign - 1);
    std::lock_guard<std::mutex> lk(pools().mu);
    Arena &a = pools().by_device[current_device()];
    a.retire();
    if (void *p = a.take(bytes, tl_alloc_stream)) return p;
    // a large request's chunk is rounded up to 1/32..1/16 of its size (a power of two), so the
    // next request of about the same size (a count output grown to a few MiB more than last
    // step's) fits in it instead of taking a new chunk: a fresh multi-GB hipMalloc in a timed
    // step once cost 0.7 s on a box whose previous process had just released its memory
    size_t chunk = bytes < kMinChunk ? kMinChunk : bytes;
    if (bytes >= kMinChunk) {
        size_t g = kMinChunk;
        while (g * 32 <= bytes) g <<= 1;
        chunk = (bytes + g - 1) / g * g;
    }
    void *raw = nullptr;
    static const bool verbose = getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1';
    if (verbose) fprintf(stderr, "[mcaat] arena: new chunk of %zu MiB for a %zu MiB request\n", chunk >> 20, bytes >> 20);
    hipError_t e = hipMalloc(&raw, chunk);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        (void)hipDeviceSynchronize();
        if (verbose) fprintf(stderr, "[mcaat] arena: hipMalloc failed, trimming free chunks\n");
        a.retire();
        a.trim();
        chunk = bytes;
        e = hipMalloc(&raw, chunk);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            throw Error(MCAAT_E_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed: " + hipGetErrorString(e));
        }
    }
    char *c = (char *)raw;
    a.chunks[c] = chunk;
    a.add_free(c, chunk, c);
    return a.take(bytes, tl_alloc_stream);
}

void dev_free(void *p, size_t, int device) {
    if (!p) return;
    // the fences are events of the buffer's device, recorded on its streams: a free from a thread
    // whose current device is another one switches for the call (a DevBuf destructor or a free
    // entry point that did not bind its context)
    int cur = device;
    (void)hipGetDevice(&cur);
    if (cur != device) (void)hipSetDevice(device);
    {
        std::lock_guard<std::mutex> lk(pools().mu);
        Arena &a = pools().by_device[device];
        a.retire();
        a.give((char *)p, a.fence_now());
    }
    if (cur != device) (void)hipSetDevice(cur);
}

void dev_trim() {
    std::lock_guard<std::mutex> lk(pools().mu);
    Arena &a = pools().by_device[current_device()];
    (void)hipDeviceSynchronize();
    a.retire();
    a.trim();
}

// a slow fill on one stream (each lane spins ~`spin` clock ticks first), then a fast one
__global__ void k_arena_fill(uint64_t *x, uint64_t n, uint64_t v, uint64_t spin) {
    const uint64_t t0 = wall_clock64();
    while (spin && wall_clock64() - t0 < spin) {
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = v;
}

void arena_check(mcaat_ctx *ctx, int64_t *out) {
    HIP_OK(hipStreamSynchronize(ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->side));
    const uint64_t n = 1u << 22;  // 32 MB
    uint64_t f0 = 0, w0 = 0, f1 = 0, w1 = 0;
    arena_stats(&f0, &w0);
    void *first = nullptr;
    int rate = 0;
    HIP_OK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, ctx->device));  // kHz
    const uint64_t spin = (uint64_t)std::max(rate, 1000) * 50;  // ~50 ms
    {
        DevBuf<uint64_t> a(n);
        first = a.p;
        hipLaunchKernelGGL(k_arena_fill, dim3(256), dim3(256), 0, ctx->stream, a.p, n, 1ull, spin);
        LAUNCH_OK();
    }  // freed while the slow fill is still queued
    DevBuf<uint64_t> b;
    {
        AllocStreamScope scope(ctx->side);
        b.alloc(n);
    }
    hipLaunchKernelGGL(k_arena_fill, dim3(256), dim3(256), 0, ctx->side, b.p, n, 2ull, 0ull);
    LAUNCH_OK();
    HIP_OK(hipStreamSynchronize(ctx->side));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    std::vector<uint64_t> h(n);
    HIP_OK(hipMemcpy(h.data(), b.p, 8 * n, hipMemcpyDeviceToHost));
    bool all2 = true;
    for (uint64_t x : h) all2 = all2 && x == 2;
    arena_stats(&f1, &w1);
    out[0] = b.p == first;
    out[1] = all2;
    out[2] = (int64_t)(w1 - w0);
    b.release();
    // (round 6) a consumer the arena does not watch (a stream of its own, as the FASTQ packer's
    // upload streams): the block is taken with no allocation stream, so the host waits for every
    // pending fence, the allocating stream's own included, before the foreign stream may write it
    HIP_OK(hipStreamSynchronize(ctx->stream));
    {
        DevBuf<uint64_t> a(n);
        first = a.p;
        hipLaunchKernelGGL(k_arena_fill, dim3(256), dim3(256), 0, ctx->stream, a.p, n, 1ull, spin);
        LAUNCH_OK();
    }
    hipStream_t fs = nullptr;
    HIP_OK(hipStreamCreateWithFlags(&fs, hipStreamNonBlocking));
    DevBuf<uint64_t> c;
    {
        AllocStreamScope scope(nullptr);
        c.alloc(n);
    }
    hipLaunchKernelGGL(k_arena_fill, dim3(256), dim3(256), 0, fs, c.p, n, 3ull, 0ull);
    const hipError_t le = hipGetLastError();
    (void)hipStreamSynchronize(fs);
    (void)hipStreamDestroy(fs);
    if (le != hipSuccess) throw Error(MCAAT_E_HIP, std::string("arena check launch: ") + hipGetErrorString(le));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    HIP_OK(hipMemcpy(h.data(), c.p, 8 * n, hipMemcpyDeviceToHost));
    bool all3 = true;
    for (uint64_t x : h) all3 = all3 && x == 3;
    out[3] = c.p == first;
    out[4] = all3;
}

void arena_usage(uint64_t *in_use, uint64_t *peak, uint64_t *reserved, bool reset_peak) {
    std::lock_guard<std::mutex> lk(pools().mu);
    Arena &a = pools().by_device[current_device()];
    uint64_t r = 0;
    for (const auto &c : a.chunks) r += c.second;
    if (in_use) *in_use = a.in_use;
    if (peak) *peak = a.peak;
    if (reserved) *reserved = r;
    if (reset_peak) a.peak = a.in_use;
}

void arena_stats(uint64_t *fences, uint64_t *waits) {
    std::lock_guard<std::mutex> lk(pools().mu);
    Arena &a = pools().by_device[current_device()];
    *fences = a.fences_recorded;
    *waits = a.waits;
}

}  // namespace mcaat
