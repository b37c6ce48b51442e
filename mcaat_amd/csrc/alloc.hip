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
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>

#include "internal.h"

namespace mcaat {

namespace {

constexpr size_t kAlign = 256;
constexpr size_t kMinChunk = 256ull << 20;  // grow by at least 256 MiB

struct Arena {
    struct Seg {
        size_t size;
        bool free;
        char *chunk;  // base of the hipMalloc'd chunk this segment belongs to
    };
    std::map<char *, Seg> segs;                       // by address
    std::set<std::pair<size_t, char *>> free_by_size;  // best fit
    std::map<char *, size_t> chunks;                  // chunk base -> size

    void add_free(char *p, size_t sz, char *chunk) {
        segs[p] = Seg{sz, true, chunk};
        free_by_size.insert({sz, p});
    }
    void *take(size_t bytes) {
        auto it = free_by_size.lower_bound({bytes, nullptr});
        if (it == free_by_size.end()) return nullptr;
        char *p = it->second;
        const size_t sz = it->first;
        free_by_size.erase(it);
        Seg &s = segs[p];
        s.free = false;
        if (sz - bytes >= kAlign) {
            s.size = bytes;
            add_free(p + bytes, sz - bytes, s.chunk);
        }
        return p;
    }
    void give(char *p) {
        auto it = segs.find(p);
        if (it == segs.end()) return;
        it->second.free = true;
        // coalesce with the next segment of the same chunk
        auto nx = std::next(it);
        if (nx != segs.end() && nx->second.free && nx->second.chunk == it->second.chunk &&
            it->first + it->second.size == nx->first) {
            free_by_size.erase({nx->second.size, nx->first});
            it->second.size += nx->second.size;
            segs.erase(nx);
        }
        // and with the previous one
        if (it != segs.begin()) {
            auto pv = std::prev(it);
            if (pv->second.free && pv->second.chunk == it->second.chunk && pv->first + pv->second.size == it->first) {
                free_by_size.erase({pv->second.size, pv->first});
                pv->second.size += it->second.size;
                segs.erase(it);
                it = pv;
            }
        }
        free_by_size.insert({it->second.size, it->first});
    }
    // release chunks that are entirely free
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

int current_device() {
    int d = 0;
    (void)hipGetDevice(&d);
    return d;
}

void *dev_alloc(size_t bytes) {
    bytes = (bytes + kAlign - 1) & ~(kAlign - 1);
    std::lock_guard<std::mutex> lk(pools().mu);
    Arena &a = pools().by_device[current_device()];
    if (void *p = a.take(bytes)) return p;
    size_t chunk = bytes < kMinChunk ? kMinChunk : bytes;
    void *raw = nullptr;
    static const bool verbose = getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1';
    if (verbose) fprintf(stderr, "[mcaat] arena: new chunk of %zu MiB for a %zu MiB request\n", chunk >> 20, bytes >> 20);
    hipError_t e = hipMalloc(&raw, chunk);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        (void)hipDeviceSynchronize();
        if (verbose) fprintf(stderr, "[mcaat] arena: hipMalloc failed, trimming free chunks\n");
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
    return a.take(bytes);
}

void dev_free(void *p, size_t, int device) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(pools().mu);
    pools().by_device[device].give((char *)p);
}

void dev_trim() {
    std::lock_guard<std::mutex> lk(pools().mu);
    Arena &a = pools().by_device[current_device()];
    (void)hipDeviceSynchronize();
    a.trim();
}

}  // namespace mcaat
