// alloc.hip — caching device allocator behind DevBuf (see internal.h).
#include <map>
#include <mutex>

#include "internal.h"

namespace mcaat {

namespace {
struct Pool {
    std::mutex mu;
    // device -> (bytes -> cached blocks)
    std::map<int, std::multimap<size_t, void *>> free_blocks;
};
Pool &pool() {
    static Pool *p = new Pool;  // intentionally leaked: outlives static destructors
    return *p;
}
int current_device() {
    int d = 0;
    (void)hipGetDevice(&d);
    return d;
}
}  // namespace

void *dev_alloc(size_t bytes) {
    const int dev = current_device();
    {
        std::lock_guard<std::mutex> lk(pool().mu);
        auto &fb = pool().free_blocks[dev];
        auto it = fb.lower_bound(bytes);
        if (it != fb.end() && it->first <= 2 * bytes + (4u << 20)) {
            void *p = it->second;
            fb.erase(it);
            return p;
        }
    }
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        dev_trim();
        e = hipMalloc(&p, bytes);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            throw Error(MCAAT_E_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed: " + hipGetErrorString(e));
        }
    }
    return p;
}

void dev_free(void *p, size_t bytes) {
    if (!p) return;
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(pool().mu);
    pool().free_blocks[dev].insert({bytes, p});
}

void dev_trim() {
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(pool().mu);
    auto &fb = pool().free_blocks[dev];
    if (!fb.empty()) (void)hipDeviceSynchronize();
    for (auto &kv : fb) (void)hipFree(kv.second);
    fb.clear();
}

}  // namespace mcaat
