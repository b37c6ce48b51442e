// IdMap (mcaat_amd/host/mcaat_host.h), the host mirror's open-addressing map, against
// std::unordered_map on random keys that include ~0 (a read's absent label, which IdMap keeps
// beside its table because it is the empty-slot marker), with and without reserve(); built with
// the sanitizer flags of this directory (tests/test_sanitizers.py).
#include <cstdio>
#include <random>
#include <unordered_map>

#include "../../mcaat_amd/host/mcaat_host.h"

int main() {
    std::mt19937_64 rng(1);
    for (int trial = 0; trial < 40; ++trial) {
        IdMap<uint32_t> m;
        std::unordered_map<uint64_t, uint32_t> u;
        const int n = 1 + (int)(rng() % 5000);
        if (trial % 2) m.reserve((size_t)n);
        for (int i = 0; i < n; ++i) {
            const uint64_t k = rng() % 50 == 0 ? ~0ULL : rng() % 100000;
            const uint32_t v = (uint32_t)(rng() % 100);
            m[k] = v;
            u[k] = v;
        }
        for (uint64_t kk = 0; kk <= 100000; ++kk) {
            const uint64_t k = kk == 100000 ? ~0ULL : kk;
            const uint32_t *p = m.find(k);
            const auto it = u.find(k);
            if ((p == nullptr) != (it == u.end()) || (p && *p != it->second) || m.contains(k) != (it != u.end())) {
                std::printf("MISMATCH trial %d key %llu\n", trial, (unsigned long long)k);
                return 1;
            }
        }
        if (m.size() != u.size()) {
            std::printf("size mismatch trial %d: %zu vs %zu\n", trial, (size_t)m.size(), u.size());
            return 1;
        }
    }
    std::printf("idmap ok\n");
    return 0;
}
