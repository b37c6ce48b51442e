// capi_host.cpp — extern "C" entry points of libmcaat_host.so (include/mcaat_host.h).
#include <algorithm>
#include <cstring>
#include <sstream>

#include "../../include/mcaat_host.h"
#include "downstream.h"

namespace {

thread_local std::string g_err;

template <class F>
int guarded(F &&f) {
    try {
        f();
        return 0;
    } catch (const std::bad_alloc &) {
        g_err = "host allocation failed";
        return MCAAT_E_NOMEM;
    } catch (const std::exception &e) {
        g_err = e.what();
        return MCAAT_E_INVALID;
    }
}

std::vector<std::vector<uint64_t>> unflatten(const uint64_t *flat, const uint64_t *off, size_t n) {
    std::vector<std::vector<uint64_t>> v(n);
    for (size_t i = 0; i < n; ++i) v[i].assign(flat + off[i], flat + off[i + 1]);
    return v;
}

}  // namespace

extern "C" {

const char *mcaat_host_last_error(void) { return g_err.c_str(); }

double mcaat_host_fuzz_ratio(const char *s1, const char *s2) { return fuzz::ratio(s1, s2); }
double mcaat_host_fuzz_partial_ratio(const char *s1, const char *s2) { return fuzz::partial_ratio(s1, s2); }

int mcaat_host_min_cover(const uint32_t *universe, size_t n_universe, const uint32_t *flat, const uint64_t *offsets,
                         size_t n_sets, uint64_t *out, size_t *n_out) {
    return guarded([&] {
        if (!n_out || (n_universe && !universe) || (n_sets && (!flat || !offsets || !out)))
            throw std::invalid_argument("null argument");
        std::unordered_set<uint32_t> u(universe, universe + n_universe);
        std::vector<std::vector<uint32_t>> sets(n_sets);
        for (size_t i = 0; i < n_sets; ++i) sets[i].assign(flat + offsets[i], flat + offsets[i + 1]);
        const auto r = solve_min_cover_problem(u, sets);
        for (size_t i = 0; i < r.size(); ++i) out[i] = r[i];
        *n_out = r.size();
    });
}

int mcaat_host_crispr_arrays(int k, const uint64_t *keys, const uint16_t *mult, uint8_t *valid, uint64_t D,
                             const uint64_t *cycles_flat, const uint64_t *cycle_offsets, size_t n_cycles,
                             const uint64_t *reads_flat, const uint64_t *read_offsets, size_t n_reads,
                             const char *output_file, size_t *n_found, int threads) {
    return guarded([&] {
        if (!keys || !mult || !valid || !cycle_offsets || !read_offsets || !output_file)
            throw std::invalid_argument("null argument");
        SDBG sdbg;
        sdbg.LoadFromArrays(k, std::vector<uint64_t>(keys, keys + D), std::vector<uint16_t>(mult, mult + D),
                            std::vector<uint8_t>(valid, valid + D));
        const auto cycles = unflatten(cycles_flat, cycle_offsets, n_cycles);
        const auto reads = unflatten(reads_flat, read_offsets, n_reads);
        const auto found = run_and_debug_spacer_ordering(reads, sdbg, cycles, (unsigned)std::max(1, threads));
        std::unordered_map<std::string, std::vector<std::string>> all_systems;
        for (const auto &[_s, repeat, spacers, _a, _b] : found) all_systems[repeat] = spacers;
        CRISPRAnalyzer analyzer(all_systems, output_file);
        analyzer.run_analysis();
        for (uint64_t e = 0; e < D; ++e) valid[e] = sdbg.IsValidEdge(e) ? 1 : 0;
        if (n_found) *n_found = found.size();
    });
}

int mcaat_host_crispr_analyzer(const char *const *repeats, const char *const *spacers, size_t n,
                               const char *output_file) {
    return guarded([&] {
        if ((n && (!repeats || !spacers)) || !output_file) throw std::invalid_argument("null argument");
        std::unordered_map<std::string, std::vector<std::string>> systems;
        for (size_t i = 0; i < n; ++i) {
            std::vector<std::string> sp;
            std::stringstream ss(spacers[i]);
            std::string t;
            while (std::getline(ss, t, ','))
                if (!t.empty()) sp.push_back(t);
            systems[repeats[i]] = sp;
        }
        CRISPRAnalyzer analyzer(systems, output_file);
        analyzer.run_analysis();
    });
}

}  // extern "C"
