/*
 * mcaat_host.h — C ABI of libmcaat_host.so: the reference's host steps after CycleFinder
 * (relevant reads -> spacer ordering -> get_systems -> CRISPRAnalyzer / CRISPR_Arrays.txt,
 * reference src/main.cpp:544-581), restated in C++ in mcaat_amd/host/ on the SDBG host mirror.
 * The mcaat CLI calls the C++ functions directly; these entry points expose the same code to
 * non-C++ callers (and to the tests) with plain pointers and sizes.
 *
 * Conventions as include/mcaat_gpu.h: 0 on success, a negative mcaat_status on error with the
 * message in mcaat_host_last_error().
 */
#ifndef MCAAT_HOST_H
#define MCAAT_HOST_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char *mcaat_host_last_error(void);

/* rapidfuzz fuzz::ratio / fuzz::partial_ratio as used by CRISPRAnalyzer
 * (post_processing.h:118,137; rapidfuzz-cpp restated, see mcaat_amd/host/fuzz.cpp) */
double mcaat_host_fuzz_ratio(const char *s1, const char *s2);
double mcaat_host_fuzz_partial_ratio(const char *s1, const char *s2);

/* solve_min_cover_problem (spacer_ordering.cpp:265-313): set i = flat[offsets[i]..offsets[i+1]),
 * universe = the n_universe listed elements; chosen set indices ascending in out (capacity
 * n_sets), their number in *n_out (0 when the reference returns {}). */
int mcaat_host_min_cover(const uint32_t *universe, size_t n_universe, const uint32_t *flat, const uint64_t *offsets,
                         size_t n_sets, uint64_t *out, size_t *n_out);

/* Steps 7-8 + CRISPRAnalyzer on a host copy of the graph (sorted BOSS keys, multiplicities,
 * valid bytes after CycleFinder), the cycles (cycles_map_to_cycles order) and the relevant
 * reads (get_reads order): run_and_debug_spacer_ordering (main_run_and_debug.cpp:32-143), then
 * CRISPRAnalyzer(all_systems, output_file).run_analysis(). *n_found = found systems before the
 * analyzer's filters. The graph's valid bytes are updated in place (the reference mutates them).
 * threads (<= 1: one) solves the independent subproblems in parallel; the output is the same. */
int mcaat_host_crispr_arrays(int k, const uint64_t *keys, const uint16_t *mult, uint8_t *valid, uint64_t D,
                             const uint64_t *cycles_flat, const uint64_t *cycle_offsets, size_t n_cycles,
                             const uint64_t *reads_flat, const uint64_t *read_offsets, size_t n_reads,
                             const char *output_file, size_t *n_found, int threads);

/* CRISPRAnalyzer alone (post_processing.h): systems given as repeats[i] with spacers
 * joined by ',' in spacers[i], inserted into the unordered_map in index order. */
int mcaat_host_crispr_analyzer(const char *const *repeats, const char *const *spacers, size_t n,
                               const char *output_file);

#ifdef __cplusplus
}
#endif
#endif
