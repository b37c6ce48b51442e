/*
 * oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of mcaat's hot path
 * (k-mer/edge counting -> SDBG -> CycleFinder) used as the parity checker.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so. The product (libmcaat_gpu.so, mcaat CLI) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned".
 *   - node_counter / sdbg_build are MEGAHIT (absent un-vendored submodule
 *     .gitmodules:10-12 in the reference, no pinned commit); the conventions
 *     restated here are fixed by this repo (DESIGN.md "SDBG conventions").
 *   - cycle_finder.cpp needs MEGAHIT's sdbg/sdbg.h and phmap headers which are
 *     absent from the image; building it would require stand-in headers, which
 *     this project does not write, so the reference is unbuildable here. The
 *     reference ships no golden vectors for the path. The
 *     restatement is therefore validated by analytic known-answer tests
 *     (tests/test_oracle_known_answer.py) and by libstdc++ order probes.
 */
#ifndef MCAAT_ORACLE_H
#define MCAAT_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_graph oracle_graph;
typedef struct oracle_cf_result oracle_cf_result;

typedef struct {
    uint64_t threshold_multiplicity; /* settings.h:34 */
    int low_abundance;               /* settings.h:35 */
    int cycle_max_length;            /* settings.h:36 */
    int cycle_min_length;            /* settings.h:37 */
    int threads;                     /* settings.h:25; 1 = deterministic reference mode */
    int cluster_bound;               /* cycle_finder.cpp:132 (500) */
    long long step_cap;              /* cycle_finder.cpp:149 (10000000) */
} oracle_cf_params;

/* Exact canonical (k+1)-mer counter. Returns number of distinct canonical edges;
 * *keys (LSB-first packed canonical (k+1)-mers, sorted ascending) and *counts are
 * malloc'ed and owned by the caller (free with oracle_free). */
uint64_t oracle_count_canonical(const uint64_t *packed, const uint64_t *offsets,
                                uint64_t n_reads, int k, int threads,
                                uint64_t **keys, uint32_t **counts);

/* reads -> SDBG (both orientations, BOSS order, multiplicity). */
oracle_graph *oracle_build(const uint64_t *packed, const uint64_t *offsets,
                           uint64_t n_reads, int k, int threads);
/* wrap existing sorted BOSS keys + mult (copied). */
oracle_graph *oracle_graph_from_arrays(const uint64_t *keys, const uint16_t *mult,
                                       uint64_t n, int k);
void oracle_graph_free(oracle_graph *g);
uint64_t oracle_graph_size(const oracle_graph *g);
int oracle_graph_k(const oracle_graph *g);
void oracle_graph_arrays(const oracle_graph *g, uint64_t *keys, uint16_t *mult);
void oracle_graph_valid(const oracle_graph *g, uint8_t *valid); /* one byte per edge */
void oracle_graph_set_valid(oracle_graph *g, const uint8_t *valid);

/* SDBG query API (MEGAHIT subset as used by mcaat) */
int oracle_outgoing(const oracle_graph *g, uint64_t e, uint64_t *out);
int oracle_incoming(const oracle_graph *g, uint64_t e, uint64_t *in);
int oracle_get_label(const oracle_graph *g, uint64_t e, uint8_t *seq);
int64_t oracle_index_binary_search(const oracle_graph *g, const uint8_t *seq);

/* CycleFinder (cycle_finder.cpp:131-492). Mutates the graph's valid bits. */
oracle_cf_result *oracle_cycle_finder(oracle_graph *g, const oracle_cf_params *p);
/* individual stages (for stage-wise GPU parity) */
uint64_t oracle_collect_tips(const oracle_graph *g, uint8_t *tip_flags);
uint64_t oracle_invalidate_mult_one(oracle_graph *g);
void oracle_recursive_reduction(oracle_graph *g, const uint8_t *tip_flags);
int oracle_depth_level_search(const oracle_graph *g, uint64_t start, int limit);

/* result accessors; entries are in commit order (threads=1 reference order) */
uint64_t oracle_cf_n_entries(const oracle_cf_result *r);
void oracle_cf_entries(const oracle_cf_result *r, uint64_t *starts,
                       uint64_t *cyc_begin /* n+1, index into cycle list */);
uint64_t oracle_cf_n_cycles(const oracle_cf_result *r);
uint64_t oracle_cf_n_nodes(const oracle_cf_result *r);
void oracle_cf_cycles(const oracle_cf_result *r, uint64_t *node_begin /* n_cycles+1 */,
                      uint64_t *nodes);
/* iteration order of the reference's unordered_map `results` (indices into entries) */
void oracle_cf_map_order(const oracle_cf_result *r, uint64_t *order);
/* stats: [0]=tips before, [1]=invalidated mult<=1, [2]=valid after prune,
 * [3]=tips after prune, [4]=candidates (passing DLS), [5]=total cycles */
void oracle_cf_stats(const oracle_cf_result *r, uint64_t *stats);
/* candidate start nodes in processing order (bucket desc, id asc) + bucket keys */
uint64_t oracle_cf_n_candidates(const oracle_cf_result *r);
void oracle_cf_candidates(const oracle_cf_result *r, uint64_t *ids, int32_t *bucket);
void oracle_cf_free(oracle_cf_result *r);

void oracle_free(void *p);

/* 4-line FASTQ -> packed 2-bit reads, split at non-ACGT symbols (the counting view of
 * DESIGN.md §2; the CPU leg of the reference's BuildLib, sdbg_build.cpp:82-115). Returns the
 * number of reads; *packed (n_words) and *offsets (n_reads+1) malloc'ed, free with oracle_free;
 * (uint64_t)-1 on an I/O or format error. */
uint64_t oracle_read_fastq(const char *path, uint64_t **packed, uint64_t *n_words, uint64_t **offsets);

/* Relevant reads (reads.cpp:20-130). reverse_pair_ends_sequence in place (reads.cpp:20-31);
 * get_reads over sequences seqs[0..n_file1) of the first file and the rest of the second
 * (reversed and complemented): returns the number of reads, node ids in *flat with
 * n+1 *offsets (malloc'ed; free with oracle_free). */
void oracle_reverse_pair_ends(char *s);
uint64_t oracle_get_reads(const oracle_graph *g, const char *const *seqs, uint64_t n_seqs, uint64_t n_file1,
                          const uint64_t *cycle_nodes, uint64_t n_nodes, uint64_t **flat, uint64_t **offsets);

#ifdef __cplusplus
}
#endif
#endif
