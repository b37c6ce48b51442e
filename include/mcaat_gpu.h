/*
 * mcaat_gpu.h — C ABI of the MI355X-native mcaat hot path
 * (node_counter -> sdbg_build -> cycle_finder). Plain pointers and sizes only.
 *
 * The reference has no FFI for this path; its boundary is three C++ classes that
 * share one Settings object. Each entry point below names the
 * reference interface it replaces. The host-side C++ mirror (mcaat_amd/host/)
 * keeps the reference class names (SDBGBuild, SDBG, CycleFinder) on top of this ABI.
 *
 * Conventions: every int-returning call returns 0 (MCAAT_OK) on success or a negative
 * mcaat_status; mcaat_last_error() gives a thread-local message (the host mirror turns
 * it into std::runtime_error, as cycle_finder.cpp:135 does). The library owns device
 * buffers; the caller owns handles and frees them. Calls on one mcaat_ctx must come
 * from one host thread (not reentrant per ctx); one ctx drives one GPU on one HIP stream.
 * Every call is synchronous with respect to the host unless stated.
 */
#ifndef MCAAT_GPU_H
#define MCAAT_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum mcaat_status {
    MCAAT_OK = 0,
    MCAAT_E_INVALID = -1,  /* bad argument */
    MCAAT_E_HIP = -2,      /* HIP runtime error (no GPU, launch failure) */
    MCAAT_E_NOMEM = -3,    /* device or host allocation failed */
    MCAAT_E_IO = -4,       /* file open/parse failure */
    MCAAT_E_CAPACITY = -5  /* a bounded structure overflowed and could not be regrown */
};

typedef struct mcaat_ctx mcaat_ctx;
typedef struct mcaat_reads mcaat_reads;
typedef struct mcaat_graph mcaat_graph;
typedef struct mcaat_cycles mcaat_cycles;
typedef struct mcaat_counts mcaat_counts;
typedef struct mcaat_mapped mcaat_mapped;
typedef struct mcaat_comm mcaat_comm;

/* ---- context ------------------------------------------------------------- */
/* Replaces: nothing in the reference (single process, OpenMP). Binds one GPU. */
int mcaat_init(int device, mcaat_ctx **out);
void mcaat_finalize(mcaat_ctx *ctx);
/* release the device memory the context's arena holds but no live object uses (the arena keeps
 * freed blocks for the next step; another process on the same GPU may need them) */
void mcaat_trim(mcaat_ctx *ctx);
const char *mcaat_last_error(void);
int mcaat_device_count(int *n);
/* load the hot path's kernel code objects on `device` now rather than at each one's first launch
 * (HIP's deferred loading); the CLI calls it with the runtime init, before its timed span */
int mcaat_preload(int device);

/* ---- reads ----------------------------------------------------------------
 * Replaces: SDBGBuild::BuildLib / SequenceLibCollection::Build (sdbg_build.cpp:82-115):
 * FASTQ/FASTA(.gz) -> 2-bit packed read library, here resident in HBM.
 * Packed stream: base j at word j>>5, bits 2*(j&31), A=0 C=1 G=2 T=3.
 * offsets[n_reads+1] are base offsets of each read in the stream. */
int mcaat_reads_from_host(mcaat_ctx *ctx, const uint64_t *packed, uint64_t n_words,
                          const uint64_t *offsets, uint64_t n_reads, mcaat_reads **out);
/* Non-ACGT symbols split a read (k-mers spanning them are dropped). gzip via zlib, bzip2 via
 * libbz2 (opened at run time; concatenated members / streams read in sequence).
 * FASTQ inputs (4-line records) are parsed on the GPU in chunks (csrc/fastq_ingest.hip;
 * chunk size MCAAT_FASTQ_CHUNK bytes, default 256 MiB); FASTA (multi-line) on the host.
 * Blank lines are accepted only before the first and after the last record. */
int mcaat_reads_from_fastx(mcaat_ctx *ctx, const char *const *files, int n_files, mcaat_reads **out);
/* (round 5) The next mcaat_reads_from_fastx on ctx runs node_counter's pass A for k (the
 * super-k-mer scatter of the k+1-mers) on each part of a host-packed FASTQ input while the
 * input is still being read, and the reads keep the result for the first count / graph build
 * with that k (mcaat_build_graph, mcaat_count_edges, mcaat_count_local). Results are the same
 * as without it. Inputs the host packer does not take, reads of differing lengths, or an
 * under-estimated input size fall back to pass A after the read. One read uses it; k = 0
 * cancels. Replaces: nothing (the reference's BuildLib and Read2SdbgS2 run one after the
 * other, sdbg_build.cpp:82-115, 171-187). */
int mcaat_count_ahead(mcaat_ctx *ctx, int k);
int mcaat_reads_info(const mcaat_reads *r, uint64_t *n_reads, uint64_t *n_bases);
/* Mapping view used by mcaat_map_reads: one entry per input record (first file as is,
 * second file reversed and complemented as reads.cpp:20-31 does; any symbol other than
 * A/C/G maps like T, reads.cpp:44-52). *separate = 0 when it is the counting view itself
 * (one input file, ACGT only, or reads not loaded from files). */
int mcaat_reads_records_info(const mcaat_reads *r, uint64_t *n_records, int *separate);
int mcaat_reads_download(const mcaat_reads *r, uint64_t *packed, uint64_t *offsets);
/* the mapping view (records) as packed stream + offsets[n_records+1]; the counting view
 * when records_info says it is not separate. Replaces the FASTQ re-parse of reads.cpp:88-130. */
int mcaat_reads_records_download(const mcaat_reads *r, uint64_t *packed, uint64_t *offsets);
/* The counting view written as 4-line FASTQ (header "@r", quality 'I'), formatted by
 * `threads` host threads: a FASTQ input for mcaat_reads_from_fastx / the CLI made from
 * resident reads (synthetic configs). Replaces: nothing in the reference. */
int mcaat_reads_write_fastq(const mcaat_reads *r, const char *path, int threads);
void mcaat_reads_free(mcaat_reads *r);

/* Synthetic metagenome: iid genomes with CRISPR arrays inserted,
 * reads with substitution errors, generated directly in HBM by a counter-based RNG. */
typedef struct {
    uint64_t seed;
    uint32_t n_genomes;
    uint64_t genome_len;
    uint32_t arrays_per_genome;
    uint32_t spacers_per_array;
    uint32_t repeat_len_min, repeat_len_max;
    uint32_t spacer_len_min, spacer_len_max;
    uint32_t read_len;
    uint64_t n_reads;
    double error_rate;
    int32_t paired; /* 1: pairs (fragment 300+-30, R2 = reverse complement of fragment end) */
} mcaat_synth_spec;
int mcaat_reads_synth(mcaat_ctx *ctx, const mcaat_synth_spec *spec, mcaat_reads **out);
/* reads [first, first+count) of the same stream: a rank's slice of one dataset */
int mcaat_reads_synth_range(mcaat_ctx *ctx, const mcaat_synth_spec *spec, uint64_t first, uint64_t count,
                            mcaat_reads **out);
/* host-side generator of the same reads (for tests and FASTQ fixtures) */
int mcaat_synth_host(const mcaat_synth_spec *spec, uint64_t *packed, uint64_t *offsets);
/* the genome sequences (n_genomes*genome_len bases, packed) and array truth */
int mcaat_synth_genome_host(const mcaat_synth_spec *spec, uint64_t *packed);
/* the planted CRISPR arrays as text, one line per array: "genome<TAB>index<TAB>repeat<TAB>
 * spacer1,spacer2,...\n" (ACGT, genome strand). *len = the full length; at most cap-1 bytes and
 * a terminating 0 are written to text (text may be null to ask the length). The ground truth a
 * reference run would take as its benchmark file (settings benchmark_file, main.cpp:559-569). */
int mcaat_synth_arrays_host(const mcaat_synth_spec *spec, char *text, uint64_t cap, uint64_t *len);

/* ---- node_counter ----------------------------------------------------------
 * Replaces: the multiplicity counting inside MEGAHIT Read2SdbgS2::Run
 * (sdbg_build.cpp:171-187). Exact canonical (k+1)-mer counts; results copied to
 * host buffers allocated with malloc (free with mcaat_free). Keys are LSB-first
 * canonical (k+1)-mers, sorted ascending. */
int mcaat_count_edges(mcaat_ctx *ctx, const mcaat_reads *r, int k, uint64_t *n_distinct,
                      uint64_t **keys, uint32_t **counts);
void mcaat_free(void *p);

/* ---- sdbg_build --------------------------------------------------------------
 * Replaces: SDBGBuild::SDBGBuild(Settings) + SDBG::LoadFromFile (sdbg_build.cpp:3-13,
 * 196-232; main.cpp:517-530). k is hard-coded to 23 in the reference
 * (sdbg_build.cpp:217); any 2 <= k <= 30 is accepted here. The graph stays in HBM. */
int mcaat_build_graph(mcaat_ctx *ctx, const mcaat_reads *r, int k, mcaat_graph **out);
int mcaat_graph_info(const mcaat_graph *g, int *k, uint64_t *n_edges);
/* Host view for the SDBG mirror (MEGAHIT SDBG API subset):
 * BOSS keys, multiplicities and one valid byte per edge (any pointer may be NULL). */
int mcaat_graph_download(const mcaat_graph *g, uint64_t *keys, uint16_t *mult, uint8_t *valid);
/* the same for edges [first, first+count) (paged host views of graphs larger than host RAM) */
int mcaat_graph_download_range(const mcaat_graph *g, uint64_t first, uint64_t count, uint64_t *keys, uint16_t *mult,
                               uint8_t *valid);
/* the valid bitmap as it is on the device: (n_edges + 63) / 64 words, edge e at bit e % 64 of
 * word e / 64 (the host SDBG mirror's IsValidEdge without a byte per edge: C3 126 MB, not 1 GB) */
int mcaat_graph_valid_words(const mcaat_graph *g, uint64_t *words);
/* Keeps device valid bits coherent with host SetInvalidEdge/SetValidEdge
 * (spacer_ordering.cpp:96-138 mutates them downstream). */
int mcaat_graph_set_valid(mcaat_graph *g, const uint64_t *ids, size_t n, int valid);
/* Batched device queries (OutgoingEdges/IncomingEdges, valid-only): out[4*i..] and
 * counts[i] for each id; order DESCENDING for outgoing, ASCENDING for incoming. */
int mcaat_graph_neighbors(const mcaat_graph *g, const uint64_t *ids, size_t n, int incoming,
                          uint64_t *out, int32_t *counts);
/* BOSS keys and multiplicities of n edges (either output may be null): the host SDBG mirror's
 * label queries for a set of nodes (GetLabel, sdbg.h) without downloading the whole graph */
int mcaat_graph_gather(const mcaat_graph *g, const uint64_t *ids, size_t n, uint64_t *keys, uint16_t *mult);
/* valid &= {ids}: keep_crispr_regions_extended_by_k (spacer_ordering.cpp:129-137) invalidates
 * every valid edge outside the extended cycle set; here one bitmap AND on the device. */
int mcaat_graph_keep_only(mcaat_graph *g, const uint64_t *ids, size_t n);
/* keep_crispr_regions_extended_by_k (spacer_ordering.cpp:78-138) whole on the device: the seeds
 * grown by `hops` rounds over the valid in- and out-neighbours of the valid frontier nodes, then
 * valid &= that region (one call instead of a host BFS of 2 x hops neighbour queries). */
int mcaat_graph_keep_region(mcaat_graph *g, const uint64_t *seeds, size_t n, uint64_t hops);
/* The valid edges and their valid out-edges as a dense graph (step 7's SCC split, Tarjan over a
 * few hundred thousand edges): *n_valid valid edge ids ascending into ids[], and for each its
 * out-neighbours (OutgoingEdges order, DESCENDING ids) as positions in ids[] at nbr[4i..4i+counts[i]).
 * With ids, nbr and counts all NULL only *n_valid is set (size the arrays, call again). */
int mcaat_graph_valid_subgraph(const mcaat_graph *g, uint64_t *n_valid, uint64_t *ids, uint32_t *nbr, uint8_t *counts);
/* Succinct (BOSS) view. Replaces: the representation of MEGAHIT's SDBG (sdbg_build.cpp:175-186
 * writes it, main.cpp:522-530 loads it; SURVEY.md §8a5, ~3 B/edge): per edge a nibble of W, last
 * and W-minus, per node (sources and targets, colex order) a sink and a has-in bit, 16-bit block
 * ranks and select samples; neighbour queries by rank/select (csrc/sdbg_succinct.hip). Built from
 * the graph as it is (valid bits included), checked against its arrays (every edge's valid out-
 * and in-neighbours, order included, when check != 0) and timed beside them. out[8]: [0] bytes of
 * the view, [1] bytes of the arrays it replaces (keys, out_info, in_info; mult and the valid
 * bitmap are shared), [2] out-list mismatches (+2^40 when the two out-degree scans disagree),
 * [3] in-list mismatches, [4] nodes (sources and sinks), [5] sinks, [6] / [7] the sums of the
 * valid out- / in-degrees of the valid edges. ms[6]: [0] the build, [1] / [2] the out-degree scan
 * on out_info / on the view (per-lane rank/select), [3] / [4] the in-degree scan on in_info / on
 * the view, [5] the out-degree scan on the view with the selects streamed over each wave. One
 * GPU (not a sharded graph). */
int mcaat_graph_succinct_check(mcaat_graph *g, int check, uint64_t *out, double *ms);
/* Checkpoint / resume. Replaces: the on-disk graph between SDBGBuild and CycleFinder
 * (MEGAHIT graph.sdbg* + SDBG::LoadFromFile, main.cpp:386-393, 522-530). The library's own
 * format (MEGAHIT's is unpinned offline): sorted BOSS keys, multiplicities and valid bits with
 * a checksum; adjacency and directory are rebuilt on load, so the loaded graph answers every
 * query as the saved one (valid bits included, e.g. after CycleFinder). */
int mcaat_graph_save(const mcaat_graph *g, const char *path);
int mcaat_graph_load(mcaat_ctx *ctx, const char *path, mcaat_graph **out);
void mcaat_graph_free(mcaat_graph *g);

/* ---- relevant-read mapping -------------------------------
 * Replaces: get_reads (reads.cpp:88-130) with get_read_from_sequence (reads.cpp:57-86)
 * and k_mer_to_node_id (reads.cpp:33-55): every record of the mapping view whose length
 * exceeds 2k and whose first or last k-mer's IndexBinarySearch id is one of cycle_nodes
 * is returned, in input order, as the ids of all its len-k+1 k-mers (~0 = absent label,
 * the reference's -1). max_batch_ids bounds the device output buffer (0: 2^28 ids).
 * Results stay valid until mcaat_mapped_free; records[i] is the mapping-view index. */
int mcaat_map_reads(const mcaat_graph *g, const mcaat_reads *r, const uint64_t *cycle_nodes, size_t n_nodes,
                    uint64_t max_batch_ids, mcaat_mapped **out);
int mcaat_mapped_get(const mcaat_mapped *m, uint64_t *n_reads, const uint64_t **ids, const uint64_t **offsets,
                     const uint64_t **records);
void mcaat_mapped_free(mcaat_mapped *m);

/* ---- multi-GPU build (one process per GPU) ---------------------
 * Replaces: the single-process Read2SdbgS2::Run of sdbg_build.cpp:171-187 when the reads
 * are split over ranks. Each rank counts its reads (mcaat_count_local), the ranks agree on
 * owner ranges of the BOSS key from the summed histogram (mcaat_counts_histogram), each
 * rank groups its oriented (BOSS key, partial count) pairs by owner
 * (mcaat_counts_partition), the caller exchanges them (all-to-all over RCCL), each owner
 * sorts and sums its pairs (mcaat_edges_reduce), the caller all-gathers the owners' arrays
 * in rank order, and every rank builds the graph from them (mcaat_graph_from_sorted).
 * Device pointers (_dev) are caller-owned device memory on this ctx's GPU. */
int mcaat_count_local(mcaat_ctx *ctx, const mcaat_reads *r, int k, mcaat_counts **out);
int mcaat_counts_info(const mcaat_counts *c, uint64_t *n_canonical);
/* hist[2^bits] (host): oriented edges per value of the top `bits` of the 2(k+1)-bit BOSS key */
int mcaat_counts_histogram(const mcaat_counts *c, int bits, uint64_t *hist);
/* owner o takes BOSS keys in [splits[o-1], splits[o]) (splits ascending, n_owners-1 of them);
 * writes the pairs owner-major into keys_dev/counts_dev (cap entries, >= 2 * n_canonical)
 * and sizes[o] (host). Palindromes contribute one pair with twice the count. */
int mcaat_counts_partition(const mcaat_counts *c, int n_owners, const uint64_t *splits, uint64_t *sizes,
                           uint64_t *keys_dev, uint32_t *counts_dev, uint64_t cap);
void mcaat_counts_free(mcaat_counts *c);
/* sorts n received pairs by key and sums the counts of equal keys (saturating at 65535):
 * *n_out unique keys ascending in keys_out_dev, multiplicities in mult_out_dev (n entries) */
int mcaat_edges_reduce(mcaat_ctx *ctx, int k, const uint64_t *keys_dev, const uint32_t *counts_dev, uint64_t n,
                       uint64_t *keys_out_dev, uint16_t *mult_out_dev, uint64_t *n_out);
/* graph from D ascending unique BOSS keys and their multiplicities (copied) */
int mcaat_graph_from_sorted(mcaat_ctx *ctx, int k, const uint64_t *keys_dev, const uint16_t *mult_dev, uint64_t D,
                            mcaat_graph **out);

/* ---- cycle_finder ------------------------------------------------------------
 * Replaces: CycleFinder::CycleFinder(Settings&) -> FindApproximateCRISPRArrays
 * (cycle_finder.cpp:131-138, 433-492). Mutates the graph's valid bits exactly as the
 * reference mutates the SDBG. Results follow the reference's threads=1 commit order
 * (bucket by descending ceil(log2 mult), ascending edge id inside a bucket). */
typedef struct {
    uint64_t threshold_multiplicity; /* settings.h:34 (default 20) */
    int32_t low_abundance;           /* settings.h:35 (default 1)  */
    int32_t cycle_max_length;        /* settings.h:36 (default 77) */
    int32_t cycle_min_length;        /* settings.h:37 (default 27) */
    int32_t cluster_bound;           /* cycle_finder.cpp:132 (500) */
    int64_t step_cap;                /* cycle_finder.cpp:149 (10000000) */
} mcaat_cf_params;
void mcaat_cf_default_params(mcaat_cf_params *p);
int mcaat_cycle_finder(mcaat_graph *g, const mcaat_cf_params *p, mcaat_cycles **out);
/* number of `results` entries (start nodes with an entry, possibly empty) */
int mcaat_cycles_count(const mcaat_cycles *c, size_t *n_entries);
/* entry i in commit order: start node, its cycles as one flat node array plus
 * n_cycles+1 offsets into it; pointers stay valid until mcaat_cycles_free */
int mcaat_cycles_get(const mcaat_cycles *c, size_t i, uint64_t *start, const uint64_t **flat,
                     const uint64_t **offsets, size_t *n_cycles);
/* All entries at once, flattened (bulk consumers): sizes[3] = {entries, cycles, node ids}.
 * Call with the four arrays NULL to size them; then entry i starts at starts[i], owns cycles
 * [entry_offsets[i], entry_offsets[i+1]) and cycle q is nodes[cycle_offsets[q] ..
 * cycle_offsets[q+1]). Same commit order as mcaat_cycles_get. */
int mcaat_cycles_export(const mcaat_cycles *c, uint64_t *sizes, uint64_t *starts, uint64_t *entry_offsets,
                        uint64_t *cycle_offsets, uint64_t *nodes);
/* stats: [0] tips before pruning, [1] invalidated mult<=1, [2] valid after pruning,
 * [3] tips after pruning, [4] start candidates passing DLS, [5] total cycles,
 * [6] FindCycle speculation rounds, [7] FindCycle re-runs after conflicts */
int mcaat_cycles_stats(const mcaat_cycles *c, uint64_t *stats);
/* start candidates in processing order and their ceil(log2 mult) bucket */
int mcaat_cycles_candidates(const mcaat_cycles *c, size_t *n, const uint64_t **ids, const int32_t **buckets);
void mcaat_cycles_free(mcaat_cycles *c);

/* ---- multi-GPU, native (one process per GPU) ----------
 * Replaces: nothing in the reference (one process, OpenMP); the C++ host drives a multi-GPU
 * run through these. A communicator joins the `world` processes of one run:
 *   RCCL: rank 0 makes a 128-byte id (mcaat_comm_unique_id), the caller hands it to every
 *         rank (pipe, file, torch.distributed), each rank calls mcaat_comm_init_rccl on its
 *         own GPU; device data moves GPU to GPU over xGMI.
 *   SHM:  every rank calls mcaat_comm_init_shm with the same "/name" (POSIX shared memory,
 *         removed once all ranks are attached); device data is staged through host memory
 *         (ranks sharing one GPU, rehearsals). ctx may be NULL: host collectives only.
 * Every comm call is collective (all ranks, same order) and synchronous. */
#define MCAAT_COMM_ID_BYTES 128
int mcaat_comm_unique_id(uint8_t *id);
int mcaat_comm_init_rccl(mcaat_ctx *ctx, int world, int rank, const uint8_t *id, mcaat_comm **out);
/* slot_bytes: staging bytes per rank (0: 256 MiB); larger messages move in rounds */
int mcaat_comm_init_shm(mcaat_ctx *ctx, int world, int rank, const char *name, uint64_t slot_bytes,
                        mcaat_comm **out);
int mcaat_comm_info(const mcaat_comm *c, int *world, int *rank);
/* Host-only self-check of the RCCL segment all-to-all's schedule (csrc/comm.hip seg_schedule, the
 * function the RCCL transport runs): every rank's schedule for random segment lists of `world`
 * ranks cut into piece_bytes pieces; checks that each pair's j-th send piece equals the peer's
 * j-th receive piece and that the pieces tile the segments and the output. *rounds = the most
 * rounds of any rank. No GPU, no communicator (this pool's boxes have one GPU, so the RCCL
 * transport's multi-rank grouping is exercised here on the host, not over xGMI). */
int mcaat_comm_schedule_check(int world, uint64_t seed, uint64_t piece_bytes, uint64_t *rounds);
int mcaat_comm_barrier(mcaat_comm *c);
/* host memory: sizes[world] = every rank's byte count; then the bytes in rank order */
int mcaat_comm_allgather_sizes(mcaat_comm *c, uint64_t bytes, uint64_t *sizes);
int mcaat_comm_allgatherv(mcaat_comm *c, const void *send, uint64_t bytes, void *recv, const uint64_t *sizes);
void mcaat_comm_free(mcaat_comm *c);
/* Part `part` of n_parts of the FASTQ inputs (replaces BuildLib for one rank): each plain
 * file is cut at 4-line record starts near part/n_parts of its size, a .gz file goes whole
 * to part 0 (one inflate stream cannot be split). MCAAT_E_IO for inputs the GPU parser does
 * not take (FASTA, wrapped or gapped records): read them whole with mcaat_reads_from_fastx
 * on one rank instead. n_parts == 1 is mcaat_reads_from_fastx. */
int mcaat_reads_from_fastx_part(mcaat_ctx *ctx, const char *const *files, int n_files, int part, int n_parts,
                                mcaat_reads **out);
/* mapping-view records that came from input file `file` (they are in file order) */
int mcaat_reads_file_records(const mcaat_reads *r, int file, uint64_t *n_records);
/* The graph of all ranks' reads (each passes its own part), built with one key-range
 * all-to-all and one all-gather; every rank receives the whole graph, edge ids identical to
 * mcaat_build_graph over all the reads. Replaces Read2SdbgS2::Run (sdbg_build.cpp:171-187). */
int mcaat_build_graph_sharded(mcaat_ctx *ctx, mcaat_comm *comm, const mcaat_reads *r, int k, mcaat_graph **out);
/* CycleFinder over ranks that each hold the same graph: pruning runs on every rank, the
 * start-candidate scan is split by id range, DepthLevelSearch and FindCycle starts are dealt
 * round-robin with one ordered commit; every rank gets the results mcaat_cycle_finder gives
 * (comm NULL: mcaat_cycle_finder). Replaces cycle_finder.cpp:394-419, 468-487. */
int mcaat_cycle_finder_comm(mcaat_graph *g, mcaat_comm *comm, const mcaat_cf_params *p, mcaat_cycles **out);
/* (round 5) Per-shard graphs. By default (knob dist.shard_cf = 1) mcaat_build_graph_sharded
 * leaves each rank its BOSS-key range of the edges (ids [first, first + n_local)) with its
 * adjacency built by one request/response exchange, and mcaat_cycle_finder_comm on such a graph
 * runs CycleFinder per shard (filter, tips, degrees and the RecursiveReduction fixpoint over
 * the ranks' ranges with message exchanges; DepthLevelSearch and FindCycle on gathered
 * search-region replicas): the same results as mcaat_cycle_finder. Entry points that read the
 * whole graph (download, neighbours, regions, read mapping, save) refuse a sharded graph until
 * mcaat_graph_unshard (collective) gathers it on every rank, valid bits included.
 * Replaces cycle_finder.cpp:346-492 over a graph split by ranges. */
int mcaat_graph_shard_info(const mcaat_graph *g, int *sharded, uint64_t *first, uint64_t *n_local);
int mcaat_graph_unshard(mcaat_graph *g, mcaat_comm *comm);

/* ---- measurement -------------------------------------------------------------
 * Per-stage device time of the last build/cycle_finder call on this ctx, measured
 * with HIP events on the library's stream. names[i] are static strings. */
int mcaat_stage_times(const mcaat_ctx *ctx, int max, const char **names, double *ms, int *n);
/* average duration (ms) and launch count of the dominant counting kernel since the
 * last reset, measured with HIP events around each launch on the library's stream */
int mcaat_kernel_timing(const mcaat_ctx *ctx, const char *kernel, double *avg_ms, uint64_t *launches,
                        double *bytes_per_launch);
void mcaat_reset_timing(mcaat_ctx *ctx);

/* ---- tuning / test knobs ----------------------------------------------------------
 * Replaces: nothing in the reference. Size limits that decide which code path a stage takes
 * (results never depend on them), so small parity inputs can reach the branches that
 * otherwise only run at C2/C3 scale. value < 0 restores the default. Known names:
 *   nc.group_budget    descriptors per pass-B/C group of L1 buckets (multi-group counting)
 *   nc.fallback_budget occurrences per global-table fallback batch
 *   nc.out_cap         initial capacity of the count output (regrowth + recount)
 *   nc.l1_slots        first-attempt capacity of each L1 bucket (pass A resize + re-run)
 *   nc.fine_bits       log2 fine partitions (8..19)
 *   nc.edge_cap        distinct edges per LDS partition before the class split / fallback
 *   nc.desc_cap        distinct super-k-mers per LDS partition before the class split / raw path
 *   nc.big_table       1: pass C always with the 8192-slot edge table (one workgroup per CU),
 *                      0: never; default: from the group after one that split more than 1 in 8
 *                      of its partitions into classes
 *   nc.overlap         0: passes B and C of successive groups in turn on one stream (default
 *                      1: the next group's pass B on a second stream while C counts this one)
 *   nc.free_sync       1: synchronise the stream before the count output's early regrowth frees
 *                      its old buffers (round 4's guard; default 0: the arena's stream order)
 *   nc.ahead           0: ignore mcaat_count_ahead (pass A after the read, default 1)
 *   sort.msd          0: radix sort only, 1: MSD sort whenever k <= 28 (default: D >= 2^16)
 *   sort.wave_limit / sort.mid_limit / sort.block_limit   level-3 bucket size limits of the
 *                      one-wave, 256-thread and 1024-thread LDS sorts (above the last: radix)
 *   sort.l3_counting   0: one-wave level-3 buckets by the bitonic network only (default 1: LDS
 *                      counting sort by the next key bits, bitonic for clustered buckets)
 *   sort.mid_counting  0: level-3 buckets above the one-wave limit by the 256-thread bitonic
 *                      network (default 1: the 256-thread LDS counting sort)
 *   sort.mid_occ       5: that counting sort at five workgroups per CU (default 4)
 *   sort.small_mid     1: a 128-thread counting-sort stage for level-3 buckets of up to 1024
 *                      items before the 256-thread one, 0: none (default: when D / 2^22 <= 768)
 *   sort.small_limit   largest bucket that stage sorts (default and maximum 1024; larger ones
 *                      are forwarded)
 *   cf.scan_u          64-edge words in flight per wave in the tips/filter and recount scans
 *                      (1, 2 default, 4)
 *   cf.prep_batch      edges per thread in flight in the peel's prep pass (2 default, 4, 8, 16)
 *   cf.dls_lanes       DepthLevelSearch searches per wave (1..64, default 16)
 *   cf.dls_stack / cf.dls_visited   initial DepthLevelSearch scratch (grows x8 on overflow)
 *   cf.fc_lock / cf.fc_relax / cf.fc_out   initial FindCycle scratch (grows on overflow)
 *   cf.fc_window       initial FindCycle speculation window
 *   cf.walk_budget     > 0: counter-driven peel walks of this many steps before the
 *                      list-ranking peel (default 0: the list-ranking peel alone)
 *   cf.ruler_mask      1 in (mask + 1) unary nodes is a peel ruler besides the chain heads
 *   cf.fused_init      0: the peel's first pass as its own kernel (default 1: done by the tips /
 *                      multiplicity-filter pass)
 *   cf.recount         1: the valid / tips recount and ChunkStartNodes' candidate filter as
 *                      their own pass after the peel (default 0: the tips / filter pass lists the
 *                      post-filter candidates and counts the post-filter tips that are not
 *                      seeds; after the peel the candidates still valid are kept and the valid
 *                      bits are popcounted)
 *   cf.dls_host        1: DepthLevelSearch candidates and results through the host (default 0:
 *                      on one GPU they stay on the device and only the passing ids come back)
 *   cf.compact         1: the peel's per-edge arrays over compact slots of the filter-valid edges,
 *                      0: one slot per edge id; unset (round 6): compact when the multiplicity
 *                      filter keeps under cf.compact_pct % (default 30) of a fresh graph's edges
 *                      (C5 keeps 18 %: its peel state 63 -> 12 GB at the same peel time)
 *   cf.peel_list_div   first ruler-list capacity D / div (default 16; the prep pass runs again
 *                      with the counted size when it overflows)
 *   cf.peel_list_cap / cf.cand_cap   first capacity of the ruler and branch lists / of the
 *                      start-candidate list (regrowth test knobs)
 *   fq.hostpack        0: FASTQ always through the GPU text parser (default 1: plain files of
 *                      upper-case ACGT 4-line records packed to 2 bits by host threads first)
 *   sdbg.adj_lds       0: adjacency by per-edge directory searches in global memory;
 *                      1 (default): group-aligned runs that own disjoint in_info slot ranges,
 *                      staged in LDS and written once; 2: per-run target key ranges in LDS with
 *                      in_info stored from the predecessor side (round 2)
 *   sdbg.adj_cap       mode 1: most owned slots a run stages in LDS (default and maximum 3072;
 *                      a larger run clears its slots and writes them directly); mode 2: largest
 *                      target key range staged (maximum 1024) */
int mcaat_set_knob(mcaat_ctx *ctx, const char *name, int64_t value);

/*   dist.shard_cf     0: the sharded build all-gathers the whole graph on every rank and
 *                      CycleFinder runs over the ranks on replicas (round 4; default 1: per shard)
 *   dist.ruler_mask   per-shard peel: 1 in (mask + 1) unary edges is a ruler besides the chain
 *                      heads (default 15 up to two ranks, 3 above: fewer walk rounds)
 *   dist.adj_ranges   0: sharded adjacency by per-edge request / response (default 1: the four
 *                      target key ranges pulled, in_info pushed back)
 *   dist.win_ranges   0: the filter windows and predecessor flags as per-edge messages (default 1:
 *                      target-range bytes pulled and pushed)
 *   dist.adj_chunk    sharded adjacency: edges per request/response exchange (default 2^26)
 *   dist.dir_edges    sharded adjacency: edges per prefix of the range's radix directory (default 2)
 *   nc.a_mini         pass A's slots per (workgroup, L1 bucket) reservation (default 1024 on one GPU,
 *                      256 for a rank of a sharded build; rounded down to a multiple of 8)
 *   dist.bfs_sync     1: the region BFS (candidates' forward region, FindCycle's backward region)
 *                      runs one routed exchange with host waits per hop, and the FindCycle reach on
 *                      the search replica reads its frontier size after every hop (round 5's forms;
 *                      default 0: the hops run back to back on the device, fixed-capacity blocks
 *                      exchanged by an all-to-all that RCCL leaves queued on the stream)
 *   dist.bfs_block    region BFS: requests per block to another rank (default 2^16; an overflow on
 *                      any rank reruns the BFS with larger blocks, kept for the next step)
 *   dist.bfs_frontier region BFS: first frontier / own-block capacity (tests; default D_local/16,
 *                      at least 2^20; an overflow reruns with more)
 *   dist.res_fixed    0: the peel's branch resolution by routed rounds (round 5's form; default 1:
 *                      fixed blocks, rounds back to back on the device, one check per batch)
 *   dist.res_batch    branch resolution rounds per batch between checks (default 8)
 *   dist.walk_block   the peel walk's tail: once every rank's records in flight fit this many, its
 *                      rounds run in fixed blocks back to back on the device (default 2^15; 0: every
 *                      round routed, round 5's form)
 *   dist.walk_batch   walk tail rounds per batch between checks (default 8)
 *   dist.res_block_mb largest block set (MB) for fixed-block resolution; larger graphs keep the
 *                      routed rounds (default 64)
 *   dist.segs_at_one  1: one rank runs the descriptor exchange through the segment all-to-all too
 *                      (its self-copy path; default 0 keeps the buckets in place) */

/* ---- allocator check ----------------------------------------------------------------------
 * Replaces: nothing in the reference. The device arena's stream order (csrc/alloc.hip): a block
 * is freed while a kernel queued on the context's main stream still writes it, then taken for
 * a kernel on the side stream. out[0] = 1 when the side allocation got the same block, out[1] =
 * 1 when every word holds the side kernel's value afterwards (the side kernel waited for the
 * fence), out[2] = the arena's fence waits during the check. Then the same with a consumer the
 * arena does not watch (a stream created for the check, the block taken with no allocation
 * stream, as the FASTQ packer's upload streams take theirs): out[3] = the same block, out[4] = 1
 * when every word holds that stream's value. out must hold 5 entries. */
int mcaat_arena_check(mcaat_ctx *ctx, int64_t *out);
/* Device memory of the library on the ctx's GPU (the arena behind every buffer): bytes in use
 * now, the most in use since the last reset (reset_peak != 0 starts a new window after
 * reading), and the chunks the arena holds. Null outputs are skipped. */
int mcaat_arena_usage(mcaat_ctx *ctx, int reset_peak, uint64_t *in_use, uint64_t *peak, uint64_t *reserved);

#ifdef __cplusplus
}
#endif
#endif
