// downstream.h — the reference's steps after CycleFinder, restated on the host SDBG mirror
// (SURVEY.md §8f rank 1): relevant reads (reads.h), spacer ordering (spacer_ordering.h),
// array extraction (tmp_utils.h get_systems), benchmark comparison (evaluation.h), the
// run_and_debug_* drivers (main_run_and_debug.h) and CRISPRAnalyzer (post_processing.h),
// which writes CRISPR_Arrays.txt. Same names, signatures (SDBG by reference), container types
// and iteration orders as the reference, so the libstdc++ orders that decide ties are the
// reference's. Differences, each documented where it sits:
//   * get_reads maps the reads on the GPU (mcaat_map_reads) from the reads already in HBM
//     instead of re-parsing the FASTQ files (same result, tests/test_read_mapping.py);
//   * solve_min_cover_problem is an exact set-cover solver (cft is an absent, unpinned
//     third-party heuristic with a 10 s time limit; spacer_ordering.cpp:265-313);
//   * rapidfuzz fuzz::ratio / partial_ratio are restated from rapidfuzz-cpp (absent).
#pragma once
#include <cstdint>
#include <iostream>
#include <limits>
#include <optional>
#include <string>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "mcaat_host.h"

// ---------------------------------------------------------------- reads.h
void reverse_pair_ends_sequence(std::string &sequence);                              // reads.cpp:20-31
uint64_t k_mer_to_node_id(const SDBG &sdbg, const std::string k_mer);                 // reads.cpp:33-55
std::vector<uint64_t> get_read_from_sequence(const SDBG &sdbg,                        // reads.cpp:57-86
                                             const std::unordered_set<uint64_t> &nodes_of_cycles,
                                             const std::string &sequence);
// reads.cpp:88-130 over the reads resident in HBM (mapping view of the input files)
std::vector<std::vector<uint64_t>> get_reads(const SDBG &sdbg, const mcaat_reads *reads,
                                             const std::vector<std::vector<uint64_t>> cycles);
// over the ranks of a multi-GPU run: each maps its own part; every rank gets all relevant
// reads in input order (n_files: number of input files)
std::vector<std::vector<uint64_t>> get_reads(const SDBG &sdbg, const mcaat_reads *reads,
                                             const std::vector<std::vector<uint64_t>> cycles, mcaat_comm *comm,
                                             int n_files);

// ---------------------------------------------------------------- spacer_ordering.h
struct Graph {  // spacer_ordering.h:20-46
    std::unordered_map<uint64_t, std::vector<uint64_t>> adjacency_list;
    std::unordered_set<uint64_t> nodes;
    void add_edge(const uint64_t from, const uint64_t to) {
        adjacency_list[from].push_back(to);
        nodes.insert(from);
        nodes.insert(to);
    }
    size_t edge_count() const {
        size_t count = 0;
        for (const auto &kv : adjacency_list) count += kv.second.size();
        return count;
    }
};

const uint32_t NOT_IN_ANY_CYCLE_INDEX = std::numeric_limits<uint32_t>::max();

struct TupleHash {  // spacer_ordering.h:50-54
    size_t operator()(const std::tuple<uint32_t, uint32_t> &t) const {
        return std::hash<uint32_t>()(std::get<0>(t)) ^ (std::hash<uint32_t>()(std::get<1>(t)) << 1);
    }
};

std::vector<std::vector<uint64_t>> find_strongly_connected_components(const SDBG &sdbg);
void keep_crispr_regions_extended_by_k(SDBG &sdbg, const size_t &k, const std::vector<std::vector<uint64_t>> &cycles);
std::vector<Graph> divide_graph_into_subgraphs(const SDBG &sdbg);
std::vector<Graph> get_crispr_regions_extended_by_k(SDBG &sdbg, const size_t &k,
                                                    const std::vector<std::vector<uint64_t>> &cycles);
std::vector<std::vector<uint64_t>> get_relevant_reads(const Graph &graph,
                                                      const std::vector<std::vector<uint64_t>> &all_reads);
std::vector<std::vector<uint64_t>> get_relevant_cycles(const Graph &graph,
                                                       const std::vector<std::vector<uint64_t>> &all_cycles);
// a region's relevant reads as pointers into the relevant-read list (C3: 367K reads of 124 ids;
// copying them per region was 365 MB of copies in step 7)
using ReadRefs = std::vector<const std::vector<uint64_t> *>;
void get_relevant_reads_and_cycles(const std::vector<Graph> &regions, const std::vector<std::vector<uint64_t>> &all_reads,
                                   const std::vector<std::vector<uint64_t>> &all_cycles, std::vector<ReadRefs> &reads_out,
                                   std::vector<std::vector<std::vector<uint64_t>>> &cycles_out);
// (round 5) `log`: where the cover's diagnostics go (std::cout by default; step 7's worker
// threads pass a per-region stream that is printed in region order)
void get_minimum_cycles_for_full_coverage(std::vector<std::vector<uint64_t>> &cycles, std::ostream &log = std::cout);
std::vector<size_t> solve_min_cover_problem(const std::unordered_set<uint32_t> &universe,
                                            const std::vector<std::vector<uint32_t>> &sets, std::ostream &log = std::cout);
std::unordered_map<uint64_t, uint32_t> get_node_to_unique_cycle_map(const std::vector<std::vector<uint64_t>> &cycles);
std::vector<uint32_t> get_all_cycle_indices(const std::unordered_map<uint64_t, uint32_t> &node_to_cycle_map);
std::vector<std::tuple<uint32_t, uint32_t>> every_possible_combination(const std::vector<uint32_t> &v);
std::vector<std::tuple<uint32_t, uint32_t>> generate_constraints_from_read(
    const Graph &graph, const std::vector<uint64_t> &read, const std::unordered_map<uint64_t, uint32_t> &node_to_cycle_map);
std::vector<std::tuple<uint32_t, uint32_t>> generate_out_of_cycles_constraints_from_read(
    const Graph &graph, const std::vector<uint64_t> &read, const std::unordered_map<uint64_t, uint32_t> &node_to_cycle_map);
std::vector<std::tuple<uint32_t, uint32_t>> generate_constraints(
    const Graph &graph, const std::vector<std::vector<uint64_t>> &reads,
    const std::unordered_map<uint64_t, uint32_t> &node_to_cycle_map);
std::vector<std::tuple<uint32_t, uint32_t>> get_maximal_spanning_tree(
    const std::vector<std::tuple<uint32_t, uint32_t>> &edges);
void resolve_cycles_greedy(std::vector<std::tuple<uint32_t, uint32_t>> &constraints,
                           std::unordered_map<uint32_t, int> &heuristic_node_values);
std::vector<uint32_t> solve_constraints_with_topological_sort(
    const std::vector<std::tuple<uint32_t, uint32_t>> &constraints, std::unordered_map<uint32_t, int> &heuristic_node_values,
    const std::vector<uint32_t> &nodes, float &confidence);
// log: where the per-subproblem constraint lines go (the step-7 driver solves subproblems on
// several threads and prints each one's lines in subproblem order)
std::vector<uint32_t> order_cycles(const Graph &graph, const std::vector<std::vector<uint64_t>> &reads,
                                   const std::vector<std::vector<uint64_t>> &cycles, float &confidence_cycle_resolution,
                                   float &confidence_topological_sort, std::ostream &log = std::cout);
std::vector<uint32_t> order_cycles(const Graph &graph, const ReadRefs &reads, const std::vector<std::vector<uint64_t>> &cycles,
                                   float &confidence_cycle_resolution, float &confidence_topological_sort,
                                   std::ostream &log = std::cout);
std::vector<std::vector<uint64_t>> get_ordered_cycles(const std::vector<uint32_t> &cycle_order,
                                                      const std::vector<std::vector<uint64_t>> &cycles);

// ---------------------------------------------------------------- tmp_utils.h
void trim_string(std::string &s);
std::pair<std::string, std::optional<std::string>> get_fastq_files_from_settings(const Settings &settings);
int get_cycle_count(const std::vector<std::vector<uint64_t>> &cycles);
std::string fetch_node_label(SDBG &sdbg, const size_t &node);
std::tuple<std::string, std::vector<std::string>, std::string> get_systems(
    SDBG &sdbg, std::vector<std::vector<uint64_t>> &ordered_cycles);

// ---------------------------------------------------------------- evaluation.h
uint16_t get_levenshtein_distance(const std::string &s1, const std::string &s2);
float get_string_similarity(const std::string &s1, const std::string &s2);
int get_number_of_duplicate_spacers(const std::vector<std::string> &spacers, const std::string &expected_sequence);
std::string get_most_similar_sequence(const std::string &sequence, const std::vector<std::string> &choices);

// ---------------------------------------------------------------- rapidfuzz (fuzz.cpp)
namespace fuzz {
double ratio(const std::string &s1, const std::string &s2);
double partial_ratio(const std::string &s1, const std::string &s2);
}  // namespace fuzz

// ---------------------------------------------------------------- main_run_and_debug.h
using FoundSystem = std::tuple<std::string, std::string, std::vector<std::string>, float, float>;
std::vector<std::vector<uint64_t>> run_and_debug_finding_of_relevant_reads(
    const std::vector<std::vector<uint64_t>> &cycles, const mcaat_reads *reads, const SDBG &sdbg,
    mcaat_comm *comm = nullptr, int n_files = 1);
// threads: host threads for the independent subproblems (output order is the serial loop's)
std::vector<FoundSystem> run_and_debug_spacer_ordering(const std::vector<std::vector<uint64_t>> &reads, SDBG &sdbg,
                                                       const std::vector<std::vector<uint64_t>> &cycles,
                                                       unsigned threads = 1);
void run_and_debug_benchmark_results(const Settings &settings, const std::vector<FoundSystem> &found_systems);
void run_and_debug_results(const std::vector<FoundSystem> &found_systems);

// ---------------------------------------------------------------- post_processing.h
class CRISPRAnalyzer {
   public:
    CRISPRAnalyzer(std::unordered_map<std::string, std::vector<std::string>> systems_map,
                   std::string output = "crispr_report.txt", int amt = 2, int minsl = 23, int maxsl = 50,
                   int minrl = 23, int maxrl = 50, int mean_sim = 90);
    std::map<std::string, std::vector<std::string>> getSystems() const { return grouped_repeat_cycles; }
    void run_analysis();

   private:
    std::vector<std::string> get_common_kmers(const std::vector<std::string> &kmers,
                                              const std::vector<std::string> &sequences);
    std::vector<std::string> find_common_prefix_kmers(const std::vector<std::string> &sequences, int k);
    std::vector<std::string> find_common_suffix_kmers(const std::vector<std::string> &sequences, int k);
    std::vector<std::string> trim_kmers_from_sequences(const std::vector<std::string> &sequences,
                                                       const std::vector<std::string> &prefixes,
                                                       const std::vector<std::string> &suffixes);
    bool validate_spacer_diversity(const std::vector<std::string> &sequences);
    std::vector<std::string> filter_substring_spacers(const std::vector<std::string> &spacers);
    std::vector<std::string> filter_by_length(const std::vector<std::string> &spacers);
    std::string reconstruct_repeat(const std::string &original, const std::vector<std::string> &prefixes,
                                   const std::vector<std::string> &suffixes);
    void generate_report(const std::string &repeat, const std::vector<std::string> &spacers, std::ofstream &out);

    std::unordered_map<std::string, std::vector<std::string>> systems;
    std::string output_path;
    int omitted_repeats = 0;
    int total_spacers = 0;
    int amount, min_sl, max_sl, min_rl, max_rl, mean_similarity;
    std::map<std::string, std::vector<std::string>> grouped_repeat_cycles;
};
