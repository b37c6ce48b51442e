// pipeline_steps.cpp — the reference's steps 6-8 drivers (src/main_run_and_debug.cpp):
// relevant reads, spacer ordering per CRISPR region, and the result / benchmark reports.
#include <chrono>
#include <fstream>
#include <iomanip>
#include <iostream>

#include "downstream.h"

namespace {

void print_elapsed(std::chrono::high_resolution_clock::time_point t0) {
    const double s = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count();
    std::cout << "\n⏳ Time elapsed: " << std::fixed << std::setprecision(2) << s << " seconds" << std::endl;
}

}  // namespace

// main_run_and_debug.cpp:3-30 (the reads come from HBM instead of the FASTQ files)
std::vector<std::vector<uint64_t>> run_and_debug_finding_of_relevant_reads(
    const std::vector<std::vector<uint64_t>> &cycles, const mcaat_reads *reads, const SDBG &sdbg, mcaat_comm *comm,
    int n_files) {
    const auto t0 = std::chrono::high_resolution_clock::now();
    auto relevant = get_reads(sdbg, reads, cycles, comm, n_files);
    std::cout << "    ▸ Found " << relevant.size() << " reads" << std::endl;
    if (relevant.empty()) {
        std::cout << "══════════════════════════════════════════════" << std::endl;
        return relevant;
    }
    print_elapsed(t0);
    return relevant;
}

// main_run_and_debug.cpp:32-143
std::vector<FoundSystem> run_and_debug_spacer_ordering(const std::vector<std::vector<uint64_t>> &reads, SDBG &sdbg,
                                                       const std::vector<std::vector<uint64_t>> &cycles) {
    const auto t0 = std::chrono::high_resolution_clock::now();
    std::cout << "  ▸ Splitting into subproblems" << std::endl;
    const size_t read_nodes = reads.at(0).size();  // the region growth radius (reference: reads.at(0).size())
    auto regions = get_crispr_regions_extended_by_k(sdbg, read_nodes, cycles);
    const auto t_regions = std::chrono::high_resolution_clock::now();

    std::cout << "  🔄 Filtering subproblems:" << std::endl;
    struct Sub {
        const Graph *g;
        std::vector<std::vector<uint64_t>> reads, cycles;
    };
    std::vector<Sub> subs;
    std::vector<std::vector<std::vector<uint64_t>>> region_reads, region_cycles;
    get_relevant_reads_and_cycles(regions, reads, cycles, region_reads, region_cycles);
    for (size_t ri = 0; ri < regions.size(); ++ri) {
        const Graph &g = regions[ri];
        auto rr = std::move(region_reads[ri]);
        auto rc = std::move(region_cycles[ri]);
        get_minimum_cycles_for_full_coverage(rc);
        // the reverse-complement twin of a region is expected to carry no relevant reads
        if (rr.empty() || rc.size() < 3) continue;
        subs.push_back({&g, std::move(rr), std::move(rc)});
    }
    std::cout << "  ✅ Filtered out " << regions.size() - subs.size() << "/" << regions.size() << " subproblems"
              << std::endl;
    const auto t_filtered = std::chrono::high_resolution_clock::now();
    std::cout << "  🔄 Solving " << subs.size() << " subproblems..." << std::endl;

    std::vector<FoundSystem> found;
    for (size_t i = 0; i < subs.size(); ++i) {
        const Sub &s = subs[i];
        std::cout << "    Subproblem " << i + 1 << "/" << subs.size() << ":" << std::endl;
        std::cout << "      🛈 Graph with " << s.g->nodes.size() << " nodes and " << s.g->edge_count() << " edges"
                  << std::endl;
        std::cout << "      🛈 Reads with " << s.reads.size() << "/" << reads.size() << " used" << std::endl;
        std::cout << "      🛈 Cycles with " << s.cycles.size() << "/" << get_cycle_count(cycles) << " used" << std::endl;
        float conf_resolution = 1.0, conf_sort = 1.0;
        const auto order = order_cycles(*s.g, s.reads, s.cycles, conf_resolution, conf_sort);
        std::cout << "      ▸ The order is ";
        for (uint32_t c : order) std::cout << c << " ";
        std::cout << std::endl;
        std::cout << "      ▸ Cycles were resolved with a confidence of " << std::fixed << std::setprecision(2)
                  << (conf_resolution * 100) << "%" << std::endl;
        std::cout << "      ▸ Topological sort has a confidence of " << (conf_sort * 100) << "%" << std::endl;
        std::cout << "      ▸ Turning the cycle order into a node order" << std::endl;
        auto ordered = get_ordered_cycles(order, s.cycles);
        if (ordered.size() < 2) {
            std::cout << "      ▸ Node order is to short and is not processed further" << std::endl;
            continue;
        }
        std::cout << "      ▸ Starting the filter process:" << std::endl;
        auto [repeat, spacers, sequence] = get_systems(sdbg, ordered);
        std::cout << "        ▸ Number of spacers: " << spacers.size() << std::endl;
        found.emplace_back(sequence, repeat, spacers, conf_resolution, conf_sort);
    }
    std::cout << "  ✅ Completed each subproblem" << std::endl;
    {
        using sec = std::chrono::duration<double>;
        const auto t_end = std::chrono::high_resolution_clock::now();
        std::cout << "TIMING_STEP7 regions_s=" << sec(t_regions - t0).count()
                  << " filter_s=" << sec(t_filtered - t_regions).count() << " solve_s=" << sec(t_end - t_filtered).count()
                  << std::endl;
    }
    print_elapsed(t0);
    return found;
}

// main_run_and_debug.cpp:145-218
void run_and_debug_benchmark_results(const Settings &settings, const std::vector<FoundSystem> &found_systems) {
    const auto t0 = std::chrono::high_resolution_clock::now();
    std::vector<std::string> truth;
    std::ifstream in(settings.benchmark_file);
    if (!in) {
        std::cerr << "Error: Could not open benchmark file: " << settings.benchmark_file << std::endl;
    } else {
        std::string line;
        while (std::getline(in, line))
            if (!line.empty()) truth.push_back(line);
        std::cout << "Loaded " << truth.size() << " benchmark sequences." << std::endl;
    }
    std::cout << "  ▸ " << found_systems.size() << " crispr sequences are found and benchmarked using " << truth.size()
              << " sequences" << std::endl;
    size_t unmatched = 0;
    float mean_similarity = 0.0;
    for (const auto &[sequence, repeat, spacers, conf_resolution, conf_sort] : found_systems) {
        const std::string expected = get_most_similar_sequence(sequence, truth);
        if (expected == "") {
            std::cout << "    ▸ No expected match for sequence: " << sequence << std::endl;
            unmatched++;
            continue;
        }
        const float sim = get_string_similarity(sequence, expected);
        const int dups = get_number_of_duplicate_spacers(spacers, expected);
        std::cout << "    ▸ ≥" << std::fixed << std::setprecision(2) << (sim * 100) << "% sequence similarity, with "
                  << spacers.size() << " spacers, " << dups << " duplicate spacers, confidence of cycle resolution: "
                  << (conf_resolution * 100) << "%, confidence of topological sort: " << (conf_sort * 100)
                  << "%, and the repeat: " << repeat << ", and sequence: " << sequence << std::endl;
        mean_similarity += sim;
    }
    mean_similarity /= static_cast<float>(found_systems.size() - unmatched);
    std::cout << "  ▸ The average sequence similarity is " << std::fixed << std::setprecision(2)
              << (mean_similarity * 100) << "% with " << unmatched << "/" << found_systems.size() << " ignored"
              << std::endl;
    print_elapsed(t0);
}

// main_run_and_debug.cpp:220-258
void run_and_debug_results(const std::vector<FoundSystem> &found_systems) {
    std::cout << "Each result has their own confidence score that can give some guidance of how accurate the "
                 "prediction is."
              << std::endl;
    std::cout << "Take these predictions with a grain of salt:" << std::endl;
    std::cout << "  🔴: Many uncertainties, e.g. no clear repeat sequence, high spacer contradictions" << std::endl;
    std::cout << "  🟠: Some uncertainties, e.g. some spacer positions are unclear and were intuitively guessed"
              << std::endl;
    std::cout << "  🟡: Minor uncertainties" << std::endl;
    std::cout << "  🟢: Highly confident with the result" << std::endl;
    std::cout << std::endl << "----------------------------------------------" << std::endl;
    int red = 0, orange = 0, yellow = 0, green = 0;
    for (const auto &[sequence, repeat, spacers, cr, ct] : found_systems) {
        if (repeat.size() <= 23 || cr < 0.5 || ct < 0.5) {
            std::cout << "  🔴 ";
            ++red;
        } else if (cr < 0.75 || ct < 0.75) {
            std::cout << "  🟠 ";
            ++orange;
        } else if (cr < 0.85 || ct < 0.85) {
            std::cout << "  🟡 ";
            ++yellow;
        } else {
            std::cout << "  🟢 ";
            ++green;
        }
        std::cout << "repeat: " << repeat << ", sequence: " << sequence << std::endl;
    }
    const int total = red + orange + yellow + green;
    std::cout << std::endl
              << "  ▸ " << found_systems.size() << " CRISPR Arrays were found with 🔴 (" << red << "/" << total
              << "), 🟠 (" << orange << "/" << total << "), 🟡 (" << yellow << "/" << total << "), 🟢 (" << green << "/"
              << total << ")" << std::endl;
}
