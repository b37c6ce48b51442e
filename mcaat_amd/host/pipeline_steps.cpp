// pipeline_steps.cpp — the reference's steps 6-8 drivers (src/main_run_and_debug.cpp):
// relevant reads, spacer ordering per CRISPR region, and the result / benchmark reports.
#include <atomic>
#include <chrono>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <thread>

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

// main_run_and_debug.cpp:32-143. The regions are disjoint SCCs, so their subproblems (cover
// filter, constraints, topological order) are independent: they are solved on `threads` host
// threads (a shared counter deals regions out), each region's lines captured, and everything
// is then printed and get_systems run in region order, so stdout, `found` and therefore
// all_systems' insertion order (CRISPR_Arrays.txt) are those of the reference's serial loop.
std::vector<FoundSystem> run_and_debug_spacer_ordering(const std::vector<std::vector<uint64_t>> &reads, SDBG &sdbg,
                                                       const std::vector<std::vector<uint64_t>> &cycles,
                                                       unsigned threads) {
    const auto t0 = std::chrono::high_resolution_clock::now();
    std::cout << "  ▸ Splitting into subproblems" << std::endl;
    const size_t read_nodes = reads.at(0).size();  // the region growth radius (reference: reads.at(0).size())
    auto regions = get_crispr_regions_extended_by_k(sdbg, read_nodes, cycles);
    const auto t_regions = std::chrono::high_resolution_clock::now();

    std::cout << "  🔄 Filtering subproblems:" << std::endl;
    std::vector<ReadRefs> region_reads;
    std::vector<std::vector<std::vector<uint64_t>>> region_cycles;
    get_relevant_reads_and_cycles(regions, reads, cycles, region_reads, region_cycles);
    struct Sub {
        bool kept = false;
        size_t n_reads = 0;
        std::vector<std::vector<uint64_t>> cycles;  // after the cover filter
        std::vector<uint32_t> order;
        float conf_resolution = 1.0, conf_sort = 1.0;
        std::string log;  // order_cycles' lines
        std::string cover_log;  // the set cover's diagnostics (printed in region order)
    };
    std::vector<Sub> subs(regions.size());
    const auto t_split = std::chrono::high_resolution_clock::now();
    std::atomic<int64_t> ns_cover{0}, ns_order{0};  // CPU time of the two parts, summed over threads
    auto solve = [&](size_t ri) {
        using hc = std::chrono::high_resolution_clock;
        Sub &s = subs[ri];
        auto rr = std::move(region_reads[ri]);
        s.cycles = std::move(region_cycles[ri]);
        const auto a = hc::now();
        {
            std::ostringstream clog;
            get_minimum_cycles_for_full_coverage(s.cycles, clog);
            s.cover_log = clog.str();
        }
        const auto b = hc::now();
        ns_cover += std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
        // the reverse-complement twin of a region is expected to carry no relevant reads
        if (rr.empty() || s.cycles.size() < 3) return;
        s.kept = true;
        s.n_reads = rr.size();
        std::ostringstream log;
        s.order = order_cycles(regions[ri], rr, s.cycles, s.conf_resolution, s.conf_sort, log);
        s.log = log.str();
        ns_order += std::chrono::duration_cast<std::chrono::nanoseconds>(hc::now() - b).count();
    };
    if (threads == 0) threads = 1;
    threads = (unsigned)std::min<size_t>(threads, std::max<size_t>(1, regions.size()));
    {
        std::atomic<size_t> next{0};
        std::vector<std::string> err(threads);
        auto worker = [&](unsigned t) {
            try {
                for (size_t ri; (ri = next.fetch_add(1)) < regions.size();) solve(ri);
            } catch (const std::exception &e) {
                err[t] = e.what();
                next.store(regions.size());
            }
        };
        std::vector<std::thread> pool;
        for (unsigned t = 1; t < threads; ++t) pool.emplace_back(worker, t);
        worker(0);
        for (auto &th : pool) th.join();
        for (const auto &e : err)
            if (!e.empty()) throw std::runtime_error(e);
    }
    size_t n_kept = 0;
    for (const Sub &s : subs) {
        n_kept += s.kept;
        std::cout << s.cover_log;  // region order, whatever thread solved it
    }
    std::cout << "  ✅ Filtered out " << regions.size() - n_kept << "/" << regions.size() << " subproblems" << std::endl;
    const auto t_solved = std::chrono::high_resolution_clock::now();
    std::cout << "  🔄 Solving " << n_kept << " subproblems..." << std::endl;

    std::vector<FoundSystem> found;
    size_t i = 0;
    for (size_t ri = 0; ri < regions.size(); ++ri) {
        Sub &s = subs[ri];
        if (!s.kept) continue;
        ++i;
        std::cout << "    Subproblem " << i << "/" << n_kept << ":" << std::endl;
        std::cout << "      🛈 Graph with " << regions[ri].nodes.size() << " nodes and " << regions[ri].edge_count()
                  << " edges" << std::endl;
        std::cout << "      🛈 Reads with " << s.n_reads << "/" << reads.size() << " used" << std::endl;
        std::cout << "      🛈 Cycles with " << s.cycles.size() << "/" << get_cycle_count(cycles) << " used" << std::endl;
        std::cout << s.log;
        std::cout << "      ▸ The order is ";
        for (uint32_t c : s.order) std::cout << c << " ";
        std::cout << std::endl;
        std::cout << "      ▸ Cycles were resolved with a confidence of " << std::fixed << std::setprecision(2)
                  << (s.conf_resolution * 100) << "%" << std::endl;
        std::cout << "      ▸ Topological sort has a confidence of " << (s.conf_sort * 100) << "%" << std::endl;
        std::cout << "      ▸ Turning the cycle order into a node order" << std::endl;
        auto ordered = get_ordered_cycles(s.order, s.cycles);
        if (ordered.size() < 2) {
            std::cout << "      ▸ Node order is to short and is not processed further" << std::endl;
            continue;
        }
        std::cout << "      ▸ Starting the filter process:" << std::endl;
        auto [repeat, spacers, sequence] = get_systems(sdbg, ordered);
        std::cout << "        ▸ Number of spacers: " << spacers.size() << std::endl;
        found.emplace_back(sequence, repeat, spacers, s.conf_resolution, s.conf_sort);
    }
    std::cout << "  ✅ Completed each subproblem" << std::endl;
    {
        using sec = std::chrono::duration<double>;
        const auto t_end = std::chrono::high_resolution_clock::now();
        std::cout << "TIMING_STEP7 regions_s=" << sec(t_regions - t0).count()
                  << " split_s=" << sec(t_split - t_regions).count() << " solve_s=" << sec(t_solved - t_split).count()
                  << " emit_s=" << sec(t_end - t_solved).count() << " threads=" << threads
                  << " cover_cpu_s=" << ns_cover.load() * 1e-9 << " order_cpu_s=" << ns_order.load() * 1e-9 << std::endl;
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
