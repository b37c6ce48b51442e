// main.cpp — the mcaat CLI over the MI355X hot path. Mirrors the release main of the
// reference (src/main.cpp:496-591): settings check, SDBG build, CycleFinder, relevant reads
// (step 6), spacer ordering (step 7), results / benchmark (step 8) and CRISPRAnalyzer, which
// writes settings.output_file (CRISPR_Arrays.txt). The cycles themselves are also written to
// <cycles_folder>/cycles.txt (not in the reference's release build).
#include <chrono>
#include <cstdio>
#include <filesystem>
#include <fstream>
#include <iostream>

#include "downstream.h"

namespace fs = std::filesystem;

static bool check_for_error(Settings &settings) {  // main.cpp:50-59
    std::cout << "Step 1. Checking the inputs: " << std::endl;
    std::string bad = settings.print_settings();
    if (bad.empty()) {
        std::cout << "All inputs are correct. [✔]" << std::endl;
        return false;
    }
    std::cout << "Please check the following: " << bad << std::endl;
    return true;
}

static std::string cycle_sequence(const SDBG &sdbg, const std::vector<uint64_t> &cycle) {
    std::vector<uint8_t> lab(sdbg.k());
    std::string s;
    for (size_t i = 0; i < cycle.size(); ++i) {
        sdbg.GetLabel(cycle[i], lab.data());
        if (i == 0) for (int j = 0; j < sdbg.k(); ++j) s += "ACGT"[lab[j] - 1];
        else s += "ACGT"[lab[sdbg.k() - 1] - 1];
    }
    return s;
}

static void banner(const char *title) {
    std::cout << "\n══════════════════════════════════════════════" << std::endl;
    std::cout << title << std::endl;
    std::cout << "══════════════════════════════════════════════" << std::endl;
}

int main(int argc, char **argv) {
    try {
        Settings settings = parse_arguments(argc, argv);
        if (check_for_error(settings)) {  // main.cpp:499-513
            std::cout << "Folder " << settings.output_folder << " will be deleted due to errors." << std::endl;
            std::cout << "Do you want that folder to be removed? (y/n): ";
            char answer = 'n';
            std::cin >> answer;
            if (answer != 'y' && answer != 'Y') {
                std::cout << "Exiting the program." << std::endl;
                return 1;
            }
            std::cout << "Removing folder: " << settings.output_folder << std::endl;
            fs::remove_all(settings.output_folder);
            return 1;
        }
        {
            // brings the HIP runtime up before the timed span (errors surface in SDBGBuild, after
            // it has written data.lib as the reference does)
            int n_dev = 0;
            (void)mcaat_device_count(&n_dev);
        }
        using clk = std::chrono::steady_clock;
        const auto t_start = clk::now();
        SDBGBuild sdbg_build(settings);                        // main.cpp:517
        const auto t_built = clk::now();
        SDBG sdbg;                                             // main.cpp:522-530
        sdbg.LoadFromDevice(sdbg_build.release_graph());
        std::cout << "Loaded the graph" << std::endl;
        settings.sdbg = &sdbg;
        std::cout << "FBCE START:" << std::endl;
        CycleFinder cycle_finder(settings);                    // main.cpp:536
        {
            // the reference's hot-path span, SDBGBuild start -> CycleFinder end (main.cpp:517-536)
            const auto t_end = clk::now();
            auto sec = [](clk::duration d) { return std::chrono::duration<double>(d).count(); };
            char line[256];
            snprintf(line, sizeof line,
                     "TIMING span_s=%.6f sdbg_build_s=%.6f build_lib_s=%.6f cycle_finder_s=%.6f",
                     sec(t_end - t_start), sec(t_built - t_start), sdbg_build.lib_seconds, sec(t_end - t_built));
            std::cout << line << std::endl;
        }
        auto cycles_map = cycle_finder.results;
        std::cout << "Number of nodes in results: " << cycles_map.size() << std::endl;
        auto cycles = cycles_map_to_cycles(cycles_map);        // main.cpp:542
        {
            const std::string out = settings.cycles_folder + "/cycles.txt";
            std::ofstream f(out);
            size_t idx = 0;
            for (const auto &[start, inner] : cycles_map)
                for (const auto &c : inner) {
                    f << ">cycle_" << idx++ << " start=" << start << " length=" << c.size() << "\n";
                    f << cycle_sequence(sdbg, c) << "\n";
                }
        }

        banner("🔸STEP 6: Finding relevant reads");             // main.cpp:544-551
        const auto reads = run_and_debug_finding_of_relevant_reads(cycles, sdbg_build.reads(), sdbg);

        banner("🔸STEP 7: Order the spacers");                  // main.cpp:553-556
        const auto found_systems = run_and_debug_spacer_ordering(reads, sdbg, cycles);

        if (settings.benchmark_file != "") {                   // main.cpp:559-569
            banner("🔸STEP 8: Compare to ground of truth using benchmark file");
            run_and_debug_benchmark_results(settings, found_systems);
        } else {
            banner("🔸STEP 8: Results");
            run_and_debug_results(found_systems);
        }
        std::cout << "══════════════════════════════════════════════" << std::endl;

        std::cout << "POST PROCESSING START:" << std::endl;    // main.cpp:573-581
        std::unordered_map<std::string, std::vector<std::string>> all_systems;
        for (const auto &[_sequence, repeat, spacers, _conf_a, _conf_b] : found_systems) all_systems[repeat] = spacers;
        CRISPRAnalyzer analyzer(all_systems, settings.output_file);
        analyzer.run_analysis();
        std::cout << "Saved in: " << settings.output_file << std::endl;

        try {                                                  // main.cpp:525,584-589: "<graph>/graph"
            fs::remove_all(settings.graph_folder + "/graph");
        } catch (const std::filesystem::filesystem_error &e) {
            std::cerr << "Warning: Could not remove graph folder: " << e.what() << std::endl;
        }
        return 0;
    } catch (const std::exception &e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
}
