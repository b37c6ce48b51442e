// main.cpp — the mcaat CLI over the MI355X hot path. Mirrors the release main of the
// reference (src/main.cpp:496-591) up to CycleFinder; steps 6-8 (read remapping, spacer
// ordering, CRISPRAnalyzer -> CRISPR_Arrays.txt) are outside this build's scope
// (DESIGN.md §Scope), so the cycles themselves are written to <cycles_folder>/cycles.txt.
#include <filesystem>
#include <fstream>
#include <iostream>

#include "mcaat_host.h"

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
        SDBGBuild sdbg_build(settings);                        // main.cpp:517
        SDBG sdbg;                                             // main.cpp:522-530
        sdbg.LoadFromDevice(sdbg_build.release_graph());
        std::cout << "Loaded the graph" << std::endl;
        settings.sdbg = &sdbg;
        std::cout << "FBCE START:" << std::endl;
        CycleFinder cycle_finder(settings);                    // main.cpp:536
        auto cycles_map = cycle_finder.results;
        std::cout << "Number of nodes in results: " << cycles_map.size() << std::endl;
        auto cycles = cycles_map_to_cycles(cycles_map);        // main.cpp:542
        const std::string out = settings.cycles_folder + "/cycles.txt";
        std::ofstream f(out);
        if (!f) throw std::runtime_error("Error: cannot write " + out);
        size_t idx = 0;
        for (const auto &[start, inner] : cycles_map)
            for (const auto &c : inner) {
                f << ">cycle_" << idx++ << " start=" << start << " length=" << c.size() << "\n";
                f << cycle_sequence(sdbg, c) << "\n";
            }
        std::cout << "Cycles written to " << out << " (" << cycles.size() << " cycles)" << std::endl;
        std::cout << "Note: read remapping, spacer ordering and CRISPR_Arrays.txt reporting are not part of "
                     "this build." << std::endl;
        return 0;
    } catch (const std::exception &e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
}
