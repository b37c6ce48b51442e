// settings.h — mcaat's Settings / CLI surface, kept drop-in compatible with the reference
// (reference include/settings.h:22-221, src/main.cpp:89-301): the same settings.txt keys,
// defaults, CLI flags and error behaviour (std::runtime_error). Additions, all optional and
// ignored by the reference as unknown keys: `kmer_k` (k is hard-coded to 23 in the
// reference, sdbg_build.cpp:217), `--gpu <index>`, and the multi-GPU `gpus` / `comm`.
#pragma once
#include <algorithm>
#include <cctype>
#include <chrono>
#include <filesystem>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

class SDBG;

struct Settings {
    std::string input_files;   // settings.h:23
    double ram = 0.0;          // GB, settings.h:24
    size_t threads = 0;        // settings.h:25
    std::string output_folder;
    std::string graph_folder;
    std::string cycles_folder;
    std::string output_file;
    std::string benchmark_file;
    int kmer_k = 23;           // reference: "-k 23" (sdbg_build.cpp:217)
    int gpu = 0;
    // checkpoint / resume of the graph (the reference keeps MEGAHIT's graph.sdbg* on disk
    // between SDBGBuild and CycleFinder, main.cpp:386-393): keep_graph writes
    // <graph_folder>/graph.mcaat_sdbg after the build and keeps it; load_graph resumes from
    // such a file instead of building (the reads are still read for the downstream steps)
    bool keep_graph = false;
    std::string load_graph;
    // multi-GPU run (not in the reference): `gpus` ranks, one process per GPU forked by main
    // before any GPU call; rank r runs on GPU (gpu + r) % device count. comm "rccl" moves data
    // GPU to GPU over xGMI, "shm" stages it through host shared memory (ranks may share a
    // GPU). rank / mcomm are filled in per process by main.
    int gpus = 1;
    std::string comm = "rccl";
    int rank = 0;
    struct mcaat_comm *mcomm = nullptr;

    struct CycleFinderSettings {           // settings.h:33-38
        uint64_t threshold_multiplicity = 20;
        bool low_abundance = true;
        int cycle_max_length = 77;
        int cycle_min_length = 27;
    } cycle_finder_settings;
    struct DNASequenceSettings {           // settings.h:39-44
        int spacer_min_length = 23;
        int spacer_max_length = 50;
        int repeat_min_length = 23;
        int repeat_max_length = 50;
    } dna_sequence_settings;

    SDBG *sdbg = nullptr;                  // settings.h:46

    static std::string get_timestamp() {
        auto now = std::chrono::system_clock::now();
        auto t = std::chrono::system_clock::to_time_t(now);
        std::stringstream ss;
        ss << std::put_time(std::localtime(&t), "%Y-%m-%d_%H-%M-%S");
        return ss.str();
    }

    // settings.h:72-100
    std::map<std::string, std::pair<bool, std::string>> validate_settings() const {
        std::map<std::string, std::pair<bool, std::string>> m;
        bool input_valid = !input_files.empty();
        m["Input Files"] = {input_valid, input_valid ? input_files + " exist(s)" : "No input files specified"};
        std::string ram_str = std::to_string(ram).substr(0, std::to_string(ram).find(".") + 3);
        bool ram_valid = ram > 1.0;
        m["RAM"] = {ram_valid, ram_valid ? ram_str + " GB" : "Value " + ram_str + " GB is invalid (must be greater than 1 GB)"};
        size_t max_t = std::thread::hardware_concurrency();
        bool threads_valid = threads > 0 && threads <= max_t;
        m["Threads"] = {threads_valid, threads_valid ? std::to_string(threads) + " thread(s)"
                                                     : "Value " + std::to_string(threads) +
                                                           " is invalid (must be between 1 and " + std::to_string(max_t) + ")"};
        bool out_valid = !output_folder.empty();
        m["Output Folder"] = {out_valid, out_valid ? output_folder : "Invalid output folder"};
        return m;
    }

    // settings.h:103-116
    std::string print_settings() const {
        std::string bad;
        for (const auto &[key, value] : validate_settings()) {
            if (value.first) std::cout << "[✔] " << key << ": " << value.second << std::endl;
            else {
                bad += key + " ";
                std::cout << "[✗] " << key << ": " << value.second << std::endl;
            }
        }
        return bad;
    }

    static bool parse_ram(const std::string &val, double &out) {
        double value = 0.0;
        char unit = 'G';
        size_t p = val.find_first_not_of("0123456789.");
        if (p != std::string::npos) {
            value = std::stod(val.substr(0, p));
            unit = (char)toupper(val[p]);
        } else {
            value = std::stod(val);
        }
        switch (unit) {
            case 'B': out = value / (1024.0 * 1024.0 * 1024.0); return true;
            case 'K': out = value / (1024.0 * 1024.0); return true;
            case 'M': out = value / 1024.0; return true;
            case 'G': out = value; return true;
            default: return false;
        }
    }

    // settings.h:127-220 (key=value, '#' and '//' comments, unknown keys ignored)
    bool LoadFromFile(const std::string &path) {
        std::ifstream file(path);
        if (!file.is_open()) {
            std::cerr << "Could not open settings file: " << path << std::endl;
            return false;
        }
        auto trim = [](std::string s) {
            const char *ws = " \t\n\r\f\v";
            s.erase(0, s.find_first_not_of(ws));
            s.erase(s.find_last_not_of(ws) + 1);
            return s;
        };
        std::string line;
        while (std::getline(file, line)) {
            size_t c = line.find('#');
            if (c != std::string::npos) line = line.substr(0, c);
            c = line.find("//");
            if (c != std::string::npos) line = line.substr(0, c);
            std::string s = trim(line);
            if (s.empty()) continue;
            size_t eq = s.find('=');
            if (eq == std::string::npos) continue;
            std::string key = trim(s.substr(0, eq)), val = trim(s.substr(eq + 1));
            if (key == "input_files") {
                std::vector<std::string> tok;
                std::string cur;
                for (char ch : val) {
                    if (ch == ',' || ch == ';') ch = ' ';
                    if (!isspace((unsigned char)ch)) cur.push_back(ch);
                    else if (!cur.empty()) { tok.push_back(cur); cur.clear(); }
                }
                if (!cur.empty()) tok.push_back(cur);
                input_files.clear();
                for (size_t i = 0; i < tok.size(); ++i) input_files += tok[i] + (i + 1 < tok.size() ? " " : "");
            } else if (key == "ram") {
                try {
                    if (!parse_ram(val, ram)) throw std::runtime_error("unit");
                } catch (...) {
                    std::cerr << "Warning: could not parse RAM value '" << val << "' in settings file" << std::endl;
                }
            } else if (key == "threads") {
                try { threads = std::stoul(val); } catch (...) {}
            } else if (key == "output_folder") output_folder = val;
            else if (key == "graph_folder") graph_folder = val;
            else if (key == "cycles_folder") cycles_folder = val;
            else if (key == "output_file") output_file = val;
            else if (key == "cycle_max_length") cycle_finder_settings.cycle_max_length = std::stoi(val);
            else if (key == "cycle_min_length") cycle_finder_settings.cycle_min_length = std::stoi(val);
            else if (key == "threshold_multiplicity") cycle_finder_settings.threshold_multiplicity = std::stoull(val);
            else if (key == "low_abundance") {
                std::transform(val.begin(), val.end(), val.begin(), ::tolower);
                cycle_finder_settings.low_abundance = (val == "true" || val == "1" || val == "yes");
            } else if (key == "spacer_min_length") dna_sequence_settings.spacer_min_length = std::stoi(val);
            else if (key == "spacer_max_length") dna_sequence_settings.spacer_max_length = std::stoi(val);
            else if (key == "repeat_min_length") dna_sequence_settings.repeat_min_length = std::stoi(val);
            else if (key == "repeat_max_length") dna_sequence_settings.repeat_max_length = std::stoi(val);
            else if (key == "kmer_k") kmer_k = std::stoi(val);
            else if (key == "keep_graph") {
                std::transform(val.begin(), val.end(), val.begin(), ::tolower);
                keep_graph = (val == "true" || val == "1" || val == "yes");
            } else if (key == "load_graph") load_graph = val;
            else if (key == "gpus") gpus = std::stoi(val);
            else if (key == "comm") comm = val;
            // unknown keys are ignored for forward-compatibility (settings.h:216)
        }
        return true;
    }
};

// main.cpp:89-301. `create_dirs` = false leaves the file system untouched (tests).
Settings parse_arguments(int argc, char *argv[], bool create_dirs = true);
double get_total_system_ram();
