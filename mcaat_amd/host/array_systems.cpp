// array_systems.cpp — from ordered cycles to (repeat, spacers, array sequence) (reference
// src/tmp_utils.cpp get_systems and helpers) and the benchmark comparison helpers (reference
// src/evaluation.cpp).
#include <algorithm>

#include "downstream.h"

void trim_string(std::string &s) {  // tmp_utils.cpp:3-6
    s.erase(0, s.find_first_not_of(" \t\n\r"));
    s.erase(s.find_last_not_of(" \t\n\r") + 1);
}

// tmp_utils.cpp:8-24: "f1 f2" -> (f1, f2); anything after the first space is the second file
std::pair<std::string, std::optional<std::string>> get_fastq_files_from_settings(const Settings &settings) {
    const size_t sp = settings.input_files.find(' ');
    if (sp == std::string::npos) return {settings.input_files, std::nullopt};
    std::string a = settings.input_files.substr(0, sp), b = settings.input_files.substr(sp + 1);
    trim_string(a);
    trim_string(b);
    return {a, std::optional<std::string>(b)};
}

int get_cycle_count(const std::vector<std::vector<uint64_t>> &cycles) {  // tmp_utils.cpp:40-48: total nodes
    int n = 0;
    for (const auto &c : cycles) n += c.size();
    return n;
}

// tmp_utils.cpp:83-90: the k symbols of the edge's source-node label as ACGT text
std::string fetch_node_label(SDBG &sdbg, const size_t &node) {
    std::vector<uint8_t> seq(sdbg.k());
    sdbg.GetLabel(node, seq.data());
    std::string label(sdbg.k(), 'A');
    for (int i = 0; i < sdbg.k(); ++i) label[i] = "ACGT"[seq[i] - 1];
    return label;
}

// tmp_utils.cpp:201-323. All ordered cycles share the repeat; walking forward from each
// cycle's first node while the cycles agree on the next label symbol (a single disagreement
// followed by agreement is a point mutation) and backward from the last node in the same way
// locates the repeat boundaries; each cycle is then rotated to start at the repeat and split
// into its repeat and spacer, the most frequent repeat is the consensus, and the array is the
// concatenation of the cycles carrying the consensus repeat, closed by one more repeat.
std::tuple<std::string, std::vector<std::string>, std::string> get_systems(
    SDBG &sdbg, std::vector<std::vector<uint64_t>> &ordered_cycles) {
    int shortest = ordered_cycles.at(0).size();
    for (const auto &c : ordered_cycles) shortest = std::min<int>(shortest, c.size());

    // one symbol of a node's label (fetch_node_label(...).at(0) / .back()) without building the
    // label string: C3 has 800 regions of ~24 cycles of ~70 nodes, and a k-symbol string per look
    // was most of the step's emit time
    const int kk = sdbg.k();
    auto symbol = [&](uint64_t node, bool last_symbol) {
        uint8_t seq[64];
        sdbg.GetLabel(node, seq);
        return "ACGT"[seq[last_symbol ? kk - 1 : 0] - 1];
    };
    // label symbol at `pos` of every cycle (front: first symbol, back: last symbol)
    auto distinct_at = [&](bool from_end, int i, bool last_symbol) {
        bool seen[4] = {false, false, false, false};
        size_t n = 0;
        for (const auto &c : ordered_cycles) {
            const uint64_t node = from_end ? c.at(c.size() - i - 1) : c.at(i);
            const char ch = symbol(node, last_symbol);
            const int b = ch == 'A' ? 0 : ch == 'C' ? 1 : ch == 'G' ? 2 : 3;
            if (!seen[b]) {
                seen[b] = true;
                ++n;
            }
        }
        return n;
    };
    int right = 0;
    for (int i = 0; i < shortest - 1; ++i) {
        if (distinct_at(false, i, false) > 1 && distinct_at(false, i + 1, false) != 1) {
            right = i;
            break;
        }
    }
    int left = 0;
    for (int i = 0; i < shortest - 1; ++i) {
        if (distinct_at(true, i, true) > 1 && distinct_at(true, i + 1, true) != 1) {
            left = i;
            break;
        }
    }
    const int repeat_length = left + right - sdbg.k();

    std::vector<std::string> spacers, repeats;
    for (const auto &c : ordered_cycles) {
        std::string spacer, repeat;
        const int shift = c.size() - left;
        for (int i = 0; i < (int)c.size(); ++i) {
            const char last = symbol(c.at((shift + i) % c.size()), true);
            (i < repeat_length ? repeat : spacer) += last;
        }
        spacers.push_back(spacer);
        repeats.push_back(repeat);
    }
    std::unordered_map<std::string, int> votes;
    for (const auto &r : repeats) votes[r]++;
    std::string consensus;
    int top = 0;
    for (const auto &kv : votes)  // first maximum in the map's iteration order
        if (kv.second > top) {
            top = kv.second;
            consensus = kv.first;
        }
    std::string sequence;
    for (size_t i = 0; i < spacers.size(); ++i)
        if (repeats[i] == consensus) sequence += repeats[i] + spacers[i];
    sequence += consensus;
    return std::make_tuple(consensus, spacers, sequence);
}

// ---------------------------------------------------------------- evaluation.cpp
uint16_t get_levenshtein_distance(const std::string &s1, const std::string &s2) {  // evaluation.cpp:3-48
    std::vector<uint16_t> prev(s1.size() + 1), cur(s1.size() + 1);
    for (size_t x = 0; x <= s1.size(); ++x) prev[x] = x;
    for (size_t y = 1; y <= s2.size(); ++y) {
        cur[0] = y;
        for (size_t x = 1; x <= s1.size(); ++x) {
            uint16_t best = prev[x - 1] + (s1[x - 1] == s2[y - 1] ? 0 : 1);
            best = std::min<uint16_t>(best, cur[x - 1] + 1);
            best = std::min<uint16_t>(best, prev[x] + 1);
            cur[x] = best;
        }
        std::swap(prev, cur);
    }
    return prev[s1.size()];
}

float get_string_similarity(const std::string &s1, const std::string &s2) {  // evaluation.cpp:50-55
    const uint16_t d = get_levenshtein_distance(s1, s2);
    const size_t m = std::max(s1.size(), s2.size());
    return 1.0 - (static_cast<float>(d) / static_cast<float>(m));
}

int get_number_of_duplicate_spacers(const std::vector<std::string> &spacers,
                                    const std::string &expected_sequence) {  // evaluation.cpp:57-78
    int extra = 0;
    for (const auto &sp : spacers) {
        int hits = 0;
        for (size_t pos = expected_sequence.find(sp); pos != std::string::npos; pos = expected_sequence.find(sp, pos + 1))
            ++hits;
        if (hits > 1) extra += hits - 1;
    }
    return extra;
}

std::string get_most_similar_sequence(const std::string &sequence,
                                      const std::vector<std::string> &choices) {  // evaluation.cpp:80-106
    std::string best;
    float best_sim = -1.0;
    for (const auto &c : choices) {
        const float sim = get_string_similarity(sequence, c);
        if (sim > best_sim) {
            best_sim = sim;
            best = c;
        }
    }
    return best;
}
