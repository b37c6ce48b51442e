// crispr_report.cpp — CRISPRAnalyzer (reference include/post_processing.h:13-261): filters the
// found (repeat -> spacers) systems and writes the report file named by settings.output_file
// (CRISPR_Arrays.txt). Iteration over the systems map and over the k-mer count maps uses the
// reference's container types filled in the reference's order, so the report lists the same
// systems in the same order with the same repeat extensions.
#include <algorithm>
#include <fstream>
#include <numeric>

#include "downstream.h"

CRISPRAnalyzer::CRISPRAnalyzer(std::unordered_map<std::string, std::vector<std::string>> systems_map,
                               std::string output, int amt, int minsl, int maxsl, int minrl, int maxrl, int mean_sim)
    : systems(std::move(systems_map)),
      output_path(std::move(output)),
      amount(amt),
      min_sl(minsl),
      max_sl(maxsl),
      min_rl(minrl),
      max_rl(maxrl),
      mean_similarity(mean_sim) {}

// k-mers shared by at least 75 % of the sequences (post_processing.h:51-66)
std::vector<std::string> CRISPRAnalyzer::get_common_kmers(const std::vector<std::string> &kmers,
                                                          const std::vector<std::string> &sequences) {
    std::unordered_map<std::string, int> freq;
    for (const auto &x : kmers) freq[x]++;
    const int need = sequences.size() * 0.75;
    std::vector<std::string> out;
    for (const auto &kv : freq)
        if (kv.second >= need) out.push_back(kv.first);
    return out;
}

std::vector<std::string> CRISPRAnalyzer::find_common_prefix_kmers(const std::vector<std::string> &sequences, int k) {
    std::vector<std::string> all;  // every prefix of length 1..k
    for (const auto &s : sequences)
        for (int len = 1; len <= std::min(k, (int)s.size()); ++len) all.push_back(s.substr(0, len));
    return get_common_kmers(all, sequences);
}

std::vector<std::string> CRISPRAnalyzer::find_common_suffix_kmers(const std::vector<std::string> &sequences, int k) {
    std::vector<std::string> all;  // every suffix of length k..1
    for (const auto &s : sequences)
        for (int from = std::max(0, (int)s.size() - k); from < (int)s.size(); ++from) all.push_back(s.substr(from));
    return get_common_kmers(all, sequences);
}

// strip the first matching common prefix and suffix, keep spacers of valid length
std::vector<std::string> CRISPRAnalyzer::trim_kmers_from_sequences(const std::vector<std::string> &sequences,
                                                                   const std::vector<std::string> &prefixes,
                                                                   const std::vector<std::string> &suffixes) {
    std::vector<std::string> out;
    for (std::string s : sequences) {
        for (const auto &p : prefixes)
            if (s.find(p) == 0) {
                s = s.substr(p.size());
                break;
            }
        for (const auto &x : suffixes)
            if (s.size() >= x.size() && s.compare(s.size() - x.size(), x.size(), x) == 0) {
                s = s.substr(0, s.size() - x.size());
                break;
            }
        if ((int)s.size() >= min_sl && (int)s.size() <= max_sl) out.push_back(s);
    }
    return out;
}

// mean pairwise fuzz::ratio must not exceed mean_similarity (post_processing.h:113-125)
bool CRISPRAnalyzer::validate_spacer_diversity(const std::vector<std::string> &sequences) {
    std::vector<double> r;
    for (size_t i = 0; i < sequences.size(); ++i)
        for (size_t j = i + 1; j < sequences.size(); ++j) r.push_back(fuzz::ratio(sequences[i], sequences[j]));
    if (r.empty()) return false;
    const double mean = std::accumulate(r.begin(), r.end(), 0.0) / r.size();
    return mean <= mean_similarity;
}

// longest first; drop a spacer that partial-matches (>= 90) one already kept
std::vector<std::string> CRISPRAnalyzer::filter_substring_spacers(const std::vector<std::string> &spacers) {
    std::vector<std::string> by_len = spacers;
    std::sort(by_len.begin(), by_len.end(), [](const std::string &a, const std::string &b) { return a.size() > b.size(); });
    std::vector<std::string> out;
    std::unordered_set<std::string> kept;
    for (const auto &s : by_len) {
        bool covered = false;
        for (const auto &k : kept)
            if (fuzz::partial_ratio(s, k) >= 90.0) {
                covered = true;
                break;
            }
        if (!covered) {
            kept.insert(s);
            out.push_back(s);
        }
    }
    return out;
}

std::vector<std::string> CRISPRAnalyzer::filter_by_length(const std::vector<std::string> &spacers) {
    std::vector<std::string> out;
    for (const auto &s : spacers)
        if ((int)s.size() >= min_sl && (int)s.size() <= max_sl) out.push_back(s);
    return out;
}

// the repeat grows by the spacers' common prefix on its right and common suffix on its left
std::string CRISPRAnalyzer::reconstruct_repeat(const std::string &original, const std::vector<std::string> &prefixes,
                                               const std::vector<std::string> &suffixes) {
    std::string r = original;
    if (!prefixes.empty()) r += prefixes.back();
    if (!suffixes.empty()) r = suffixes.front() + r;
    return r;
}

void CRISPRAnalyzer::generate_report(const std::string &repeat, const std::vector<std::string> &spacers,
                                     std::ofstream &out) {
    const char *rule = "--------------------------------------------------\n";
    out << rule << repeat << "\n" << rule;
    grouped_repeat_cycles[repeat] = {};
    for (const auto &s : spacers) {
        out << s << "\n";
        grouped_repeat_cycles[repeat].push_back(s);
    }
    out << rule << "Number of Spacers: " << spacers.size() << "\n" << rule << "\n";
}

// post_processing.h:176-259
void CRISPRAnalyzer::run_analysis() {
    std::ofstream report(output_path);
    report << "CRISPR Analysis Report\n"
           << "The tool was run with the following parameters:\n"
           << "Amount of Spacers: " << amount << "\n"
           << "[Min:Max] Length of Spacers: [" << min_sl << ":" << max_sl << "]\n"
           << "[Min:Max] Length of Repeats: [" << min_rl << ":" << max_rl << "]\n"
           << "Mean Similarity Between Spacers: " << mean_similarity << "\n"
           << "Conservation Threshold: 80%\n"
           << "--------------------------------------------------\n";
    auto bad_repeat = [&](const std::string &r) { return (int)r.size() < min_rl || (int)r.size() > max_rl; };
    for (const auto &kv : systems) {
        const std::string &repeat = kv.first;
        const std::vector<std::string> &spacers = kv.second;
        if (spacers.size() < 2) {
            omitted_repeats++;
            continue;
        }
        const int k = this->max_rl - repeat.size();
        auto pre = find_common_prefix_kmers(spacers, k);
        auto suf = find_common_suffix_kmers(spacers, k);
        if (bad_repeat(reconstruct_repeat(repeat, pre, suf))) {
            omitted_repeats++;
            continue;
        }
        const auto trimmed = trim_kmers_from_sequences(spacers, pre, suf);
        if ((int)trimmed.size() < amount) {
            omitted_repeats++;
            continue;
        }
        const std::unordered_set<std::string> distinct(trimmed.begin(), trimmed.end());
        std::vector<std::string> cand(distinct.begin(), distinct.end());
        cand = filter_by_length(filter_substring_spacers(cand));
        if ((int)cand.size() < amount) {
            omitted_repeats++;
            continue;
        }
        // k-mers again after the substring filter, then trim once more
        pre = find_common_prefix_kmers(cand, k);
        suf = find_common_suffix_kmers(cand, k);
        const std::string final_repeat = reconstruct_repeat(repeat, pre, suf);
        if (bad_repeat(final_repeat)) {
            omitted_repeats++;
            continue;
        }
        cand = trim_kmers_from_sequences(cand, pre, suf);
        if ((int)cand.size() < amount || !validate_spacer_diversity(cand)) {
            omitted_repeats++;
            continue;
        }
        generate_report(final_repeat, cand, report);
        total_spacers += cand.size();
    }
    report << "Number of Systems: " << (systems.size() - omitted_repeats) << "\n"
           << "Number of Spacers: " << total_spacers << "\n"
           << "Omitted Repeats: " << omitted_repeats << "\n";
}
