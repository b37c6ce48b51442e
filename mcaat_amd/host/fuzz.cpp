// fuzz.cpp — the two rapidfuzz scores CRISPRAnalyzer uses (post_processing.h:118,137).
// rapidfuzz-cpp is an absent third-party dependency with no pinned version (SURVEY.md §8f:
// "parity unpinned"); this restates its published definitions (rapidfuzz-cpp 3.x):
//   ratio(a, b)         = 100 * (1 - indel(a, b) / (|a| + |b|)), indel = |a| + |b| - 2 LCS
//                         (100 when both are empty);
//   partial_ratio(a, b) = best ratio of the shorter string against the windows of the longer
//                         one: its prefixes shorter than the needle (skipped when their last
//                         symbol is not in the needle), every full-length window, and its
//                         suffixes from |long|-|short| on (skipped when their first symbol is
//                         not in the needle); for equal lengths the swapped direction is tried
//                         too unless the first already scored 100. Empty input: 100 if both
//                         are empty, else 0.
// CRISPRAnalyzer only compares spacers of 23..50 symbols, so the short-needle (<= 64)
// variant is the one restated.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "downstream.h"

namespace {

// bit-parallel LCS (Hyyro's formulation, as rapidfuzz computes it for patterns of <= 64
// symbols): PM[c] has bit i set where a[i] == c; one add/or per symbol of b
struct Pattern {
    uint64_t pm[256] = {};
    size_t n = 0;
    Pattern(const char *a, size_t na) : n(na) {
        for (size_t i = 0; i < na; ++i) pm[(unsigned char)a[i]] |= 1ULL << i;
    }
    size_t lcs(const char *b, size_t nb) const {
        uint64_t S = ~0ULL;
        for (size_t j = 0; j < nb; ++j) {
            const uint64_t u = S & pm[(unsigned char)b[j]];
            S = (S + u) | (S - u);
        }
        const uint64_t mask = n >= 64 ? ~0ULL : ((1ULL << n) - 1);
        return (size_t)__builtin_popcountll(~S & mask);
    }
};

size_t lcs_length(const char *a, size_t na, const char *b, size_t nb) {
    if (!na || !nb) return 0;
    if (na <= 64) return Pattern(a, na).lcs(b, nb);
    if (nb <= 64) return Pattern(b, nb).lcs(a, na);
    std::vector<uint32_t> row(nb + 1, 0);
    for (size_t i = 0; i < na; ++i) {
        uint32_t diag = 0;
        for (size_t j = 0; j < nb; ++j) {
            const uint32_t up = row[j + 1];
            row[j + 1] = a[i] == b[j] ? diag + 1 : std::max(up, row[j]);
            diag = up;
        }
    }
    return row[nb];
}

double ratio_raw(const char *a, size_t na, const char *b, size_t nb) {
    const size_t sum = na + nb;
    if (!sum) return 100.0;
    const size_t dist = sum - 2 * lcs_length(a, na, b, nb);
    return (1.0 - static_cast<double>(dist) / static_cast<double>(sum)) * 100.0;
}

double partial_short_needle(const std::string &needle, const std::string &hay) {
    const size_t n1 = needle.size(), n2 = hay.size();
    bool in_needle[256] = {false};
    for (unsigned char c : needle) in_needle[c] = true;
    double best = 0.0;
    const Pattern pat(needle.data(), std::min<size_t>(n1, 64));  // used when n1 <= 64 (CRISPRAnalyzer's spacers)
    auto consider = [&](size_t first, size_t len) {
        double r;
        if (n1 <= 64) {
            const size_t sum = n1 + len;
            r = sum ? (1.0 - static_cast<double>(sum - 2 * pat.lcs(hay.data() + first, len)) / static_cast<double>(sum)) * 100.0
                    : 100.0;
        } else {
            r = ratio_raw(needle.data(), n1, hay.data() + first, len);
        }
        if (r > best) best = r;
    };
    for (size_t i = 1; i < n1 && best < 100.0; ++i)
        if (in_needle[(unsigned char)hay[i - 1]]) consider(0, i);
    for (size_t i = 0; i + n1 < n2 && best < 100.0; ++i) consider(i, n1);
    for (size_t i = n2 - n1; i < n2 && best < 100.0; ++i)
        if (in_needle[(unsigned char)hay[i]]) consider(i, n2 - i);
    return best;
}

}  // namespace

namespace fuzz {

double ratio(const std::string &s1, const std::string &s2) { return ratio_raw(s1.data(), s1.size(), s2.data(), s2.size()); }

double partial_ratio(const std::string &s1, const std::string &s2) {
    if (s1.size() > s2.size()) return partial_ratio(s2, s1);
    if (s1.empty() || s2.empty()) return s1.size() == s2.size() ? 100.0 : 0.0;
    double r = partial_short_needle(s1, s2);
    if (r != 100.0 && s1.size() == s2.size()) r = std::max(r, partial_short_needle(s2, s1));
    return r;
}

}  // namespace fuzz
