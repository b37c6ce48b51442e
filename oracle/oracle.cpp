/*
 * oracle.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h). CPU restatement of the
 * mcaat hot path. Nothing in the product links this file.
 *
 * Parity status: "parity unpinned" (oracle.h).
 *
 * Encoding conventions (DESIGN.md "SDBG conventions", shared with the HIP path
 * only through this written spec, not through code):
 *   base codes A=0 C=1 G=2 T=3; packed reads: base j at word j>>5, bits 2*(j&31)
 *   edge e = s[0..k] ((k+1)-mer). lsb(e) = sum s[i] << 2i.
 *   canonical(e) = min(lsb(e), lsb(rc(e))).
 *   BOSS key K(e) = ((lsb & mask_2k) << 2) | s[k]: colex order of the source-node
 *   label s[0..k-1] (compared from s[k-1] backwards) then the outgoing symbol W.
 *   Edge id = rank of K among all distinct oriented edges.
 *   mult(e) = occ(e) + occ(rc(e)) (palindromes: 2*occ), saturating at 65535.
 */
#include "oracle.h"

#include <omp.h>
#include <parallel/algorithm>
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

using std::vector;

namespace {

inline uint64_t mask_bits(int nbits) { return nbits >= 64 ? ~0ULL : ((1ULL << nbits) - 1); }

inline int base_at(const uint64_t *packed, uint64_t j) { return (packed[j >> 5] >> (2 * (j & 31))) & 3; }

/* reverse the order of the 2-bit groups of an E-symbol LSB-first value */
inline uint64_t rev_groups(uint64_t x, int E) {
    uint64_t r = 0;
    for (int i = 0; i < E; ++i) { r = (r << 2) | (x & 3); x >>= 2; }
    return r;
}

inline uint64_t lsb_rc(uint64_t lsb, int E) { return rev_groups(lsb, E) ^ mask_bits(2 * E); }

inline uint64_t boss_key(uint64_t lsb, int k) {
    return ((lsb & mask_bits(2 * k)) << 2) | (lsb >> (2 * k));
}

/* canonical (k+1)-mers of all reads, one vector per thread then merged */
vector<uint64_t> collect_canonical(const uint64_t *packed, const uint64_t *offsets, uint64_t n_reads,
                                   int k, int threads) {
    const int E = k + 1;
    const uint64_t M = mask_bits(2 * E);
    vector<vector<uint64_t>> parts(threads);
#pragma omp parallel num_threads(threads)
    {
        auto &out = parts[omp_get_thread_num()];
#pragma omp for schedule(dynamic, 4096)
        for (uint64_t r = 0; r < n_reads; ++r) {
            const uint64_t a = offsets[r], b = offsets[r + 1];
            uint64_t lsb = 0, msb = 0;
            for (uint64_t j = a; j < b; ++j) {
                const uint64_t c = base_at(packed, j);
                lsb = (lsb >> 2) | (c << (2 * (E - 1)));
                msb = ((msb << 2) | c) & M;
                if (j - a + 1 >= (uint64_t)E) {
                    const uint64_t rc = msb ^ M;
                    out.push_back(lsb < rc ? lsb : rc);
                }
            }
        }
    }
    size_t total = 0;
    for (auto &p : parts) total += p.size();
    vector<uint64_t> all;
    all.reserve(total);
    for (auto &p : parts) { all.insert(all.end(), p.begin(), p.end()); vector<uint64_t>().swap(p); }
    return all;
}

struct Graph {
    int k = 0;
    vector<uint64_t> key;   // sorted BOSS keys
    vector<uint16_t> mult;
    vector<uint8_t> valid;  // one byte per edge (race-free parallel SetInvalidEdge)

    uint64_t size() const { return key.size(); }
    uint64_t lower(uint64_t q) const { return std::lower_bound(key.begin(), key.end(), q) - key.begin(); }

    /* MEGAHIT API subset, valid-only neighbour semantics. */
    bool IsValidEdge(uint64_t e) const { return valid[e] != 0; }
    void SetInvalidEdge(uint64_t e) { valid[e] = 0; }
    void SetValidEdge(uint64_t e) { valid[e] = 1; }
    uint16_t EdgeMultiplicity(uint64_t e) const { return mult[e]; }

    /* outgoing edges = edges of node target(e); emitted in DESCENDING id order */
    int OutgoingEdges(uint64_t e, uint64_t *out) const {
        const uint64_t K = key[e], W = K & 3, R = K >> 2;
        const uint64_t Rt = (W << (2 * (k - 1))) | (R >> 2);
        uint64_t lo = lower(Rt << 2);
        uint64_t tmp[4];
        int n = 0;
        for (uint64_t i = lo; i < size() && (key[i] >> 2) == Rt; ++i)
            if (valid[i]) tmp[n++] = i;
        for (int i = 0; i < n; ++i) out[i] = tmp[n - 1 - i];
        return n;
    }
    /* incoming edges: (k-1)-group of the label suffix, W == last label symbol; ASCENDING */
    int IncomingEdges(uint64_t e, uint64_t *in) const {
        const uint64_t K = key[e];
        const uint64_t c = (K >> (2 * k)) & 3;
        const uint64_t G = (K >> 2) & mask_bits(2 * (k - 1));
        uint64_t lo = lower(G << 4);
        int n = 0;
        for (uint64_t i = lo; i < size() && (key[i] >> 4) == G; ++i)
            if ((key[i] & 3) == c && valid[i]) in[n++] = i;
        return n;
    }
    int EdgeOutdegree(uint64_t e) const { uint64_t t[4]; return OutgoingEdges(e, t); }
    int EdgeIndegree(uint64_t e) const { uint64_t t[4]; return IncomingEdges(e, t); }
    bool EdgeOutdegreeZero(uint64_t e) const { return EdgeOutdegree(e) == 0; }
    int GetLabel(uint64_t e, uint8_t *seq) const {
        const uint64_t R = key[e] >> 2;
        for (int i = 0; i < k; ++i) seq[i] = ((R >> (2 * i)) & 3) + 1;
        return k;
    }
    int64_t IndexBinarySearch(const uint8_t *seq) const {
        uint64_t R = 0;
        for (int i = 0; i < k; ++i) R |= (uint64_t)((seq[i] - 1) & 3) << (2 * i);
        uint64_t lo = lower(R << 2);
        int64_t last = -1;
        for (uint64_t i = lo; i < size() && (key[i] >> 2) == R; ++i) last = (int64_t)i;
        return last;
    }
};

/* ---------------- CycleFinder restatement (cycle_finder.cpp) ---------------- */
struct CycleFinderO {
    Graph &sdbg;
    oracle_cf_params st;
    uint16_t cluster_bounds = 500;          // cycle_finder.cpp:132
    vector<uint8_t> visited;                // cycle_finder.h:33 (vector<bool>)
    vector<std::pair<uint64_t, vector<vector<uint64_t>>>> committed;  // commit order
    std::unordered_map<uint64_t, vector<vector<uint64_t>>> results;   // cycle_finder.h:60
    vector<uint64_t> cand_ids; vector<int32_t> cand_bucket;
    uint64_t stats[6] = {0, 0, 0, 0, 0, 0};

    CycleFinderO(Graph &g, const oracle_cf_params &p) : sdbg(g), st(p) {
        if (st.cluster_bound > 0) cluster_bounds = (uint16_t)st.cluster_bound;
        if (st.step_cap <= 0) st.step_cap = 10000000;
    }

    // cycle_finder.cpp:29-36
    bool IncomingNotEqualToCurrentNode(uint64_t node, size_t indeg) {
        vector<uint64_t> in(std::max<size_t>(indeg, 4));
        sdbg.IncomingEdges(node, in.data());
        for (size_t i = 0; i < indeg; ++i) if (in[i] == node) return true;
        return false;
    }
    // cycle_finder.cpp:40-52
    bool BackgroundCheck(uint64_t original, size_t repeat_mult, uint64_t nb) {
        auto nm = sdbg.EdgeMultiplicity(nb);
        if (visited[nb]) return false;
        if (repeat_mult / nm > 500) return false;
        if (original == nb) return false;
        return true;
    }
    // cycle_finder.cpp:58-72
    void GetOutgoings(uint64_t node, std::unordered_set<uint64_t> &set, size_t rm) {
        int od = sdbg.EdgeOutdegree(node);
        if (od == 0 || !sdbg.IsValidEdge(node)) return;
        uint64_t out[4];
        int flag = sdbg.OutgoingEdges(node, out);
        if (flag != -1)
            for (int i = 0; i < od; ++i)
                if (BackgroundCheck(node, rm, out[i]) && sdbg.IsValidEdge(out[i])) set.insert(out[i]);
    }
    // cycle_finder.cpp:76-88
    void GetIncomings(uint64_t node, std::unordered_set<uint64_t> &set, size_t rm) {
        int id = sdbg.EdgeIndegree(node);
        if (id == 0 || !sdbg.IsValidEdge(node)) return;
        uint64_t in[4];
        int flag = sdbg.IncomingEdges(node, in);
        if (flag != -1)
            for (int i = 0; i < id; ++i)
                if (BackgroundCheck(node, rm, in[i]) && sdbg.IsValidEdge(in[i])) set.insert(in[i]);
    }
    // cycle_finder.cpp:111-123 (DLS/peel helper, no background check)
    void GetIncomingsPlain(uint64_t node, std::unordered_set<uint64_t> &set) {
        int id = sdbg.EdgeIndegree(node);
        if (id == 0 || !sdbg.IsValidEdge(node)) return;
        uint64_t in[4];
        int flag = sdbg.IncomingEdges(node, in);
        if (flag != -1)
            for (int i = 0; i < id; ++i)
                if (sdbg.IsValidEdge(in[i])) set.insert(in[i]);
    }

    // cycle_finder.cpp:140-225
    vector<vector<uint64_t>> FindCycle(uint64_t start, vector<uint64_t> path, std::map<uint64_t, int> lock,
                                       vector<std::unordered_set<uint64_t>> stack, vector<int> bl) {
        const int maxl = st.cycle_max_length, minl = st.cycle_min_length;
        int counter = 0;
        vector<vector<uint64_t>> cycles;
        long long steps = 0;
        while (!stack.empty()) {
            steps += 1;
            if (steps > st.step_cap) break;
            std::unordered_set<uint64_t> neighbors = stack.back();
            bool flag = true;
            for (auto nb : neighbors) {
                if (nb == start) {
                    bl.back() = 1;
                    if (path.size() > (size_t)minl) {
                        cycles.push_back(path);
                        counter += 1;
                        if (counter >= cluster_bounds) { cycles.clear(); flag = false; }
                    }
                } else if ((int)path.size() < lock.try_emplace(nb, maxl).first->second) {
                    neighbors.erase(nb);
                    path.push_back(nb);
                    bl.push_back(maxl);
                    lock[nb] = path.size();
                    stack.back().erase(nb);
                    std::unordered_set<uint64_t> outs;
                    GetOutgoings(nb, outs, sdbg.EdgeMultiplicity(start));
                    stack.push_back(outs);
                    flag = false;
                    break;
                }
            }
            if (flag) {
                stack.pop_back();
                uint64_t v = path.back();
                path.pop_back();
                int b = bl.back();
                bl.pop_back();
                if (!bl.empty()) bl.back() = std::min(bl.back(), b);
                if (b < maxl) {
                    /* NB: the reference stores node ids as int here (cycle_finder.cpp:192-207);
                     * this restatement keeps 64-bit ids (identical below 2^31, defined above). */
                    vector<std::pair<int, uint64_t>> relax;
                    relax.push_back({b, v});
                    std::unordered_set<uint64_t> path_set(path.begin(), path.end());
                    while (!relax.empty()) {
                        int blv = relax.back().first;
                        uint64_t u = relax.back().second;
                        relax.pop_back();
                        if (lock.try_emplace(u, maxl).first->second < maxl - blv + 1) {
                            lock[u] = maxl - blv + 1;
                            std::unordered_set<uint64_t> ins;
                            GetIncomings(u, ins, sdbg.EdgeMultiplicity(start));
                            for (auto w : ins)
                                if (path_set.find(w) == path_set.end()) relax.push_back({blv + 1, w});
                        }
                    }
                }
            }
        }
        if (cycles.empty()) return {};
        for (const auto &c : cycles)
            for (auto x : c) visited[x] = 1;
        return cycles;
    }
    // cycle_finder.cpp:231-243
    vector<vector<uint64_t>> FindCycleUtil(uint64_t start) {
        vector<uint64_t> path{start};
        std::map<uint64_t, int> lock;
        vector<std::unordered_set<uint64_t>> stack;
        vector<int> bl;
        lock[start] = 0;
        std::unordered_set<uint64_t> outs;
        GetOutgoings(start, outs, sdbg.EdgeMultiplicity(start));
        stack.push_back(outs);
        bl.push_back(st.cycle_max_length);
        return FindCycle(start, path, lock, stack, bl);
    }
    // cycle_finder.cpp:248-343
    bool DepthLevelSearch(uint64_t start, uint64_t target, int limit) const {
        struct SE { uint64_t node; int depth; };
        vector<SE> stk;
        std::unordered_set<uint64_t> vis;
        stk.push_back({start, 0});
        while (!stk.empty()) {
            SE cur = stk.back();
            stk.pop_back();
            uint64_t v = cur.node;
            int depth = cur.depth;
            if (!sdbg.IsValidEdge(v)) continue;
            if (sdbg.EdgeOutdegreeZero(v)) continue;
            int od = sdbg.EdgeOutdegree(v);
            uint64_t nbrs[4];
            int flag = sdbg.OutgoingEdges(v, nbrs);
            if (flag == -1) continue;
            if (depth >= limit) continue;
            for (int i = 0; i < od; ++i) {
                uint64_t nb = nbrs[i];
                if (!sdbg.IsValidEdge(nb)) continue;
                bool not_visited = vis.find(nb) == vis.end();
                bool start_revisit = (nb == start && depth > 0);
                if (not_visited || start_revisit) { vis.insert(nb); stk.push_back({nb, depth + 1}); }
            }
            if (v == target && depth > 1) return true;
        }
        return false;
    }
    // cycle_finder.cpp:346-357
    vector<uint64_t> CollectTips() {
        vector<uint64_t> tips;
        const uint64_t D = sdbg.size();
        vector<vector<uint64_t>> parts(st.threads);
#pragma omp parallel num_threads(st.threads)
        {
            auto &o = parts[omp_get_thread_num()];
#pragma omp for schedule(static)
            for (uint64_t n = 0; n < D; ++n)
                if (sdbg.EdgeOutdegree(n) == 0 && sdbg.IsValidEdge(n)) o.push_back(n);
        }
        for (auto &p : parts) tips.insert(tips.end(), p.begin(), p.end());
        return tips;
    }
    // cycle_finder.cpp:359-371, recursion replaced by an explicit frame stack that
    // visits nodes in exactly the recursive order (no stack overflow on long chains).
    void RecursiveReduction(uint64_t tip) {
        struct Frame { vector<uint64_t> parents; size_t i; };
        vector<Frame> fs;
        auto enter = [&](uint64_t t) -> bool {
            if (sdbg.EdgeOutdegree(t) > 0) return false;
            std::unordered_set<uint64_t> ps;
            GetIncomingsPlain(t, ps);
            sdbg.SetInvalidEdge(t);
            fs.push_back({vector<uint64_t>(ps.begin(), ps.end()), 0});
            return true;
        };
        enter(tip);
        while (!fs.empty()) {
            Frame &f = fs.back();
            if (f.i >= f.parents.size()) { fs.pop_back(); continue; }
            uint64_t p = f.parents[f.i++];
            if (sdbg.IsValidEdge(p)) enter(p);
        }
    }
    // cycle_finder.cpp:372-382
    uint64_t InvalidateMultiplicityOneNodes() {
        uint64_t inv = 0;
        const uint64_t D = sdbg.size();
#pragma omp parallel for num_threads(st.threads) reduction(+ : inv)
        for (uint64_t n = 0; n < D; ++n)
            if (sdbg.EdgeMultiplicity(n) <= 1) { sdbg.SetInvalidEdge(n); inv += 1; }
        return inv;
    }
    // cycle_finder.cpp:387-427 (bucket contents sorted = the threads=1 order)
    void ChunkStartNodes(std::map<int, vector<uint64_t>, std::greater<int>> &chunks) {
        if (!st.low_abundance) InvalidateMultiplicityOneNodes();
        const uint64_t D = sdbg.size();
        vector<vector<std::pair<int, uint64_t>>> parts(st.threads);
#pragma omp parallel num_threads(st.threads)
        {
            auto &o = parts[omp_get_thread_num()];
#pragma omp for schedule(dynamic, 20000)
            for (uint64_t node = 0; node < D; ++node) {
                if (!sdbg.IsValidEdge(node)) continue;
                size_t indeg = sdbg.EdgeIndegree(node);
                if (indeg >= 2 && sdbg.EdgeMultiplicity(node) > st.threshold_multiplicity) {
                    if (IncomingNotEqualToCurrentNode(node, indeg)) continue;
                    if (!DepthLevelSearch(node, node, st.cycle_max_length)) continue;
                    double l2 = std::ceil(std::log2(double(sdbg.EdgeMultiplicity(node))));
                    o.push_back({(int)l2, node});
                }
            }
        }
        for (auto &p : parts)
            for (auto &pr : p) chunks[pr.first].push_back(pr.second);
        for (auto &kv : chunks) std::sort(kv.second.begin(), kv.second.end());
    }
    // cycle_finder.cpp:433-492 (bucket loop with threads=1 semantics)
    void Run() {
        vector<uint64_t> tips = CollectTips();
        stats[0] = tips.size();
        stats[1] = InvalidateMultiplicityOneNodes();
        for (uint64_t t : tips) RecursiveReduction(t);
        uint64_t valid = 0;
        for (uint64_t n = 0; n < sdbg.size(); ++n) valid += sdbg.IsValidEdge(n);
        stats[2] = valid;
        stats[3] = CollectTips().size();
        visited.assign(sdbg.size(), 0);
        std::map<int, vector<uint64_t>, std::greater<int>> chunks;
        ChunkStartNodes(chunks);
        for (auto &kv : chunks)
            for (auto id : kv.second) { cand_ids.push_back(id); cand_bucket.push_back(kv.first); }
        stats[4] = cand_ids.size();
        uint64_t total = 0;
        for (auto &kv : chunks) {
            for (uint64_t s : kv.second) {
                if (visited[s]) continue;
                auto cyc = FindCycleUtil(s);
                total += cyc.size();
                results[s] = cyc;
                committed.push_back({s, std::move(cyc)});
            }
        }
        stats[5] = total;
    }
};

/* ---------------- relevant reads (reads.cpp) ---------------- */
// reads.cpp:20-31
void reverse_pair_ends_sequence(std::string &sequence) {
    std::reverse(sequence.begin(), sequence.end());
    for (char &base : sequence) {
        if (base == 'A') base = 'T';
        else if (base == 'T') base = 'A';
        else if (base == 'C') base = 'G';
        else if (base == 'G') base = 'C';
    }
}
// reads.cpp:33-55
uint64_t k_mer_to_node_id(const Graph &sdbg, const std::string &k_mer) {
    if ((int)k_mer.size() != sdbg.k) return 0;
    std::vector<uint8_t> seq(sdbg.k);
    for (int i = 0; i < sdbg.k; ++i) {
        const char c = k_mer[i];
        seq[i] = c == 'A' ? 1 : c == 'C' ? 2 : c == 'G' ? 3 : 4;
    }
    return (uint64_t)sdbg.IndexBinarySearch(seq.data());
}
// reads.cpp:57-86
std::vector<uint64_t> get_read_from_sequence(const Graph &sdbg, const std::unordered_set<uint64_t> &nodes_of_cycles,
                                             const std::string &sequence) {
    const uint32_t K = sdbg.k;
    if (sequence.size() <= 2 * K) return {};
    const uint64_t start_node_id = k_mer_to_node_id(sdbg, sequence.substr(0, K));
    const uint64_t end_node_id = k_mer_to_node_id(sdbg, sequence.substr(sequence.size() - K, K));
    if (!nodes_of_cycles.count(start_node_id) && !nodes_of_cycles.count(end_node_id)) return {};
    std::vector<uint64_t> read = {start_node_id};
    for (size_t i = 1; i < sequence.size() - K; ++i) read.push_back(k_mer_to_node_id(sdbg, sequence.substr(i, K)));
    read.push_back(end_node_id);
    return read;
}

}  // namespace

struct oracle_graph { Graph g; };
struct oracle_cf_result {
    vector<uint64_t> starts, cyc_begin, node_begin, nodes, map_order, cand_ids;
    vector<int32_t> cand_bucket;
    uint64_t stats[6];
};

extern "C" {

uint64_t oracle_count_canonical(const uint64_t *packed, const uint64_t *offsets, uint64_t n_reads, int k,
                                int threads, uint64_t **keys, uint32_t **counts) {
    if (threads < 1) threads = 1;
    vector<uint64_t> all = collect_canonical(packed, offsets, n_reads, k, threads);
    __gnu_parallel::sort(all.begin(), all.end());
    uint64_t n = 0;
    for (size_t i = 0; i < all.size(); ++i) if (i == 0 || all[i] != all[i - 1]) ++n;
    *keys = (uint64_t *)malloc(sizeof(uint64_t) * (n ? n : 1));
    *counts = (uint32_t *)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint64_t j = 0;
    for (size_t i = 0; i < all.size();) {
        size_t e = i;
        while (e < all.size() && all[e] == all[i]) ++e;
        (*keys)[j] = all[i];
        (*counts)[j] = (uint32_t)std::min<uint64_t>(e - i, 0xFFFFFFFFu);
        ++j;
        i = e;
    }
    return n;
}

uint64_t oracle_read_fastq(const char *path, uint64_t **packed, uint64_t *n_words, uint64_t **offsets) {
    FILE *f = fopen(path, "rb");
    if (!f) return ~0ULL;
    vector<uint64_t> words, offs{0};
    uint64_t nb = 0;
    auto put = [&](int c) {
        if ((nb & 31) == 0) words.push_back(0);
        words.back() |= (uint64_t)c << (2 * (nb & 31));
        ++nb;
    };
    auto close_read = [&]() { if (nb != offs.back()) offs.push_back(nb); };
    std::vector<char> buf(1 << 24);
    std::string line;
    uint64_t lineno = 0;
    bool bad = false;
    size_t got;
    auto on_line = [&](const std::string &l) {
        const uint64_t r = lineno++ & 3;
        if (r == 0 && (l.empty() || l[0] != '@')) bad = true;
        if (r != 1) return;
        for (char ch : l) {
            const int c = ch == 'A' || ch == 'a' ? 0 : ch == 'C' || ch == 'c' ? 1 : ch == 'G' || ch == 'g' ? 2
                          : ch == 'T' || ch == 't' ? 3 : -1;
            if (c < 0) close_read();
            else put(c);
        }
        close_read();
    };
    while ((got = fread(buf.data(), 1, buf.size(), f)) > 0) {
        size_t a = 0;
        for (size_t i = 0; i < got; ++i)
            if (buf[i] == '\n') {
                line.append(buf.data() + a, i - a);
                if (!line.empty() && line.back() == '\r') line.pop_back();
                on_line(line);
                line.clear();
                a = i + 1;
            }
        line.append(buf.data() + a, got - a);
    }
    if (!line.empty()) on_line(line);
    fclose(f);
    if (bad || (lineno & 3) != 0) return ~0ULL;
    *n_words = words.size();
    *packed = (uint64_t *)malloc(8 * (words.size() ? words.size() : 1));
    if (!words.empty()) memcpy(*packed, words.data(), 8 * words.size());
    *offsets = (uint64_t *)malloc(8 * offs.size());
    memcpy(*offsets, offs.data(), 8 * offs.size());
    return offs.size() - 1;
}

oracle_graph *oracle_build(const uint64_t *packed, const uint64_t *offsets, uint64_t n_reads, int k, int threads) {
    uint64_t *ck = nullptr; uint32_t *cc = nullptr;
    uint64_t n = oracle_count_canonical(packed, offsets, n_reads, k, threads, &ck, &cc);
    const int E = k + 1;
    vector<std::pair<uint64_t, uint16_t>> edges;
    edges.reserve(2 * n);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t a = ck[i], b = lsb_rc(a, E);
        if (a == b) {
            edges.push_back({boss_key(a, k), (uint16_t)std::min<uint64_t>(2ULL * cc[i], 65535)});
        } else {
            uint16_t m = (uint16_t)std::min<uint64_t>(cc[i], 65535);
            edges.push_back({boss_key(a, k), m});
            edges.push_back({boss_key(b, k), m});
        }
    }
    free(ck); free(cc);
    __gnu_parallel::sort(edges.begin(), edges.end());
    oracle_graph *g = new oracle_graph;
    g->g.k = k;
    g->g.key.resize(edges.size());
    g->g.mult.resize(edges.size());
    for (size_t i = 0; i < edges.size(); ++i) { g->g.key[i] = edges[i].first; g->g.mult[i] = edges[i].second; }
    g->g.valid.assign(edges.size(), 1);
    return g;
}

oracle_graph *oracle_graph_from_arrays(const uint64_t *keys, const uint16_t *mult, uint64_t n, int k) {
    oracle_graph *g = new oracle_graph;
    g->g.k = k;
    g->g.key.assign(keys, keys + n);
    g->g.mult.assign(mult, mult + n);
    g->g.valid.assign(n, 1);
    return g;
}
void oracle_graph_free(oracle_graph *g) { delete g; }
uint64_t oracle_graph_size(const oracle_graph *g) { return g->g.size(); }
int oracle_graph_k(const oracle_graph *g) { return g->g.k; }
void oracle_graph_arrays(const oracle_graph *g, uint64_t *keys, uint16_t *mult) {
    if (keys) memcpy(keys, g->g.key.data(), 8 * g->g.size());
    if (mult) memcpy(mult, g->g.mult.data(), 2 * g->g.size());
}
void oracle_graph_valid(const oracle_graph *g, uint8_t *valid) { memcpy(valid, g->g.valid.data(), g->g.size()); }
void oracle_graph_set_valid(oracle_graph *g, const uint8_t *valid) {
    for (uint64_t i = 0; i < g->g.size(); ++i) g->g.valid[i] = valid[i] ? 1 : 0;
}
int oracle_outgoing(const oracle_graph *g, uint64_t e, uint64_t *out) { return g->g.OutgoingEdges(e, out); }
int oracle_incoming(const oracle_graph *g, uint64_t e, uint64_t *in) { return g->g.IncomingEdges(e, in); }
int oracle_get_label(const oracle_graph *g, uint64_t e, uint8_t *seq) { return g->g.GetLabel(e, seq); }
int64_t oracle_index_binary_search(const oracle_graph *g, const uint8_t *seq) { return g->g.IndexBinarySearch(seq); }

uint64_t oracle_collect_tips(const oracle_graph *g, uint8_t *tip_flags) {
    uint64_t n = 0;
    for (uint64_t e = 0; e < g->g.size(); ++e) {
        uint8_t t = (g->g.EdgeOutdegree(e) == 0 && g->g.IsValidEdge(e)) ? 1 : 0;
        if (tip_flags) tip_flags[e] = t;
        n += t;
    }
    return n;
}
uint64_t oracle_invalidate_mult_one(oracle_graph *g) {
    oracle_cf_params p{20, 1, 77, 27, 1, 500, 10000000};
    CycleFinderO cf(g->g, p);
    return cf.InvalidateMultiplicityOneNodes();
}
void oracle_recursive_reduction(oracle_graph *g, const uint8_t *tip_flags) {
    oracle_cf_params p{20, 1, 77, 27, 1, 500, 10000000};
    CycleFinderO cf(g->g, p);
    for (uint64_t e = 0; e < g->g.size(); ++e)
        if (tip_flags[e]) cf.RecursiveReduction(e);
}
int oracle_depth_level_search(const oracle_graph *g, uint64_t start, int limit) {
    oracle_cf_params p{20, 1, limit, 27, 1, 500, 10000000};
    CycleFinderO cf(const_cast<Graph &>(g->g), p);
    return cf.DepthLevelSearch(start, start, limit) ? 1 : 0;
}

oracle_cf_result *oracle_cycle_finder(oracle_graph *g, const oracle_cf_params *p) {
    oracle_cf_params q = *p;
    if (q.threads < 1) q.threads = 1;
    CycleFinderO cf(g->g, q);
    cf.Run();
    oracle_cf_result *r = new oracle_cf_result;
    memcpy(r->stats, cf.stats, sizeof(r->stats));
    r->cyc_begin.push_back(0);
    r->node_begin.push_back(0);
    std::unordered_map<uint64_t, size_t> index_of;
    for (size_t i = 0; i < cf.committed.size(); ++i) {
        auto &e = cf.committed[i];
        r->starts.push_back(e.first);
        index_of[e.first] = i;
        for (auto &c : e.second) {
            r->nodes.insert(r->nodes.end(), c.begin(), c.end());
            r->node_begin.push_back(r->nodes.size());
        }
        r->cyc_begin.push_back(r->node_begin.size() - 1);
    }
    for (auto &kv : cf.results) r->map_order.push_back(index_of[kv.first]);
    r->cand_ids = cf.cand_ids;
    r->cand_bucket = cf.cand_bucket;
    return r;
}
uint64_t oracle_cf_n_entries(const oracle_cf_result *r) { return r->starts.size(); }
void oracle_cf_entries(const oracle_cf_result *r, uint64_t *starts, uint64_t *cyc_begin) {
    memcpy(starts, r->starts.data(), 8 * r->starts.size());
    memcpy(cyc_begin, r->cyc_begin.data(), 8 * r->cyc_begin.size());
}
uint64_t oracle_cf_n_cycles(const oracle_cf_result *r) { return r->node_begin.size() - 1; }
uint64_t oracle_cf_n_nodes(const oracle_cf_result *r) { return r->nodes.size(); }
void oracle_cf_cycles(const oracle_cf_result *r, uint64_t *node_begin, uint64_t *nodes) {
    memcpy(node_begin, r->node_begin.data(), 8 * r->node_begin.size());
    if (!r->nodes.empty()) memcpy(nodes, r->nodes.data(), 8 * r->nodes.size());
}
void oracle_cf_map_order(const oracle_cf_result *r, uint64_t *order) {
    if (!r->map_order.empty()) memcpy(order, r->map_order.data(), 8 * r->map_order.size());
}
void oracle_cf_stats(const oracle_cf_result *r, uint64_t *stats) { memcpy(stats, r->stats, sizeof(r->stats)); }
uint64_t oracle_cf_n_candidates(const oracle_cf_result *r) { return r->cand_ids.size(); }
void oracle_cf_candidates(const oracle_cf_result *r, uint64_t *ids, int32_t *bucket) {
    if (!r->cand_ids.empty()) {
        memcpy(ids, r->cand_ids.data(), 8 * r->cand_ids.size());
        memcpy(bucket, r->cand_bucket.data(), 4 * r->cand_bucket.size());
    }
}
void oracle_cf_free(oracle_cf_result *r) { delete r; }
void oracle_free(void *p) { free(p); }

void oracle_reverse_pair_ends(char *s) {
    std::string t(s);
    reverse_pair_ends_sequence(t);
    memcpy(s, t.data(), t.size());
}

// reads.cpp:88-130: seqs[0..n_file1) from the first file, the rest from the second
uint64_t oracle_get_reads(const oracle_graph *g, const char *const *seqs, uint64_t n_seqs, uint64_t n_file1,
                          const uint64_t *cycle_nodes, uint64_t n_nodes, uint64_t **flat, uint64_t **offsets) {
    std::unordered_set<uint64_t> nodes_of_cycles(cycle_nodes, cycle_nodes + n_nodes);
    std::vector<uint64_t> f, o{0};
    for (uint64_t i = 0; i < n_seqs; ++i) {
        std::string seq(seqs[i]);
        if (i >= n_file1) reverse_pair_ends_sequence(seq);
        auto read = get_read_from_sequence(g->g, nodes_of_cycles, seq);
        if (read.empty()) continue;
        f.insert(f.end(), read.begin(), read.end());
        o.push_back(f.size());
    }
    *flat = (uint64_t *)malloc(8 * (f.size() + 1));
    *offsets = (uint64_t *)malloc(8 * o.size());
    memcpy(*flat, f.data(), 8 * f.size());
    memcpy(*offsets, o.data(), 8 * o.size());
    return o.size() - 1;
}

}  // extern "C"
