// array_order.cpp — spacer ordering (reference src/spacer_ordering.cpp): split the graph into
// CRISPR regions, pick the cycles of each region, derive order constraints from the relevant
// reads and topologically sort the cycles.
//
// Wherever the reference's result depends on a libstdc++ unordered container's iteration
// order (node_to_cycle_map, the weighted constraint map, ...), the same container type is
// filled by the same sequence of operations, so the order — and every tie it decides — is the
// reference's. Elsewhere the restatement is free: the k-hop region growth is a frontier BFS
// over batched (device) neighbour queries, Tarjan's recursion is an explicit stack, and
// the invalidation of everything outside the regions is one bitmap AND.
#include <algorithm>
#include <chrono>
#include <functional>
#include <iomanip>
#include <iostream>
#include <numeric>

#include "downstream.h"

namespace {

// Tarjan's SCC from `root` (spacer_ordering.cpp:3-51) with an explicit frame stack visiting
// successors in OutgoingEdges order, exactly as the recursion does. The nodes it can reach are
// the valid ones, taken as a dense graph (SDBG::ValidSubgraph: positions in the ascending list
// of valid ids, out-neighbours as positions), so index / low / on-stack are arrays and a step
// reads no hash table.
struct Tarjan {
    const std::vector<uint32_t> &nbr;  // 4 per node
    const std::vector<uint8_t> &cnt;
    std::vector<int> index, low;       // -1: not visited
    std::vector<char> on_stack;
    std::vector<uint32_t> stack;
    std::vector<std::vector<uint32_t>> components;  // positions
    int counter = 0;
    Tarjan(const std::vector<uint32_t> &nb, const std::vector<uint8_t> &c)
        : nbr(nb), cnt(c), index(c.size(), -1), low(c.size(), 0), on_stack(c.size(), 0) {}

    struct Frame {
        uint32_t v;
        int n, next;
    };
    void open(std::vector<Frame> &frames, uint32_t v) {
        index[v] = counter;
        low[v] = counter;
        ++counter;
        stack.push_back(v);
        on_stack[v] = 1;
        frames.push_back(Frame{v, (int)cnt[v], 0});
    }
    void run(uint32_t root) {
        std::vector<Frame> frames;
        open(frames, root);
        while (!frames.empty()) {
            Frame &f = frames.back();
            if (f.next < f.n) {
                const uint32_t w = nbr[4 * (size_t)f.v + f.next++];
                if (index[w] < 0) {
                    open(frames, w);  // invalidates f
                } else if (on_stack[w]) {
                    low[f.v] = std::min(low[f.v], index[w]);
                }
                continue;
            }
            const uint32_t v = f.v;
            if (low[v] == index[v]) {
                std::vector<uint32_t> comp;
                uint32_t w;
                do {
                    w = stack.back();
                    stack.pop_back();
                    on_stack[w] = 0;
                    comp.push_back(w);
                } while (w != v);
                if (comp.size() > 1) components.push_back(std::move(comp));
            }
            frames.pop_back();
            if (!frames.empty()) {  // back in the caller: low[parent] = min(low[parent], low[v])
                const uint32_t p = frames.back().v;
                low[p] = std::min(low[p], low[v]);
            }
        }
    }
};

std::vector<uint32_t> merge_runs(const std::vector<uint32_t> &v) {  // A,A,B,C,C -> A,B,C
    std::vector<uint32_t> out;
    for (size_t i = 0; i < v.size(); ++i)
        if (i == 0 || v[i] != out.back()) out.push_back(v[i]);
    return out;
}

}  // namespace

static double g_ids_s = 0, g_scc_s = 0, g_map_s = 0;  // TIMING_REGIONS detail
static uint64_t g_n_ids = 0;
// components as positions in ids (the valid edges, ascending), in the recursion's order
static std::vector<std::vector<uint32_t>> scc_positions(const SDBG &sdbg, std::vector<uint64_t> &ids,
                                                        std::vector<uint32_t> &nbr, std::vector<uint8_t> &cnt) {
    using clk = std::chrono::high_resolution_clock;
    const auto t0 = clk::now();
    sdbg.ValidSubgraph(ids, nbr, cnt);
    const auto t1 = clk::now();
    Tarjan t(nbr, cnt);
    for (uint32_t v = 0; v < ids.size(); ++v)  // valid nodes in ascending id order
        if (t.index[v] < 0) t.run(v);
    g_ids_s = std::chrono::duration<double>(t1 - t0).count();
    g_scc_s = std::chrono::duration<double>(clk::now() - t1).count();
    g_n_ids = ids.size();
    return std::move(t.components);
}

std::vector<std::vector<uint64_t>> find_strongly_connected_components(const SDBG &sdbg) {
    std::vector<uint64_t> ids;
    std::vector<uint32_t> nbr;
    std::vector<uint8_t> cnt;
    std::vector<std::vector<uint64_t>> out;
    for (const auto &c : scc_positions(sdbg, ids, nbr, cnt)) {
        out.emplace_back();
        for (uint32_t v : c) out.back().push_back(ids[v]);
    }
    return out;
}

// spacer_ordering.cpp:78-138: the cycle nodes grown by k hops over valid in- and out-edges
// (the reference's k rounds over the whole set reach exactly the k-hop neighbourhood), then
// every valid edge outside that set is invalidated.
void keep_crispr_regions_extended_by_k(SDBG &sdbg, const size_t &k, const std::vector<std::vector<uint64_t>> &cycles) {
    if (sdbg.device()) {  // the whole growth and the AND on the GPU, one call
        std::vector<uint64_t> seeds;
        for (const auto &cycle : cycles) seeds.insert(seeds.end(), cycle.begin(), cycle.end());
        using clk = std::chrono::high_resolution_clock;
        const auto a = clk::now();
        sdbg.KeepRegion(seeds, k);
        const auto b = clk::now();
        const std::vector<uint64_t> live = sdbg.ValidIds();
        const auto c = clk::now();
        sdbg.PrefetchOutgoing(live);
        sdbg.PrefetchKeys(live);
        std::cout << "TIMING_GROW keep_s=" << std::chrono::duration<double>(b - a).count()
                  << " ids_s=" << std::chrono::duration<double>(c - b).count()
                  << " prefetch_s=" << std::chrono::duration<double>(clk::now() - c).count() << " live=" << live.size()
                  << std::endl;
        return;
    }
    IdMap<char> region;  // membership (the order of `keep` does not matter: one bitmap AND)
    std::vector<uint64_t> keep;
    auto insert = [&](uint64_t e) {
        char &c = region[e];
        if (c) return false;
        c = 1;
        keep.push_back(e);
        return true;
    };
    std::vector<uint64_t> frontier;
    for (const auto &cycle : cycles)
        for (uint64_t e : cycle)
            if (insert(e)) frontier.push_back(e);
    std::vector<uint64_t> nb;
    std::vector<int32_t> cnt;
    for (size_t hop = 0; hop < k && !frontier.empty(); ++hop) {
        std::vector<uint64_t> expand;
        for (uint64_t e : frontier)
            if (sdbg.IsValidEdge(e)) expand.push_back(e);
        std::vector<uint64_t> next;
        for (int dir = 0; dir < 2; ++dir) {
            sdbg.NeighborsBatch(expand, dir == 0, nb, cnt);
            for (size_t i = 0; i < expand.size(); ++i)
                for (int j = 0; j < cnt[i]; ++j)
                    if (insert(nb[4 * i + j])) next.push_back(nb[4 * i + j]);
        }
        frontier.swap(next);
    }
    sdbg.KeepOnly(keep);
    // every node the SCC split and the subgraphs query from here on is one of these: their
    // out-neighbours (valid-only, after the AND) and labels in two device calls
    std::vector<uint64_t> live;
    for (uint64_t e : keep)
        if (sdbg.IsValidEdge(e)) live.push_back(e);
    sdbg.PrefetchOutgoing(live);
    sdbg.PrefetchKeys(live);
}

// spacer_ordering.cpp:140-173: one Graph per SCC, edges inside the component only
std::vector<Graph> divide_graph_into_subgraphs(const SDBG &sdbg) {
    std::vector<Graph> subgraphs;
    std::vector<uint64_t> ids;
    std::vector<uint32_t> nbr;
    std::vector<uint8_t> cnt;
    const auto comps = scc_positions(sdbg, ids, nbr, cnt);
    const auto t0 = std::chrono::high_resolution_clock::now();
    std::vector<uint32_t> comp_of(ids.size(), 0);  // component + 1 by position (components are disjoint)
    for (uint32_t ci = 0; ci < comps.size(); ++ci)
        for (uint32_t v : comps[ci]) comp_of[v] = ci + 1;
    g_map_s = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count();
    for (uint32_t ci = 0; ci < comps.size(); ++ci) {
        const auto &comp = comps[ci];
        Graph sub;
        sub.nodes.reserve(comp.size());
        sub.adjacency_list.reserve(comp.size());
        for (uint32_t v : comp)  // every node of a component is valid; its out-edges in OutgoingEdges order
            for (int j = 0; j < cnt[v]; ++j) {
                const uint32_t w = nbr[4 * (size_t)v + j];
                if (comp_of[w] == ci + 1) sub.add_edge(ids[v], ids[w]);
            }
        if (!sub.nodes.empty()) subgraphs.push_back(std::move(sub));
    }
    return subgraphs;
}

std::vector<Graph> get_crispr_regions_extended_by_k(SDBG &sdbg, const size_t &k,
                                                    const std::vector<std::vector<uint64_t>> &cycles) {
    using clk = std::chrono::high_resolution_clock;
    const auto t0 = clk::now();
    keep_crispr_regions_extended_by_k(sdbg, k, cycles);
    const auto t1 = clk::now();
    auto out = divide_graph_into_subgraphs(sdbg);
    std::cout << "TIMING_REGIONS grow_s=" << std::chrono::duration<double>(t1 - t0).count()
              << " divide_s=" << std::chrono::duration<double>(clk::now() - t1).count() << " ids_s=" << g_ids_s
              << " scc_s=" << g_scc_s << " map_s=" << g_map_s << " n_ids=" << g_n_ids << std::endl;
    return out;
}

// spacer_ordering.cpp:184-198: reads starting or ending inside the region
std::vector<std::vector<uint64_t>> get_relevant_reads(const Graph &graph,
                                                      const std::vector<std::vector<uint64_t>> &all_reads) {
    std::vector<std::vector<uint64_t>> kept;
    for (const auto &r : all_reads)
        if (graph.nodes.count(r.at(0)) || graph.nodes.count(r.at(r.size() - 1))) kept.push_back(r);
    return kept;
}

// spacer_ordering.cpp:200-221: cycles lying entirely inside the region
std::vector<std::vector<uint64_t>> get_relevant_cycles(const Graph &graph,
                                                       const std::vector<std::vector<uint64_t>> &all_cycles) {
    std::vector<std::vector<uint64_t>> kept;
    for (const auto &c : all_cycles)
        if (std::all_of(c.begin(), c.end(), [&](uint64_t x) { return graph.nodes.count(x) > 0; })) kept.push_back(c);
    return kept;
}

// Both of the above for every region in one pass over the reads and one over the cycles. The
// regions are strongly connected components, so a node lies in at most one of them: a read
// can only be relevant to the regions holding its first or its last node, and a cycle only to
// the region holding its first node. Per region the lists are the same, in the same order, as
// get_relevant_reads / get_relevant_cycles give (800 regions x 367K reads at C3: 27 s -> <1 s).
void get_relevant_reads_and_cycles(const std::vector<Graph> &regions, const std::vector<std::vector<uint64_t>> &all_reads,
                                   const std::vector<std::vector<uint64_t>> &all_cycles, std::vector<ReadRefs> &reads_out,
                                   std::vector<std::vector<std::vector<uint64_t>>> &cycles_out) {
    IdMap<uint32_t> region_of;  // region + 1 (regions are disjoint SCCs)
    size_t total = 0;
    for (const auto &r : regions) total += r.nodes.size();
    region_of.reserve(total);
    for (uint32_t i = 0; i < regions.size(); ++i)
        for (uint64_t x : regions[i].nodes) {
            uint32_t &v = region_of[x];
            if (!v) v = i + 1;
        }
    reads_out.assign(regions.size(), {});
    cycles_out.assign(regions.size(), {});
    auto find = [&](uint64_t x) {
        const uint32_t *v = region_of.find(x);
        return v ? *v - 1 : UINT32_MAX;
    };
    for (const auto &r : all_reads) {
        const uint32_t a = find(r.at(0)), b = find(r.at(r.size() - 1));
        if (a != UINT32_MAX) reads_out[a].push_back(&r);
        if (b != UINT32_MAX && b != a) reads_out[b].push_back(&r);
    }
    for (const auto &c : all_cycles) {
        if (c.empty()) {  // vacuously inside every region
            for (auto &v : cycles_out) v.push_back(c);
            continue;
        }
        const uint32_t a = find(c[0]);
        if (a != UINT32_MAX && std::all_of(c.begin(), c.end(), [&](uint64_t x) { return find(x) == a; }))
            cycles_out[a].push_back(c);
    }
}

// spacer_ordering.cpp:223-263: drop the cycles a minimum set cover does not need. The
// reference's removal loop compares the ORIGINAL kept indices against positions in the
// shrinking vector (its bound and index both use the current size); that exact walk is
// restated here, because it decides which cycles survive when the cover drops some.
void get_minimum_cycles_for_full_coverage(std::vector<std::vector<uint64_t>> &cycles, std::ostream &log) {
    if (cycles.empty()) return;
    std::unordered_map<uint64_t, uint32_t> dense;
    uint32_t next_id = 0;
    std::unordered_set<uint32_t> universe;
    std::vector<std::vector<uint32_t>> sets;
    for (const auto &c : cycles) {
        std::vector<uint32_t> s;
        for (uint64_t x : c) {
            auto it = dense.find(x);
            uint32_t id;
            if (it != dense.end()) {
                id = it->second;
            } else {
                id = next_id++;
                dense.emplace(x, id);
            }
            s.push_back(id);
            universe.insert(id);
        }
        sets.push_back(std::move(s));
    }
    if (universe.empty() || sets.empty()) return;
    const std::vector<size_t> kept = solve_min_cover_problem(universe, sets, log);
    const std::unordered_set<size_t> keep(kept.begin(), kept.end());
    for (size_t i = 0; i < cycles.size(); ++i) {
        const size_t pos = cycles.size() - 1 - i;
        if (keep.count(pos)) continue;
        cycles.erase(cycles.begin() + pos);
    }
}

// spacer_ordering.cpp:265-313. The reference calls cft (Caprara-Fischetti-Toth set-covering
// heuristic, third-party, absent here, 10 s time limit). This is an exact minimum set cover
// with deterministic tie-breaking: mandatory sets (sole cover of an element), dominated sets
// dropped, then branch and bound on the element with the fewest covering sets (lowest set
// index first), bounded by a node budget after which the best cover found (greedy seed) is
// kept. The returned indices are ascending; callers only use them as a set.
std::vector<size_t> solve_min_cover_problem(const std::unordered_set<uint32_t> &universe,
                                            const std::vector<std::vector<uint32_t>> &sets, std::ostream &log) {
    if (universe.empty() || sets.empty()) {
        log << "Error: Unable to find min cover as the universe or sets are empty" << std::endl;
        return {};
    }
    const size_t n = universe.size();
    for (uint32_t x : universe)
        if (x >= n) {
            log << "Error: Unable to find min cover as the universe elements are invalid" << std::endl;
            return {};
        }
    for (const auto &s : sets)
        for (uint32_t x : s)
            if (x >= n) {
                log << "Error: Unable to find min cover as the sets elements are invalid" << std::endl;
                return {};
            }
    // element -> covering sets (ascending, deduplicated)
    std::vector<std::vector<uint32_t>> covers(n);
    std::vector<std::vector<uint32_t>> S(sets.size());
    for (uint32_t i = 0; i < sets.size(); ++i) {
        S[i] = sets[i];
        std::sort(S[i].begin(), S[i].end());
        S[i].erase(std::unique(S[i].begin(), S[i].end()), S[i].end());
        for (uint32_t x : S[i]) covers[x].push_back(i);
    }
    for (uint32_t x = 0; x < n; ++x)
        if (covers[x].empty()) return {};  // infeasible
    std::vector<char> chosen(sets.size(), 0), covered(n, 0);
    auto take = [&](uint32_t i) {
        chosen[i] = 1;
        for (uint32_t x : S[i]) covered[x] = 1;
    };
    for (uint32_t x = 0; x < n; ++x)
        if (covers[x].size() == 1) take(covers[x][0]);
    std::vector<uint32_t> rest;
    for (uint32_t x = 0; x < n; ++x)
        if (!covered[x]) rest.push_back(x);
    std::vector<size_t> result;
    if (!rest.empty()) {
        // candidate sets restricted to the uncovered elements; drop empty and dominated ones
        std::vector<std::vector<uint32_t>> R(sets.size());
        std::vector<uint32_t> cand;
        for (uint32_t i = 0; i < sets.size(); ++i) {
            if (chosen[i]) continue;
            for (uint32_t x : S[i])
                if (!covered[x]) R[i].push_back(x);
            if (!R[i].empty()) cand.push_back(i);
        }
        std::vector<uint32_t> live;
        for (uint32_t i : cand) {
            bool dominated = false;
            for (uint32_t j : cand) {
                if (j == i || R[j].size() < R[i].size()) continue;
                if (R[j].size() == R[i].size() && j > i) continue;  // equal sets: keep the lower index
                if (std::includes(R[j].begin(), R[j].end(), R[i].begin(), R[i].end())) { dominated = true; break; }
            }
            if (!dominated) live.push_back(i);
        }
        std::vector<std::vector<uint32_t>> cov(n);
        size_t max_size = 1;
        for (uint32_t i : live) {
            for (uint32_t x : R[i]) cov[x].push_back(i);
            max_size = std::max(max_size, R[i].size());
        }
        // greedy seed: most new elements, lowest index on ties
        std::vector<uint32_t> best;
        {
            std::vector<char> c(covered);
            size_t left = rest.size();
            while (left) {
                uint32_t bi = 0;
                size_t bg = 0;
                for (uint32_t i : live) {
                    size_t gain = 0;
                    for (uint32_t x : R[i]) gain += !c[x];
                    if (gain > bg) { bg = gain; bi = i; }
                }
                best.push_back(bi);
                for (uint32_t x : R[bi]) if (!c[x]) { c[x] = 1; --left; }
            }
        }
        // branch and bound
        std::vector<uint32_t> cur;
        std::vector<int> cnt(n, 0);  // how many chosen sets cover x (beyond the mandatory ones)
        size_t uncovered = rest.size();
        long budget = 2000000;
        std::function<void()> dfs = [&]() {
            if (--budget < 0) return;
            if (uncovered == 0) {
                if (cur.size() < best.size()) best = cur;
                return;
            }
            if (cur.size() + (uncovered + max_size - 1) / max_size >= best.size()) return;
            uint32_t pick = 0;
            size_t fewest = SIZE_MAX;
            for (uint32_t x : rest)
                if (!covered[x] && cnt[x] == 0 && cov[x].size() < fewest) { fewest = cov[x].size(); pick = x; }
            for (uint32_t i : cov[pick]) {
                cur.push_back(i);
                for (uint32_t x : R[i]) if (cnt[x]++ == 0) --uncovered;
                dfs();
                for (uint32_t x : R[i]) if (--cnt[x] == 0) ++uncovered;
                cur.pop_back();
            }
        };
        dfs();
        for (uint32_t i : best) chosen[i] = 1;
    }
    for (size_t i = 0; i < sets.size(); ++i)
        if (chosen[i]) result.push_back(i);
    return result;
}

// spacer_ordering.cpp:315-340: node -> index of the only cycle containing it
std::unordered_map<uint64_t, uint32_t> get_node_to_unique_cycle_map(const std::vector<std::vector<uint64_t>> &cycles) {
    std::vector<std::unordered_set<uint64_t>> node_sets;
    for (const auto &c : cycles) node_sets.emplace_back(c.begin(), c.end());
    std::unordered_map<uint64_t, uint64_t> owners;  // node -> number of cycles holding it
    for (const auto &s : node_sets)
        for (uint64_t x : s) ++owners[x];
    std::unordered_map<uint64_t, uint32_t> unique;
    for (uint32_t i = 0; i < node_sets.size(); ++i)
        for (const uint64_t x : node_sets[i])  // the reference's insertion order
            if (owners[x] == 1) unique[x] = i;
    return unique;
}

std::vector<uint32_t> get_all_cycle_indices(const std::unordered_map<uint64_t, uint32_t> &node_to_cycle_map) {
    std::vector<uint32_t> idx;  // first-seen order over the map (spacer_ordering.cpp:342-354)
    for (const auto &kv : node_to_cycle_map)
        if (std::find(idx.begin(), idx.end(), kv.second) == idx.end()) idx.push_back(kv.second);
    return idx;
}

std::vector<std::tuple<uint32_t, uint32_t>> every_possible_combination(const std::vector<uint32_t> &v) {
    std::vector<std::tuple<uint32_t, uint32_t>> pairs;  // spacer_ordering.cpp:356-372
    for (size_t i = 0; i < v.size(); ++i)
        for (size_t j = i + 1; j < v.size(); ++j)
            if (v[i] != v[j]) pairs.emplace_back(v[i], v[j]);
    return pairs;
}

// spacer_ordering.cpp:374-412: every ordered pair of the cycles the read passes through (the
// reference computes the merged run list but returns the pairs over the unmerged sequence)
std::vector<std::tuple<uint32_t, uint32_t>> generate_constraints_from_read(
    const Graph &, const std::vector<uint64_t> &read, const std::unordered_map<uint64_t, uint32_t> &node_to_cycle_map) {
    std::vector<uint32_t> seq;
    for (uint64_t x : read) {
        auto it = node_to_cycle_map.find(x);
        if (it != node_to_cycle_map.end()) seq.push_back(it->second);
    }
    return every_possible_combination(seq);
}

// spacer_ordering.cpp:414-458: a read starting and ending in cycles constrains its first run
// (which may be "outside every cycle") against the next one
std::vector<std::tuple<uint32_t, uint32_t>> generate_out_of_cycles_constraints_from_read(
    const Graph &, const std::vector<uint64_t> &read, const std::unordered_map<uint64_t, uint32_t> &node_to_cycle_map) {
    if (!node_to_cycle_map.count(read.at(0)) || !node_to_cycle_map.count(read.at(read.size() - 1))) return {};
    std::vector<uint32_t> seq;
    for (uint64_t x : read) {
        auto it = node_to_cycle_map.find(x);
        seq.push_back(it == node_to_cycle_map.end() ? NOT_IN_ANY_CYCLE_INDEX : it->second);
    }
    const std::vector<uint32_t> runs = merge_runs(seq);
    if (runs.size() > 1) return {std::make_tuple(runs[0], runs[1])};
    return {};
}

std::vector<std::tuple<uint32_t, uint32_t>> generate_constraints(
    const Graph &graph, const std::vector<std::vector<uint64_t>> &reads,
    const std::unordered_map<uint64_t, uint32_t> &node_to_cycle_map) {  // spacer_ordering.cpp:460-486
    std::vector<std::tuple<uint32_t, uint32_t>> all;
    for (const auto &r : reads) {
        for (const auto &c : generate_constraints_from_read(graph, r, node_to_cycle_map)) all.push_back(c);
        for (const auto &c : generate_out_of_cycles_constraints_from_read(graph, r, node_to_cycle_map)) all.push_back(c);
    }
    return all;
}

// spacer_ordering.cpp:488-544: Kruskal on the constraint multigraph, heaviest edge first
// (ties: larger tuple first), union by rank with path compression
std::vector<std::tuple<uint32_t, uint32_t>> get_maximal_spanning_tree(
    const std::vector<std::tuple<uint32_t, uint32_t>> &edges) {
    std::unordered_map<uint32_t, uint32_t> parent;
    std::unordered_map<uint32_t, int> rank;
    std::function<uint32_t(uint32_t)> root = [&](uint32_t x) -> uint32_t {
        if (!parent.count(x)) {
            parent[x] = x;
            rank[x] = 0;
        }
        if (parent[x] != x) parent[x] = root(parent[x]);
        return parent[x];
    };
    std::unordered_map<std::tuple<uint32_t, uint32_t>, int, TupleHash> weight;
    for (const auto &e : edges) weight[e]++;
    std::vector<std::pair<int, std::tuple<uint32_t, uint32_t>>> order;
    for (const auto &kv : weight) order.push_back({kv.second, kv.first});
    std::sort(order.begin(), order.end(), std::greater<std::pair<int, std::tuple<uint32_t, uint32_t>>>());
    std::vector<std::tuple<uint32_t, uint32_t>> tree;
    for (const auto &we : order) {
        const uint32_t a = root(std::get<0>(we.second)), b = root(std::get<1>(we.second));
        if (a == b) continue;
        if (rank[a] < rank[b]) parent[a] = b;
        else if (rank[a] > rank[b]) parent[b] = a;
        else {
            parent[b] = a;
            rank[a]++;
        }
        tree.push_back(we.second);
    }
    return tree;
}

// spacer_ordering.cpp:546-567: constraints off the spanning tree are dropped (each costs its
// target one heuristic point unless it involves "outside every cycle")
void resolve_cycles_greedy(std::vector<std::tuple<uint32_t, uint32_t>> &constraints,
                           std::unordered_map<uint32_t, int> &heuristic_node_values) {
    const auto tree = get_maximal_spanning_tree(constraints);
    const std::unordered_set<std::tuple<uint32_t, uint32_t>, TupleHash> in_tree(tree.begin(), tree.end());
    std::vector<std::tuple<uint32_t, uint32_t>> kept;
    for (const auto &c : constraints) {
        const uint32_t from = std::get<0>(c), to = std::get<1>(c);
        if (!in_tree.count(c) && from != NOT_IN_ANY_CYCLE_INDEX && to != NOT_IN_ANY_CYCLE_INDEX)
            heuristic_node_values[to] -= 1;
        else
            kept.push_back(c);
    }
    constraints = std::move(kept);
}

// spacer_ordering.cpp:569-646 (tail recursion as a loop): repeatedly emit the start node with
// the best affection + heuristic score (last one on ties), remove its out-edges crediting
// their targets, and promote targets left without incoming edges
static void apply_topological_sort(std::vector<uint32_t> &starts, const std::unordered_map<uint32_t, int> &affection,
                                   std::unordered_map<uint32_t, int> &heuristic,
                                   std::unordered_map<std::tuple<uint32_t, uint32_t>, int, TupleHash> &edges,
                                   std::vector<uint32_t> &order, float &confidence) {
    while (!starts.empty()) {
        int best = 0;
        float best_value = std::numeric_limits<float>::lowest();
        float abs_sum = 0.0;
        for (size_t i = 0; i < starts.size(); ++i) {
            const float a = static_cast<float>(affection.at(starts[i]));
            const float h = static_cast<float>(heuristic.at(starts[i]));
            const float value = a * 1.0 + h;  // evaluated in double, stored as float (as the reference)
            if (value >= best_value) {
                best_value = value;
                best = (int)i;
            }
            abs_sum += std::abs(value);
        }
        confidence += (std::abs(best_value) / abs_sum);
        const uint32_t s = starts[best];
        order.push_back(s);
        starts.erase(starts.begin() + best);
        std::vector<uint32_t> released;
        std::vector<std::tuple<uint32_t, uint32_t>> gone;
        for (const auto &kv : edges) {
            if (std::get<0>(kv.first) != s) continue;
            released.push_back(std::get<1>(kv.first));
            heuristic[std::get<1>(kv.first)] += kv.second;
            gone.push_back(kv.first);
        }
        for (const auto &e : gone) edges.erase(e);
        for (uint32_t t : released) {
            bool incoming = false;
            for (const auto &kv : edges)
                if (std::get<1>(kv.first) == t) { incoming = true; break; }
            if (!incoming) starts.push_back(t);
        }
    }
}

std::vector<uint32_t> solve_constraints_with_topological_sort(
    const std::vector<std::tuple<uint32_t, uint32_t>> &constraints, std::unordered_map<uint32_t, int> &heuristic_node_values,
    const std::vector<uint32_t> &nodes, float &confidence) {  // spacer_ordering.cpp:648-717
    std::unordered_map<std::tuple<uint32_t, uint32_t>, int, TupleHash> edges;
    for (const auto &c : constraints)
        if (std::get<0>(c) != NOT_IN_ANY_CYCLE_INDEX && std::get<1>(c) != NOT_IN_ANY_CYCLE_INDEX) edges[c]++;
    std::vector<uint32_t> starts;
    for (uint32_t v : nodes) {
        const bool has_in = std::any_of(constraints.begin(), constraints.end(), [&](const auto &c) {
            return std::get<0>(c) != NOT_IN_ANY_CYCLE_INDEX && std::get<1>(c) == v;
        });
        if (!has_in) starts.push_back(v);
    }
    // affection: +1 per read entering the cycle from outside, -1 per read leaving to outside
    std::unordered_map<uint32_t, int> affection;
    for (uint32_t v : nodes) affection[v] = 0;
    for (const auto &c : constraints) {
        const uint32_t a = std::get<0>(c), b = std::get<1>(c);
        if (a != NOT_IN_ANY_CYCLE_INDEX && b != NOT_IN_ANY_CYCLE_INDEX) continue;
        if (a == NOT_IN_ANY_CYCLE_INDEX) affection[b]++;
        else affection[a]--;
    }
    std::vector<uint32_t> order;
    confidence = 0.0;
    apply_topological_sort(starts, affection, heuristic_node_values, edges, order, confidence);
    confidence /= order.size();
    return order;
}

// ---- the same constraints as (distinct pair, multiplicity) in first-occurrence order --------
// Everything downstream of generate_constraints depends on the constraint list only through
// (a) each distinct pair's multiplicity (Kruskal's weights, heuristic penalties, affection,
// topological edge weights, the confidence ratio) and (b) the order in which distinct pairs
// first occur (the insertion order of the topological sort's unordered_map, whose iteration
// order decides ties; re-inserting a present key changes nothing). A read's pairs are
// every_possible_combination of its cycle-index sequence: with the sequence as runs (value a_p,
// length c_p), pair (a_p, a_q), p < q, a_p != a_q, occurs c_p * c_q times and the pairs first
// occur in (p, q) order — O(runs^2) per read instead of O(nodes^2) (C3: 800 regions x ~460
// reads x ~120 nodes; step 7 of the CLI 15.5 s). MCAAT_ORDER_REF=1 runs the list form.
struct WeightedConstraints {
    std::vector<std::tuple<uint32_t, uint32_t>> pair;
    std::vector<int64_t> weight;
    std::unordered_map<std::tuple<uint32_t, uint32_t>, uint32_t, TupleHash> index;
    void add(std::tuple<uint32_t, uint32_t> t, int64_t w) {
        auto it = index.find(t);
        if (it == index.end()) {
            index.emplace(t, (uint32_t)pair.size());
            pair.push_back(t);
            weight.push_back(w);
        } else {
            weight[it->second] += w;
        }
    }
    int64_t total() const {
        int64_t n = 0;
        for (int64_t w : weight) n += w;
        return n;
    }
};

static WeightedConstraints generate_constraints_weighted(const ReadRefs &reads,
                                                         const std::unordered_map<uint64_t, uint32_t> &node_to_cycle_map) {
    WeightedConstraints wc;
    // the map's lookups (every node of every read) from a flat copy: the unordered_map itself
    // only matters for its iteration order (get_all_cycle_indices)
    IdMap<uint32_t> n2c;
    n2c.reserve(node_to_cycle_map.size());
    for (const auto &kv : node_to_cycle_map) n2c[kv.first] = kv.second;
    std::vector<uint32_t> seq;                   // cycle index per node, NOT_IN_ANY_CYCLE_INDEX outside
    std::vector<std::pair<uint32_t, int64_t>> runs;  // runs of the in-cycle subsequence
    for (const auto *rp : reads) {
        const auto &r = *rp;
        seq.clear();
        for (uint64_t x : r) {
            const uint32_t *c = n2c.find(x);
            seq.push_back(c ? *c : NOT_IN_ANY_CYCLE_INDEX);
        }
        runs.clear();
        for (uint32_t v : seq) {
            if (v == NOT_IN_ANY_CYCLE_INDEX) continue;
            if (!runs.empty() && runs.back().first == v) ++runs.back().second;
            else runs.push_back({v, 1});
        }
        for (size_t p = 0; p < runs.size(); ++p)
            for (size_t q = p + 1; q < runs.size(); ++q)
                if (runs[p].first != runs[q].first)
                    wc.add(std::make_tuple(runs[p].first, runs[q].first), runs[p].second * runs[q].second);
        // generate_out_of_cycles_constraints_from_read
        if (!seq.empty() && seq.front() != NOT_IN_ANY_CYCLE_INDEX && seq.back() != NOT_IN_ANY_CYCLE_INDEX) {
            const std::vector<uint32_t> m = merge_runs(seq);
            if (m.size() > 1) wc.add(std::make_tuple(m[0], m[1]), 1);
        }
    }
    return wc;
}

static void resolve_cycles_greedy_weighted(WeightedConstraints &wc, std::unordered_map<uint32_t, int> &heuristic) {
    // get_maximal_spanning_tree: weights per distinct pair, heaviest first, ties by larger tuple
    std::vector<std::pair<int64_t, std::tuple<uint32_t, uint32_t>>> order;
    for (size_t i = 0; i < wc.pair.size(); ++i) order.push_back({wc.weight[i], wc.pair[i]});
    std::sort(order.begin(), order.end(), std::greater<std::pair<int64_t, std::tuple<uint32_t, uint32_t>>>());
    std::unordered_map<uint32_t, uint32_t> parent;
    std::unordered_map<uint32_t, int> rank;
    std::function<uint32_t(uint32_t)> root = [&](uint32_t x) -> uint32_t {
        if (!parent.count(x)) {
            parent[x] = x;
            rank[x] = 0;
        }
        if (parent[x] != x) parent[x] = root(parent[x]);
        return parent[x];
    };
    std::unordered_set<std::tuple<uint32_t, uint32_t>, TupleHash> in_tree;
    for (const auto &we : order) {
        const uint32_t a = root(std::get<0>(we.second)), b = root(std::get<1>(we.second));
        if (a == b) continue;
        if (rank[a] < rank[b]) parent[a] = b;
        else if (rank[a] > rank[b]) parent[b] = a;
        else {
            parent[b] = a;
            rank[a]++;
        }
        in_tree.insert(we.second);
    }
    WeightedConstraints kept;
    for (size_t i = 0; i < wc.pair.size(); ++i) {
        const auto &c = wc.pair[i];
        const uint32_t from = std::get<0>(c), to = std::get<1>(c);
        if (!in_tree.count(c) && from != NOT_IN_ANY_CYCLE_INDEX && to != NOT_IN_ANY_CYCLE_INDEX)
            heuristic[to] -= (int)wc.weight[i];
        else
            kept.add(c, wc.weight[i]);
    }
    wc = std::move(kept);
}

static std::vector<uint32_t> solve_topological_weighted(const WeightedConstraints &wc,
                                                        std::unordered_map<uint32_t, int> &heuristic,
                                                        const std::vector<uint32_t> &nodes, float &confidence) {
    std::unordered_map<std::tuple<uint32_t, uint32_t>, int, TupleHash> edges;
    for (size_t i = 0; i < wc.pair.size(); ++i) {  // first-occurrence order, as the list fills it
        const auto &c = wc.pair[i];
        if (std::get<0>(c) != NOT_IN_ANY_CYCLE_INDEX && std::get<1>(c) != NOT_IN_ANY_CYCLE_INDEX)
            edges[c] += (int)wc.weight[i];
    }
    std::unordered_set<uint32_t> has_in;
    for (const auto &c : wc.pair)
        if (std::get<0>(c) != NOT_IN_ANY_CYCLE_INDEX) has_in.insert(std::get<1>(c));
    std::vector<uint32_t> starts;
    for (uint32_t v : nodes)
        if (!has_in.count(v)) starts.push_back(v);
    std::unordered_map<uint32_t, int> affection;
    for (uint32_t v : nodes) affection[v] = 0;
    for (size_t i = 0; i < wc.pair.size(); ++i) {
        const uint32_t a = std::get<0>(wc.pair[i]), b = std::get<1>(wc.pair[i]);
        if (a != NOT_IN_ANY_CYCLE_INDEX && b != NOT_IN_ANY_CYCLE_INDEX) continue;
        if (a == NOT_IN_ANY_CYCLE_INDEX) affection[b] += (int)wc.weight[i];
        else affection[a] -= (int)wc.weight[i];
    }
    std::vector<uint32_t> order;
    confidence = 0.0;
    apply_topological_sort(starts, affection, heuristic, edges, order, confidence);
    confidence /= order.size();
    return order;
}

std::vector<uint32_t> order_cycles(const Graph &graph, const std::vector<std::vector<uint64_t>> &reads,
                                   const std::vector<std::vector<uint64_t>> &cycles, float &confidence_cycle_resolution,
                                   float &confidence_topological_sort, std::ostream &log) {
    ReadRefs refs;
    refs.reserve(reads.size());
    for (const auto &r : reads) refs.push_back(&r);
    return order_cycles(graph, refs, cycles, confidence_cycle_resolution, confidence_topological_sort, log);
}

std::vector<uint32_t> order_cycles(const Graph &graph, const ReadRefs &reads, const std::vector<std::vector<uint64_t>> &cycles,
                                   float &confidence_cycle_resolution, float &confidence_topological_sort,
                                   std::ostream &log) {  // spacer_ordering.cpp:719-754
    const auto node_to_cycle = get_node_to_unique_cycle_map(cycles);
    const auto cycle_ids = get_all_cycle_indices(node_to_cycle);
    const char *ref = getenv("MCAAT_ORDER_REF");
    if (!(ref && ref[0] == '1')) {
        auto wc = generate_constraints_weighted(reads, node_to_cycle);
        const int64_t before = wc.total();
        log << "      ▸ " << before << " constraints derived" << std::endl;
        std::unordered_map<uint32_t, int> heuristic;
        for (uint32_t c : cycle_ids) heuristic[c] = 0;
        resolve_cycles_greedy_weighted(wc, heuristic);
        const int64_t after = wc.total();
        confidence_cycle_resolution = static_cast<float>(after) / static_cast<float>(before);
        log << "      ▸ " << after << " constraints remain after resolving cycles (confidence = " << std::fixed
                  << std::setprecision(2) << (confidence_cycle_resolution * 100) << "%)" << std::endl;
        return solve_topological_weighted(wc, heuristic, cycle_ids, confidence_topological_sort);
    }
    std::vector<std::vector<uint64_t>> copies;  // the list form (MCAAT_ORDER_REF=1) takes the reads themselves
    copies.reserve(reads.size());
    for (const auto *r : reads) copies.push_back(*r);
    auto constraints = generate_constraints(graph, copies, node_to_cycle);
    log << "      ▸ " << constraints.size() << " constraints derived" << std::endl;
    std::unordered_map<uint32_t, int> heuristic;
    for (uint32_t c : cycle_ids) heuristic[c] = 0;
    const int before = constraints.size();
    resolve_cycles_greedy(constraints, heuristic);
    confidence_cycle_resolution = static_cast<float>(constraints.size()) / static_cast<float>(before);
    log << "      ▸ " << constraints.size() << " constraints remain after resolving cycles (confidence = "
              << std::fixed << std::setprecision(2) << (confidence_cycle_resolution * 100) << "%)" << std::endl;
    return solve_constraints_with_topological_sort(constraints, heuristic, cycle_ids, confidence_topological_sort);
}

std::vector<std::vector<uint64_t>> get_ordered_cycles(const std::vector<uint32_t> &cycle_order,
                                                      const std::vector<std::vector<uint64_t>> &cycles) {
    std::vector<std::vector<uint64_t>> out;  // spacer_ordering.cpp:756-770
    for (uint32_t i : cycle_order)
        if (i < cycles.size()) out.push_back(cycles[i]);
    return out;
}
