// CPU sanitizer leg: the oracle and the host downstream code built with
// AddressSanitizer + UndefinedBehaviorSanitizer (Makefile beside this file) and run on a read
// set given as a binary file. Same flow as tests/test_downstream.py::_oracle_downstream:
// oracle graph -> CycleFinder (threads=1) -> relevant reads -> spacer ordering + CRISPRAnalyzer
// (mcaat_host_crispr_arrays) -> the report file. Prints "stats ..." for the test to compare.
//
// usage: driver <reads.bin> <k> <threshold> <report.txt>
//   reads.bin: u64 n_words, u64 n_reads, packed words, n_reads+1 offsets (library layout)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <vector>

#include "../../include/mcaat_host.h"
#include "../../oracle/oracle.h"

static std::string unpack(const std::vector<uint64_t> &p, uint64_t a, uint64_t b) {
    std::string s;
    for (uint64_t j = a; j < b; ++j) s += "ACGT"[(p[j >> 5] >> (2 * (j & 31))) & 3];
    return s;
}

int main(int argc, char **argv) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s reads.bin k threshold report.txt\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    uint64_t nw = 0, nr = 0;
    if (fread(&nw, 8, 1, f) != 1 || fread(&nr, 8, 1, f) != 1) return 2;
    std::vector<uint64_t> packed(nw + 1, 0), offs(nr + 1);
    if (fread(packed.data(), 8, nw, f) != nw || fread(offs.data(), 8, nr + 1, f) != nr + 1) return 2;
    fclose(f);
    const int k = atoi(argv[2]);

    oracle_graph *g = oracle_build(packed.data(), offs.data(), nr, k, 1);
    oracle_cf_params prm{};
    prm.threshold_multiplicity = strtoull(argv[3], nullptr, 10);
    prm.low_abundance = 1;
    prm.cycle_max_length = 77;
    prm.cycle_min_length = 27;
    prm.threads = 1;
    prm.cluster_bound = 500;
    prm.step_cap = 10000000;
    oracle_cf_result *r = oracle_cycle_finder(g, &prm);
    uint64_t st[6];
    oracle_cf_stats(r, st);

    // cycles in cycles_map_to_cycles order (the results map's iteration order)
    const uint64_t ne = oracle_cf_n_entries(r), nc = oracle_cf_n_cycles(r), nn = oracle_cf_n_nodes(r);
    std::vector<uint64_t> starts(ne + 1), cb(ne + 1), nb(nc + 1), nodes(nn + 1), order(ne + 1);
    oracle_cf_entries(r, starts.data(), cb.data());
    oracle_cf_cycles(r, nb.data(), nodes.data());
    oracle_cf_map_order(r, order.data());
    std::vector<uint64_t> cflat, coff{0};
    std::set<uint64_t> cyc_nodes;
    for (uint64_t i = 0; i < ne; ++i)
        for (uint64_t c = cb[order[i]]; c < cb[order[i] + 1]; ++c) {
            for (uint64_t x = nb[c]; x < nb[c + 1]; ++x) {
                cflat.push_back(nodes[x]);
                cyc_nodes.insert(nodes[x]);
            }
            coff.push_back(cflat.size());
        }
    // relevant reads (reads.cpp:88-130)
    std::vector<std::string> seqs(nr);
    std::vector<const char *> cs(nr);
    for (uint64_t i = 0; i < nr; ++i) {
        seqs[i] = unpack(packed, offs[i], offs[i + 1]);
        cs[i] = seqs[i].c_str();
    }
    std::vector<uint64_t> cn(cyc_nodes.begin(), cyc_nodes.end());
    uint64_t *rflat = nullptr, *roff = nullptr;
    const uint64_t n_rel = oracle_get_reads(g, cs.data(), nr, nr, cn.data(), cn.size(), &rflat, &roff);
    // host copy of the graph after CycleFinder -> spacer ordering + CRISPRAnalyzer
    const uint64_t D = oracle_graph_size(g);
    std::vector<uint64_t> keys(D + 1);
    std::vector<uint16_t> mult(D + 1);
    std::vector<uint8_t> valid(D + 1);
    oracle_graph_arrays(g, keys.data(), mult.data());
    oracle_graph_valid(g, valid.data());
    size_t n_found = 0;
    const int rc = mcaat_host_crispr_arrays(k, keys.data(), mult.data(), valid.data(), D, cflat.data(), coff.data(),
                                            coff.size() - 1, rflat, roff, n_rel, argv[4], &n_found, 4);
    if (rc != 0) {
        fprintf(stderr, "mcaat_host_crispr_arrays: %s\n", mcaat_host_last_error());
        return 1;
    }
    printf("stats %llu %llu %llu %llu %llu %llu relevant %llu found %zu\n", (unsigned long long)st[0],
           (unsigned long long)st[1], (unsigned long long)st[2], (unsigned long long)st[3], (unsigned long long)st[4],
           (unsigned long long)st[5], (unsigned long long)n_rel, n_found);
    oracle_free(rflat);
    oracle_free(roff);
    oracle_cf_free(r);
    oracle_graph_free(g);
    return 0;
}
