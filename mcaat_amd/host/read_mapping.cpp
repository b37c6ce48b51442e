// reads.cpp — relevant reads (reference src/reads.cpp). The per-sequence helpers are kept
// for host callers; get_reads itself runs on the GPU over the reads already in HBM.
#include <algorithm>

#include "downstream.h"

void reverse_pair_ends_sequence(std::string &sequence) {  // reads.cpp:20-31
    std::reverse(sequence.begin(), sequence.end());
    for (char &base : sequence) {
        switch (base) {
            case 'A': base = 'T'; break;
            case 'T': base = 'A'; break;
            case 'C': base = 'G'; break;
            case 'G': base = 'C'; break;
        }
    }
}

uint64_t k_mer_to_node_id(const SDBG &sdbg, const std::string k_mer) {  // reads.cpp:33-55
    if ((int)k_mer.size() != sdbg.k()) return 0;
    std::vector<uint8_t> seq(sdbg.k());
    for (int i = 0; i < sdbg.k(); ++i) {
        const char c = k_mer[i];
        seq[i] = c == 'A' ? 1 : c == 'C' ? 2 : c == 'G' ? 3 : 4;
    }
    return (uint64_t)sdbg.IndexBinarySearch(seq.data());
}

std::vector<uint64_t> get_read_from_sequence(const SDBG &sdbg, const std::unordered_set<uint64_t> &nodes_of_cycles,
                                             const std::string &sequence) {  // reads.cpp:57-86
    const uint32_t K = sdbg.k();
    if (sequence.size() <= 2 * K) return {};
    const uint64_t start_node_id = k_mer_to_node_id(sdbg, sequence.substr(0, K));
    const uint64_t end_node_id = k_mer_to_node_id(sdbg, sequence.substr(sequence.size() - K, K));
    if (nodes_of_cycles.find(start_node_id) == nodes_of_cycles.end() &&
        nodes_of_cycles.find(end_node_id) == nodes_of_cycles.end())
        return {};
    std::vector<uint64_t> read = {start_node_id};
    for (size_t i = 1; i < sequence.size() - K; ++i) read.push_back(k_mer_to_node_id(sdbg, sequence.substr(i, K)));
    read.push_back(end_node_id);
    return read;
}

// reads.cpp:88-130. The reference re-reads the FASTQ files (file 2 reverse-complemented) and
// binary-searches every k-mer of every read; here the reads are still in HBM (mapping view
// built while parsing, mcaat_reads_records_info) and mcaat_map_reads probes only read ends
// against the cycle labels before resolving the relevant reads' k-mers.
std::vector<std::vector<uint64_t>> get_reads(const SDBG &sdbg, const mcaat_reads *reads,
                                             const std::vector<std::vector<uint64_t>> cycles) {
    return get_reads(sdbg, reads, cycles, nullptr, 1);
}

// host allgather of one vector per rank (rank order)
template <class T>
static std::vector<T> gather_all(mcaat_comm *comm, int world, const std::vector<T> &mine, std::vector<uint64_t> &counts) {
    std::vector<uint64_t> sizes(world);
    mcaat_check(mcaat_comm_allgather_sizes(comm, mine.size() * sizeof(T), sizes.data()), "comm");
    uint64_t total = 0;
    for (uint64_t b : sizes) total += b;
    std::vector<T> all(total / sizeof(T));
    mcaat_check(mcaat_comm_allgatherv(comm, mine.data(), mine.size() * sizeof(T), all.data(), sizes.data()), "comm");
    counts.resize(world);
    for (int r = 0; r < world; ++r) counts[r] = sizes[r] / sizeof(T);
    return all;
}

// With comm, every rank maps its own part of the reads (mcaat_reads_from_fastx_part: a
// contiguous record range of each input file) and the relevant reads of all ranks come back
// in input order, file by file and, inside a file, the ranks' parts in rank order.
std::vector<std::vector<uint64_t>> get_reads(const SDBG &sdbg, const mcaat_reads *reads,
                                             const std::vector<std::vector<uint64_t>> cycles, mcaat_comm *comm,
                                             int n_files) {
    std::unordered_set<uint64_t> nodes_of_cycles;
    for (const auto &cycle : cycles)
        for (const auto &node : cycle) nodes_of_cycles.insert(node);
    std::vector<uint64_t> nodes(nodes_of_cycles.begin(), nodes_of_cycles.end());
    std::sort(nodes.begin(), nodes.end());
    if (!sdbg.device()) throw std::runtime_error("get_reads: the SDBG has no device graph");
    mcaat_mapped *m = nullptr;
    mcaat_check(mcaat_map_reads(sdbg.device(), reads, nodes.data(), nodes.size(), 0, &m), "mapping the reads");
    uint64_t n = 0;
    const uint64_t *ids = nullptr, *off = nullptr, *rec = nullptr;
    mcaat_check(mcaat_mapped_get(m, &n, &ids, &off, &rec), "mcaat_mapped_get");
    int world = 1;
    if (comm) mcaat_check(mcaat_comm_info(comm, &world, nullptr), "mcaat_comm_info");
    if (world == 1) {
        std::vector<std::vector<uint64_t>> out(n);
        for (uint64_t i = 0; i < n; ++i) out[i].assign(ids + off[i], ids + off[i + 1]);
        mcaat_mapped_free(m);
        return out;
    }
    std::vector<std::vector<uint64_t>> out;
    uint64_t lo = 0, i = 0;
    for (int f = 0; f < n_files; ++f) {
        uint64_t nf = 0;
        mcaat_check(mcaat_reads_file_records(reads, f, &nf), "mcaat_reads_file_records");
        std::vector<uint64_t> lens, flat;
        for (; i < n && rec[i] < lo + nf; ++i) {
            lens.push_back(off[i + 1] - off[i]);
            flat.insert(flat.end(), ids + off[i], ids + off[i + 1]);
        }
        lo += nf;
        std::vector<uint64_t> nl, ni;
        const std::vector<uint64_t> all_lens = gather_all(comm, world, lens, nl);
        const std::vector<uint64_t> all_ids = gather_all(comm, world, flat, ni);
        uint64_t a = 0;
        for (uint64_t len : all_lens) {
            out.emplace_back(all_ids.begin() + a, all_ids.begin() + a + len);
            a += len;
        }
    }
    mcaat_mapped_free(m);
    return out;
}
