// mcaat_host.h — the reference's hot-path classes (SDBGBuild, SDBG, CycleFinder) over the
// C ABI of libmcaat_gpu.so. Same names, constructor signatures, public members and error
// behaviour as reference include/sdbg_build.h:21-33, MEGAHIT sdbg/sdbg.h (API subset used
// by mcaat) and include/cycle_finder.h:25-85, so `main` reads the same.
#pragma once
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <array>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mcaat_gpu.h"
#include "settings.h"

// throws std::runtime_error(mcaat_last_error()) for a negative status
void mcaat_check(int rc, const char *what);

// One GPU context per process (one process per GPU).
mcaat_ctx *mcaat_host_ctx(int device);  // device < 0: the one already bound (else 0)
// the GPU of this process's rank (settings.gpu on one GPU)
int mcaat_rank_device(const Settings &s);

// Reference: SDBGBuild(Settings) writes <graph>/data.lib (sdbg_build.cpp:25-75), builds the
// read library and the SDBG (MEGAHIT). Here: the same data.lib, FASTQ/FASTA(.gz) -> packed
// reads in HBM -> node_counter -> sdbg_build; the graph stays resident on the GPU.
class SDBGBuild {
   public:
    explicit SDBGBuild(Settings settings);
    ~SDBGBuild();
    mcaat_graph *graph() const { return graph_; }
    // the reads stay in HBM for the relevant-read mapping (the reference re-reads the files)
    const mcaat_reads *reads() const { return reads_; }
    mcaat_graph *release_graph() {
        mcaat_graph *g = graph_;
        graph_ = nullptr;
        return g;
    }
    double lib_seconds = 0;  // BuildLib wall time (FASTQ -> 2-bit reads in HBM)

   private:
    std::string WriteLibFile();
    void BuildLib();
    void BuildSDBG();
    Settings settings;
    mcaat_reads *reads_ = nullptr;
    mcaat_graph *graph_ = nullptr;
};

// Open-addressing map from edge ids to V, linear probing in a power-of-two table kept at most
// half full: the host caches of the downstream steps hold ~1M entries at C3, where
// std::unordered_map's node allocations dominated step 7. The empty-slot marker ~0 is also a
// key callers use (a read's absent label, the reference's -1): it lives beside the table.
template <class V>
class IdMap {
   public:
    void clear() {
        keys_.clear();
        vals_.clear();
        n_ = 0;
        has_max_ = false;
    }
    bool empty() const { return n_ == 0; }
    size_t size() const { return n_; }
    void reserve(size_t n) {
        size_t cap = 16;
        while (cap < 2 * n + 2) cap <<= 1;
        if (cap > keys_.size()) rehash(cap);
    }
    const V *find(uint64_t k) const {
        if (k == kEmpty) return has_max_ ? &max_val_ : nullptr;
        if (keys_.empty()) return nullptr;
        for (size_t i = slot(k);; i = (i + 1) & (keys_.size() - 1)) {
            if (keys_[i] == k) return &vals_[i];
            if (keys_[i] == kEmpty) return nullptr;
        }
    }
    bool contains(uint64_t k) const { return find(k) != nullptr; }
    V &operator[](uint64_t k) {
        if (k == kEmpty) {
            if (!has_max_) {
                has_max_ = true;
                max_val_ = V{};
                ++n_;
            }
            return max_val_;
        }
        if (2 * (n_ + 1) > keys_.size()) rehash(keys_.empty() ? 16 : 2 * keys_.size());
        size_t i = slot(k);
        for (; keys_[i] != k; i = (i + 1) & (keys_.size() - 1))
            if (keys_[i] == kEmpty) {
                keys_[i] = k;
                vals_[i] = V{};
                ++n_;
                break;
            }
        return vals_[i];
    }

   private:
    static constexpr uint64_t kEmpty = ~0ULL;
    size_t slot(uint64_t k) const {
        uint64_t x = k * 0x9E3779B97F4A7C15ULL;
        return (size_t)(x ^ (x >> 29)) & (keys_.size() - 1);
    }
    void rehash(size_t cap) {
        std::vector<uint64_t> ok(cap, kEmpty);
        std::vector<V> ov(cap);
        ok.swap(keys_);
        ov.swap(vals_);
        n_ = has_max_ ? 1 : 0;
        for (size_t i = 0; i < ok.size(); ++i)
            if (ok[i] != kEmpty) (*this)[ok[i]] = ov[i];
    }
    std::vector<uint64_t> keys_;
    std::vector<V> vals_;
    size_t n_ = 0;
    bool has_max_ = false;
    V max_val_{};
};

// MEGAHIT SDBG API subset, valid-only neighbour semantics (DESIGN.md "SDBG conventions").
// Queries run on a host mirror of the device arrays; SetInvalidEdge/SetValidEdge update both.
class SDBG {
   public:
    SDBG() = default;
    ~SDBG();
    SDBG(const SDBG &) = delete;
    SDBG &operator=(const SDBG &) = delete;
    // adopt a device graph (replaces SDBG::LoadFromFile of the on-disk MEGAHIT graph)
    void LoadFromDevice(mcaat_graph *g);
    // the library's own graph file (mcaat_graph_save / mcaat_graph_load), on GPU 0's context
    void LoadFromFile(const char *path);
    void SaveToFile(const char *path) const;
    // host-only graph (no device copy) from sorted BOSS keys, multiplicities and valid bytes
    void LoadFromArrays(int k, std::vector<uint64_t> keys, std::vector<uint16_t> mult, std::vector<uint8_t> valid);
    // refresh the host mirror after device-side mutation (CycleFinder)
    void SyncFromDevice();
    // valid &= {ids} on the host mirror and the device graph (one bitmap AND on the GPU)
    void KeepOnly(const std::vector<uint64_t> &ids);
    // device graphs: valid &= the seeds grown by `hops` rounds over valid neighbours, on the GPU
    // (mcaat_graph_keep_region); the host mirror re-reads the bits on its next query
    void KeepRegion(const std::vector<uint64_t> &seeds, uint64_t hops);
    mcaat_graph *device() const { return g_; }

    uint64_t size() const { return D_; }
    int k() const { return k_; }
    bool IsValidEdge(uint64_t e) const { return (host_valid()[e >> 6] >> (e & 63)) & 1; }
    void SetInvalidEdge(uint64_t e);
    void SetValidEdge(uint64_t e);
    uint16_t EdgeMultiplicity(uint64_t e) const { return host_mult()[e]; }
    int OutgoingEdges(uint64_t e, uint64_t *out) const;  // descending ids
    int IncomingEdges(uint64_t e, uint64_t *in) const;   // ascending ids
    int EdgeOutdegree(uint64_t e) const {
        uint64_t t[4];
        return OutgoingEdges(e, t);
    }
    int EdgeIndegree(uint64_t e) const {
        uint64_t t[4];
        return IncomingEdges(e, t);
    }
    bool EdgeOutdegreeZero(uint64_t e) const { return EdgeOutdegree(e) == 0; }
    // valid neighbours of many edges in one call (on the device when the graph is there):
    // out[4i .. 4i+counts[i]) in OutgoingEdges / IncomingEdges order
    void NeighborsBatch(const std::vector<uint64_t> &ids, bool incoming, std::vector<uint64_t> &out,
                        std::vector<int32_t> &counts) const;
    uint32_t GetLabel(uint64_t e, uint8_t *seq) const;      // symbols 1..4 = ACGT
    // Host-side query caches for a known node set (not in MEGAHIT's API): the keys of `ids`
    // (labels, multiplicities) and their valid out-neighbours as of now, fetched from the device
    // graph in one call each, so label and neighbour queries on them need no copy of the whole
    // graph on the host (C3: 10 GB, 2 s) and no binary searches over it. Neighbour entries are
    // dropped when valid bits change; keys never change.
    void PrefetchKeys(const std::vector<uint64_t> &ids);
    void PrefetchOutgoing(const std::vector<uint64_t> &ids);
    // valid edge ids in ascending order
    std::vector<uint64_t> ValidIds() const;
    // the valid edges (ascending) and each one's valid out-neighbours (OutgoingEdges order) as
    // positions in that list, nbr[4i .. 4i + cnt[i]) (one device call on a device graph)
    void ValidSubgraph(std::vector<uint64_t> &ids, std::vector<uint32_t> &nbr, std::vector<uint8_t> &cnt) const;
    int64_t IndexBinarySearch(const uint8_t *seq) const;    // -1 if absent
    static constexpr uint64_t kNullID = ~0ULL;

   private:
    uint64_t lower(uint64_t q) const;
    // The host arrays are materialised from the device graph on the first host-side query
    // (none of the hot path needs them: CycleFinder runs on the device), and the valid bytes
    // are re-read after a device-side mutation.
    const std::vector<uint64_t> &host_key() const;
    const std::vector<uint16_t> &host_mult() const;
    // the valid bits as a bitmap (edge e: bit e % 64 of word e / 64), 1 bit per edge on the host
    const std::vector<uint64_t> &host_valid() const;
    mcaat_graph *g_ = nullptr;
    int k_ = 0;
    uint64_t D_ = 0;
    mutable bool have_arrays_ = false, have_valid_ = false;
    mutable std::vector<uint64_t> key_;
    mutable std::vector<uint16_t> mult_;
    mutable std::vector<uint64_t> vbits_;
    IdMap<std::pair<uint64_t, uint16_t>> kcache_;  // id -> (key, mult)
    IdMap<std::array<uint64_t, 5>> ocache_;       // id -> (n, out[4])
};

// Reference: CycleFinder(Settings&) runs FindApproximateCRISPRArrays in the constructor and
// leaves `results` (cycle_finder.cpp:131-138, cycle_finder.h:60). Results are inserted in the
// reference's threads=1 commit order, so the unordered_map iteration order is the reference's.
class CycleFinder {
   public:
    explicit CycleFinder(Settings &settings);
    std::unordered_map<uint64_t, std::vector<std::vector<uint64_t>>> results;
    std::vector<uint64_t> commit_order;  // start nodes in commit order
    uint64_t stats[8] = {0, 0, 0, 0, 0, 0, 0, 0};

   private:
    Settings &settings;
};

// tmp_utils.cpp:26-38
std::vector<std::vector<uint64_t>> cycles_map_to_cycles(
    const std::unordered_map<uint64_t, std::vector<std::vector<uint64_t>>> &cycles_map);
