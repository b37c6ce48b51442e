// mcaat_host.cpp — SDBGBuild / SDBG / CycleFinder over the C ABI (see mcaat_host.h).
#include "mcaat_host.h"

#include <algorithm>
#include <cstring>
#include <chrono>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <sstream>

namespace fs = std::filesystem;

void mcaat_check(int rc, const char *what) {
    if (rc != MCAAT_OK) throw std::runtime_error(std::string(what) + ": " + mcaat_last_error());
}

// device < 0: the context already bound (the run's --gpu / rank device), else device 0
mcaat_ctx *mcaat_host_ctx(int device) {
    static mcaat_ctx *ctx = nullptr;
    static int dev = -1;
    if (device < 0) device = ctx ? dev : 0;
    if (ctx && dev != device) {
        mcaat_finalize(ctx);
        ctx = nullptr;
    }
    if (!ctx) {
        mcaat_check(mcaat_init(device, &ctx), "mcaat_init");
        dev = device;
    }
    return ctx;
}

// GPU of this process's rank in a multi-GPU run (rank 0 / one GPU: settings.gpu)
int mcaat_rank_device(const Settings &s) {
    if (s.gpus <= 1) return s.gpu;
    int n = 0;
    mcaat_check(mcaat_device_count(&n), "mcaat_device_count");
    if (n < 1) throw std::runtime_error("no HIP device available");
    return (s.gpu + s.rank) % n;
}

// ---------------------------------------------------------------- SDBGBuild
SDBGBuild::SDBGBuild(Settings s) : settings(s) {
    const auto t0 = std::chrono::steady_clock::now();
    BuildLib();
    lib_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    BuildSDBG();
}

SDBGBuild::~SDBGBuild() {
    if (graph_) mcaat_graph_free(graph_);
    if (reads_) mcaat_reads_free(reads_);
}

// sdbg_build.cpp:25-75: "<graph>/data.lib" = comment line + "se"|"pe" + input files
std::string SDBGBuild::WriteLibFile() {
    std::cout << "\n-----------------------------------------\n" << std::endl;
    std::cout << "2. Building the SDBG: " << std::endl;
    fs::path dir(settings.graph_folder);
    try {
        if (!fs::exists(dir)) fs::create_directories(dir);
    } catch (const fs::filesystem_error &e) {
        std::cerr << "Error creating directories: " << e.what() << std::endl;
        return "";
    }
    fs::path lib = dir / "data.lib";
    std::ofstream f(lib, std::ios::out | std::ios::trunc);
    if (!f) {
        std::cerr << "Error creating file: " << lib << std::endl;
        return "";
    }
    std::istringstream iss(settings.input_files);
    std::vector<std::string> tok;
    std::string t;
    while (iss >> t) tok.push_back(t);
    f << "#lib file for the SDBG from " + settings.input_files + "\n";
    f << std::string(tok.size() > 1 ? "pe" : "se") + " " + settings.input_files;
    return lib.string();
}

void SDBGBuild::BuildLib() {
    if (settings.rank == 0) WriteLibFile();
    std::istringstream iss(settings.input_files);
    std::vector<std::string> files;
    std::string t;
    while (iss >> t) files.push_back(t);
    std::vector<const char *> cf;
    for (auto &x : files) cf.push_back(x.c_str());
    mcaat_ctx *ctx = mcaat_host_ctx(mcaat_rank_device(settings));
    if (settings.gpus <= 1 || !settings.mcomm) {
        // the count's first pass runs on the input's parts while they are read (same results)
        // (MCAAT_COUNT_AHEAD=0: after the read, as the reference orders them)
        const char *e = std::getenv("MCAAT_COUNT_AHEAD");
        if (settings.load_graph.empty() && !(e && e[0] == '0'))
            mcaat_check(mcaat_count_ahead(ctx, settings.kmer_k), "count ahead");
        mcaat_check(mcaat_reads_from_fastx(ctx, cf.data(), (int)cf.size(), &reads_), "reading input files");
        return;
    }
    // each rank reads its part of every file; inputs that cannot be split (FASTA, wrapped or
    // gapped FASTQ) are read whole by rank 0, and the other ranks count nothing
    const int rc = mcaat_reads_from_fastx_part(ctx, cf.data(), (int)cf.size(), settings.rank, settings.gpus, &reads_);
    std::vector<uint64_t> sizes(settings.gpus);
    const uint8_t ok = rc == MCAAT_OK;
    mcaat_check(mcaat_comm_allgather_sizes(settings.mcomm, 1, sizes.data()), "comm");
    std::vector<uint8_t> oks(settings.gpus);
    mcaat_check(mcaat_comm_allgatherv(settings.mcomm, &ok, 1, oks.data(), sizes.data()), "comm");
    if (std::all_of(oks.begin(), oks.end(), [](uint8_t x) { return x != 0; })) return;
    if (reads_) mcaat_reads_free(reads_);
    reads_ = nullptr;
    if (settings.rank == 0) {
        std::cout << "Inputs read whole on rank 0 (" << mcaat_last_error() << ")" << std::endl;
        mcaat_check(mcaat_reads_from_fastx(ctx, cf.data(), (int)cf.size(), &reads_), "reading input files");
    } else {
        const uint64_t off0 = 0;
        mcaat_check(mcaat_reads_from_host(ctx, nullptr, 0, &off0, 0, &reads_), "empty read part");
    }
}

void SDBGBuild::BuildSDBG() {
    mcaat_ctx *ctx = mcaat_host_ctx(mcaat_rank_device(settings));
    if (!settings.load_graph.empty()) {  // every rank loads the whole graph
        mcaat_check(mcaat_graph_load(ctx, settings.load_graph.c_str(), &graph_), "loading the graph");
        std::cout << "Resumed the graph from " << settings.load_graph << std::endl;
    } else {
        if (settings.gpus > 1 && settings.mcomm)
            mcaat_check(mcaat_build_graph_sharded(ctx, settings.mcomm, reads_, settings.kmer_k, &graph_),
                        "building the SDBG over the ranks");
        else
            mcaat_check(mcaat_build_graph(ctx, reads_, settings.kmer_k, &graph_), "building the SDBG");
        if (settings.keep_graph && settings.gpus > 1 && settings.mcomm)  // the whole graph is saved
            mcaat_check(mcaat_graph_unshard(graph_, settings.mcomm), "gathering the sharded graph");
        if (settings.keep_graph && settings.rank == 0) {
            const std::string out = settings.graph_folder + "/graph.mcaat_sdbg";
            mcaat_check(mcaat_graph_save(graph_, out.c_str()), "saving the graph");
            std::cout << "Graph kept in " << out << std::endl;
        }
    }
    std::cout << "\n-----------------------------------------\n" << std::endl;
}

// ---------------------------------------------------------------- SDBG
SDBG::~SDBG() {
    if (g_) mcaat_graph_free(g_);
}

void SDBG::LoadFromDevice(mcaat_graph *g) {
    if (g_ && g_ != g) mcaat_graph_free(g_);
    g_ = g;
    mcaat_check(mcaat_graph_info(g_, &k_, &D_), "mcaat_graph_info");
    have_arrays_ = have_valid_ = false;
    kcache_.clear();
    ocache_.clear();
    std::vector<uint64_t>().swap(key_);
    std::vector<uint16_t>().swap(mult_);
    std::vector<uint64_t>().swap(vbits_);
}

void SDBG::LoadFromFile(const char *path) {
    mcaat_graph *g = nullptr;
    // on the GPU this process already works on (settings.gpu / the rank's device): binding
    // device 0 here would finalize that context
    mcaat_check(mcaat_graph_load(mcaat_host_ctx(-1), path, &g), "SDBG::LoadFromFile");
    LoadFromDevice(g);
}

void SDBG::SaveToFile(const char *path) const {
    if (!g_) throw std::runtime_error("SDBG::SaveToFile: no device graph");
    mcaat_check(mcaat_graph_save(g_, path), "SDBG::SaveToFile");
}

void SDBG::LoadFromArrays(int k, std::vector<uint64_t> keys, std::vector<uint16_t> mult,
                          std::vector<uint8_t> valid) {
    if (keys.size() != mult.size() || keys.size() != valid.size())
        throw std::runtime_error("SDBG::LoadFromArrays: array sizes differ");
    if (g_) mcaat_graph_free(g_);
    g_ = nullptr;
    k_ = k;
    D_ = keys.size();
    key_ = std::move(keys);
    mult_ = std::move(mult);
    vbits_.assign((D_ + 63) / 64, 0);
    for (uint64_t e = 0; e < D_; ++e)
        if (valid[e]) vbits_[e >> 6] |= 1ULL << (e & 63);
    have_arrays_ = have_valid_ = true;
    kcache_.clear();
    ocache_.clear();
}

const std::vector<uint64_t> &SDBG::host_key() const {
    if (!have_arrays_ && g_) {
        key_.resize(D_);
        mult_.resize(D_);
        mcaat_check(mcaat_graph_download(g_, key_.data(), mult_.data(), nullptr), "mcaat_graph_download");
        have_arrays_ = true;
    }
    return key_;
}

const std::vector<uint16_t> &SDBG::host_mult() const {
    host_key();
    return mult_;
}

const std::vector<uint64_t> &SDBG::host_valid() const {
    if (!have_valid_ && g_) {
        vbits_.resize((D_ + 63) / 64);
        mcaat_check(mcaat_graph_valid_words(g_, vbits_.data()), "mcaat_graph_valid_words");
        have_valid_ = true;
    }
    return vbits_;
}

void SDBG::SyncFromDevice() {
    if (g_) have_valid_ = false;  // re-read on the next host query
    ocache_.clear();
}

void SDBG::KeepOnly(const std::vector<uint64_t> &ids) {
    ocache_.clear();
    if (have_valid_ || !g_) {
        // valid &= keep: the kept ids' bits survive, everything else clears (no second D-byte
        // array)
        std::vector<uint64_t> live;
        for (uint64_t e : ids)
            if (e < D_ && ((vbits_[e >> 6] >> (e & 63)) & 1)) live.push_back(e);
        std::fill(vbits_.begin(), vbits_.end(), 0);
        for (uint64_t e : live) vbits_[e >> 6] |= 1ULL << (e & 63);
    }
    if (g_) mcaat_check(mcaat_graph_keep_only(g_, ids.data(), ids.size()), "mcaat_graph_keep_only");
}

void SDBG::KeepRegion(const std::vector<uint64_t> &seeds, uint64_t hops) {
    if (!g_) throw std::runtime_error("SDBG::KeepRegion: no device graph");
    ocache_.clear();
    mcaat_check(mcaat_graph_keep_region(g_, seeds.data(), seeds.size(), hops), "mcaat_graph_keep_region");
    have_valid_ = false;
}

void SDBG::SetInvalidEdge(uint64_t e) {
    ocache_.clear();
    if (have_valid_ || !g_) vbits_[e >> 6] &= ~(1ULL << (e & 63));
    if (g_) mcaat_check(mcaat_graph_set_valid(g_, &e, 1, 0), "mcaat_graph_set_valid");
}

void SDBG::SetValidEdge(uint64_t e) {
    ocache_.clear();
    if (have_valid_ || !g_) vbits_[e >> 6] |= 1ULL << (e & 63);
    if (g_) mcaat_check(mcaat_graph_set_valid(g_, &e, 1, 1), "mcaat_graph_set_valid");
}

uint64_t SDBG::lower(uint64_t q) const {
    const auto &key = host_key();
    return std::lower_bound(key.begin(), key.end(), q) - key.begin();
}

int SDBG::OutgoingEdges(uint64_t e, uint64_t *out) const {
    if (!ocache_.empty()) {
        if (const auto *a = ocache_.find(e)) {
            const int n = (int)(*a)[0];
            for (int i = 0; i < n; ++i) out[i] = (*a)[1 + i];
            return n;
        }
    }
    const auto &key_ = host_key();
    const auto &vb = host_valid();
    const uint64_t K = key_[e], W = K & 3, R = K >> 2;
    const uint64_t Rt = (W << (2 * (k_ - 1))) | (R >> 2);
    uint64_t tmp[4];
    int n = 0;
    for (uint64_t i = lower(Rt << 2); i < size() && (key_[i] >> 2) == Rt; ++i)
        if ((vb[i >> 6] >> (i & 63)) & 1) tmp[n++] = i;
    for (int i = 0; i < n; ++i) out[i] = tmp[n - 1 - i];
    return n;
}

int SDBG::IncomingEdges(uint64_t e, uint64_t *in) const {
    const auto &key_ = host_key();
    const auto &vb = host_valid();
    const uint64_t K = key_[e];
    const uint64_t c = (K >> (2 * k_)) & 3;
    const uint64_t G = (K >> 2) & ((1ULL << (2 * (k_ - 1))) - 1);
    int n = 0;
    for (uint64_t i = lower(G << 4); i < size() && (key_[i] >> 4) == G; ++i)
        if ((key_[i] & 3) == c && ((vb[i >> 6] >> (i & 63)) & 1)) in[n++] = i;
    return n;
}

void SDBG::NeighborsBatch(const std::vector<uint64_t> &ids, bool incoming, std::vector<uint64_t> &out,
                          std::vector<int32_t> &counts) const {
    out.assign(4 * ids.size(), 0);
    counts.assign(ids.size(), 0);
    if (ids.empty()) return;
    if (g_) {
        mcaat_check(mcaat_graph_neighbors(g_, ids.data(), ids.size(), incoming ? 1 : 0, out.data(), counts.data()),
                    "mcaat_graph_neighbors");
        return;
    }
    for (size_t i = 0; i < ids.size(); ++i)
        counts[i] = incoming ? IncomingEdges(ids[i], &out[4 * i]) : OutgoingEdges(ids[i], &out[4 * i]);
}

void SDBG::PrefetchKeys(const std::vector<uint64_t> &ids) {
    if (!g_ || ids.empty()) return;
    std::vector<uint64_t> want;
    for (uint64_t e : ids)
        if (!kcache_.contains(e)) want.push_back(e);
    if (want.empty()) return;
    std::vector<uint64_t> kk(want.size());
    std::vector<uint16_t> mm(want.size());
    mcaat_check(mcaat_graph_gather(g_, want.data(), want.size(), kk.data(), mm.data()), "mcaat_graph_gather");
    kcache_.reserve(kcache_.size() + want.size());
    for (size_t i = 0; i < want.size(); ++i) kcache_[want[i]] = {kk[i], mm[i]};
}

void SDBG::PrefetchOutgoing(const std::vector<uint64_t> &ids) {
    if (!g_ || ids.empty()) return;
    std::vector<uint64_t> nb;
    std::vector<int32_t> cnt;
    NeighborsBatch(ids, false, nb, cnt);
    ocache_.reserve(ocache_.size() + ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
        std::array<uint64_t, 5> a{(uint64_t)cnt[i], 0, 0, 0, 0};
        for (int j = 0; j < cnt[i]; ++j) a[1 + j] = nb[4 * i + j];
        ocache_[ids[i]] = a;
    }
}

std::vector<uint64_t> SDBG::ValidIds() const {
    const auto &v = host_valid();
    std::vector<uint64_t> out;
    for (uint64_t w = 0; w < v.size(); ++w)  // all-zero words skipped
        for (uint64_t x = v[w]; x; x &= x - 1) out.push_back(64 * w + (uint64_t)__builtin_ctzll(x));
    return out;
}

void SDBG::ValidSubgraph(std::vector<uint64_t> &ids, std::vector<uint32_t> &nbr, std::vector<uint8_t> &cnt) const {
    if (g_) {
        uint64_t n = 0;
        mcaat_check(mcaat_graph_valid_subgraph(g_, &n, nullptr, nullptr, nullptr), "mcaat_graph_valid_subgraph");
        ids.assign(n, 0);
        nbr.assign(4 * n, 0);
        cnt.assign(n, 0);
        if (n) mcaat_check(mcaat_graph_valid_subgraph(g_, &n, ids.data(), nbr.data(), cnt.data()), "mcaat_graph_valid_subgraph");
        return;
    }
    ids = ValidIds();
    nbr.assign(4 * ids.size(), 0);
    cnt.assign(ids.size(), 0);
    for (size_t i = 0; i < ids.size(); ++i) {
        uint64_t out[4];
        const int n = OutgoingEdges(ids[i], out);
        cnt[i] = (uint8_t)n;
        for (int j = 0; j < n; ++j)
            nbr[4 * i + j] = (uint32_t)(std::lower_bound(ids.begin(), ids.end(), out[j]) - ids.begin());
    }
}

uint32_t SDBG::GetLabel(uint64_t e, uint8_t *seq) const {
    const auto *kc = kcache_.find(e);
    const uint64_t R = (kc ? kc->first : host_key()[e]) >> 2;
    for (int i = 0; i < k_; ++i) seq[i] = (uint8_t)(((R >> (2 * i)) & 3) + 1);
    return (uint32_t)k_;
}

int64_t SDBG::IndexBinarySearch(const uint8_t *seq) const {
    uint64_t R = 0;
    for (int i = 0; i < k_; ++i) R |= (uint64_t)((seq[i] - 1) & 3) << (2 * i);
    const auto &key_ = host_key();
    int64_t last = -1;
    for (uint64_t i = lower(R << 2); i < size() && (key_[i] >> 2) == R; ++i) last = (int64_t)i;
    return last;
}

// ---------------------------------------------------------------- CycleFinder
CycleFinder::CycleFinder(Settings &s) : settings(s) {
    if (settings.sdbg == nullptr)  // cycle_finder.cpp:134-136
        throw std::runtime_error("CycleFinder requires settings.sdbg to be set to a valid SDBG instance");
    mcaat_cf_params p;
    mcaat_cf_default_params(&p);
    p.threshold_multiplicity = settings.cycle_finder_settings.threshold_multiplicity;
    p.low_abundance = settings.cycle_finder_settings.low_abundance ? 1 : 0;
    p.cycle_max_length = settings.cycle_finder_settings.cycle_max_length;
    p.cycle_min_length = settings.cycle_finder_settings.cycle_min_length;
    mcaat_cycles *c = nullptr;
    mcaat_check(mcaat_cycle_finder_comm(settings.sdbg->device(), settings.gpus > 1 ? settings.mcomm : nullptr, &p, &c),
                "CycleFinder");
    size_t n = 0;
    mcaat_cycles_count(c, &n);
    mcaat_cycles_stats(c, stats);
    std::cout << "Graph size: " << settings.sdbg->size() << " nodes; gathered tips: " << stats[0] << std::endl;
    std::cout << "Pre-filter: invalidated " << stats[1] << " node(s) with multiplicity <= 1." << std::endl;
    std::cout << "After pruning, tips: " << stats[3] << ", valid edges: " << stats[2] << std::endl;
    std::cout << "Start nodes found in chunks: " << stats[4] << std::endl;
    for (size_t i = 0; i < n; ++i) {
        uint64_t start = 0;
        const uint64_t *flat = nullptr, *off = nullptr;
        size_t nc = 0;
        mcaat_cycles_get(c, i, &start, &flat, &off, &nc);
        std::vector<std::vector<uint64_t>> cycles(nc);
        for (size_t j = 0; j < nc; ++j) cycles[j].assign(flat + off[j], flat + off[j + 1]);
        results[start] = std::move(cycles);  // commit order == reference insertion order
        commit_order.push_back(start);
    }
    mcaat_cycles_free(c);
    settings.sdbg->SyncFromDevice();  // the reference mutates the SDBG's valid bits
    std::cout << "Cycle enumeration completed: total cycles=" << stats[5] << ", result nodes=" << results.size()
              << std::endl;
}

std::vector<std::vector<uint64_t>> cycles_map_to_cycles(
    const std::unordered_map<uint64_t, std::vector<std::vector<uint64_t>>> &cycles_map) {
    std::vector<std::vector<uint64_t>> cycles;
    for (const auto &[_, inner] : cycles_map)
        for (const auto &c : inner) cycles.push_back(c);
    return cycles;
}
