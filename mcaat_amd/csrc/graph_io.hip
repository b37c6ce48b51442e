// graph_io.hip — dump / load of the device SDBG (checkpoint and resume).
//
// Replaces: the on-disk graph the reference keeps between SDBGBuild and CycleFinder
// (MEGAHIT graph.sdbg* written by Read2SdbgS2 and read back by SDBG::LoadFromFile, reference
// main.cpp:386-393, 522-530; tmp_utils.cpp:52). MEGAHIT's file format cannot be pinned
// offline (un-vendored submodule), so this is the library's own format: what
// defines the graph (sorted BOSS keys, multiplicities, valid bits); the adjacency words and
// the radix directory are rebuilt on load (sdbg_finish), so a loaded graph answers every
// query exactly as the dumped one.
//
// File (little-endian): 16-byte magic "MCAAT-SDBG-v1\0\0\0", u32 k, u32 flags (0), u64 D,
// u64 valid words, then keys (8 B x D), multiplicities (2 B x D, zero-padded to 8 B), valid
// bitmap (8 B x words), and a u64 checksum of all the words before it (mix64 chain).
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"

namespace mcaat {

namespace {

constexpr char kMagic[16] = "MCAAT-SDBG-v1";
constexpr uint64_t kChunkWords = 1ull << 25;  // 256 MiB of host staging per transfer

struct Sum {
    uint64_t h = 0x6d6361617473ULL;
    void add(const uint64_t *w, size_t n) {
        uint64_t x = h;
        for (size_t i = 0; i < n; ++i) x = mix64(x ^ w[i]);
        h = x;
    }
};

struct File {
    FILE *f = nullptr;
    std::string path;
    File(const char *p, const char *mode) : path(p) {
        f = fopen(p, mode);
        if (!f) throw Error(MCAAT_E_IO, std::string("cannot open ") + p);
    }
    ~File() {
        if (f) fclose(f);
    }
    void write(const void *p, size_t n) {
        if (fwrite(p, 1, n, f) != n) throw Error(MCAAT_E_IO, "write failed: " + path);
    }
    void read(void *p, size_t n) {
        if (fread(p, 1, n, f) != n) throw Error(MCAAT_E_IO, "truncated graph file: " + path);
    }
};

// device array of `bytes` bytes <-> file, staged through a host buffer, summed as words
void dev_to_file(File &out, const void *dev, uint64_t bytes, Sum &sum, std::vector<uint64_t> &stage) {
    const uint64_t padded = (bytes + 7) / 8 * 8;
    for (uint64_t a = 0; a < padded; a += 8 * kChunkWords) {
        const uint64_t n = std::min<uint64_t>(8 * kChunkWords, padded - a);
        const uint64_t have = a < bytes ? std::min<uint64_t>(n, bytes - a) : 0;
        std::memset(stage.data(), 0, n);
        if (have) HIP_OK(hipMemcpy(stage.data(), (const uint8_t *)dev + a, have, hipMemcpyDeviceToHost));
        sum.add(stage.data(), n / 8);
        out.write(stage.data(), n);
    }
}

void file_to_dev(File &in, void *dev, uint64_t bytes, Sum &sum, std::vector<uint64_t> &stage) {
    const uint64_t padded = (bytes + 7) / 8 * 8;
    for (uint64_t a = 0; a < padded; a += 8 * kChunkWords) {
        const uint64_t n = std::min<uint64_t>(8 * kChunkWords, padded - a);
        in.read(stage.data(), n);
        sum.add(stage.data(), n / 8);
        const uint64_t have = a < bytes ? std::min<uint64_t>(n, bytes - a) : 0;
        if (have) HIP_OK(hipMemcpy((uint8_t *)dev + a, stage.data(), have, hipMemcpyHostToDevice));
    }
}

}  // namespace

void graph_save(const mcaat_graph *g, const char *path) {
    File out(path, "wb");
    const uint64_t nw = g->n_words();
    Sum sum;
    uint64_t head[4] = {0, 0, 0, 0};
    std::memcpy(head, kMagic, 16);
    head[2] = (uint64_t)(uint32_t)g->k;  // k, flags = 0
    head[3] = g->D;
    out.write(head, sizeof head);
    out.write(&nw, 8);
    sum.add(head, 4);
    sum.add(&nw, 1);
    std::vector<uint64_t> stage(kChunkWords);
    HIP_OK(hipStreamSynchronize(g->ctx->stream));
    dev_to_file(out, g->key.p, 8 * g->D, sum, stage);
    dev_to_file(out, g->mult.p, 2 * g->D, sum, stage);
    dev_to_file(out, g->valid.p, 8 * nw, sum, stage);
    out.write(&sum.h, 8);
}

void graph_load(mcaat_ctx *ctx, const char *path, mcaat_graph *g) {
    File in(path, "rb");
    uint64_t head[4], nw = 0;
    in.read(head, sizeof head);
    if (std::memcmp(head, kMagic, 16) != 0) throw Error(MCAAT_E_IO, std::string("not an mcaat graph file: ") + path);
    const int k = (int)(uint32_t)head[2];
    const uint64_t D = head[3];
    in.read(&nw, 8);
    if (k < 2 || k > kMaxK || (head[2] >> 32) != 0 || nw != (D + 63) / 64 || D > (1ull << kIdxBits))
        throw Error(MCAAT_E_IO, std::string("corrupt graph file header: ") + path);
    Sum sum;
    sum.add(head, 4);
    sum.add(&nw, 1);
    std::vector<uint64_t> stage(kChunkWords);
    g->ctx = ctx;
    g->k = k;
    g->D = D;
    g->key.alloc(D ? D : 1);
    g->mult.alloc(mcaat_graph::mult_entries(D));
    file_to_dev(in, g->key.p, 8 * D, sum, stage);
    file_to_dev(in, g->mult.p, 2 * D, sum, stage);
    DevBuf<uint64_t> valid(nw ? nw : 1);
    file_to_dev(in, valid.p, 8 * nw, sum, stage);
    uint64_t want = 0;
    in.read(&want, 8);
    if (want != sum.h) throw Error(MCAAT_E_IO, std::string("graph file checksum mismatch: ") + path);
    sdbg_finish(ctx, g);  // directory, adjacency words, all-valid bitmap
    if (nw) HIP_OK(hipMemcpyAsync(g->valid.p, valid.p, 8 * nw, hipMemcpyDeviceToDevice, ctx->stream));
    g->all_valid = false;  // the saved bits (e.g. after a CycleFinder run)
    HIP_OK(hipStreamSynchronize(ctx->stream));
}

}  // namespace mcaat
