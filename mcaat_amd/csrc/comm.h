// comm.h — collectives between the ranks of a multi-GPU run (comm.hip) and the
// distributed pieces of the hot path built on them (dist.hip).
#pragma once
#include <memory>
#include <vector>

#include "internal.h"

namespace mcaat {

// One rank of `world`. Every call is collective (all ranks, same order) and returns when
// this rank's part is complete (RCCL's device all-to-alls: when queued on the context stream,
// ahead of everything later on it). Device buffers live on the context's GPU.
struct Comm {
    int rank = 0, world = 1;
    // collective calls so far (diagnostics: the exchange rounds of a bulk-synchronous stage);
    // a collective that calls another one internally counts once
    uint64_t n_coll = 0;
    // of them, the device all-to-alls (alltoallv_dev, alltoall_fixed): RCCL leaves them queued on
    // the stream, so they cost no host round trip (diagnostics: the rest are the host waits)
    uint64_t n_queued = 0;
    int coll_depth = 0;
    struct Counted {
        Comm &c;
        explicit Counted(Comm &x) : c(x) {
            if (c.coll_depth++ == 0) ++c.n_coll;
        }
        ~Counted() { --c.coll_depth; }
    };
    virtual ~Comm() = default;
    virtual const char *kind() const = 0;
    virtual void barrier() = 0;
    // every rank contributes `bytes` host bytes; `out` = all contributions in rank order,
    // sizes[r] = rank r's byte count
    virtual void allgatherv_host(const void *send, uint64_t bytes, std::vector<uint8_t> &out,
                                 std::vector<uint64_t> &sizes) = 0;
    // rank r sends send_bytes[d] bytes (at the prefix-sum offset) to each rank d and receives
    // recv_bytes[s] bytes from each rank s into recv (prefix-sum offsets, rank order)
    // (send_off / recv_off: explicit byte offsets per rank instead of the prefix sums; a rank
    // with 0 bytes each way is skipped, so a caller that moved its own share already passes 0)
    virtual void alltoallv_dev(const void *send, const uint64_t *send_bytes, void *recv,
                               const uint64_t *recv_bytes, const uint64_t *send_off = nullptr,
                               const uint64_t *recv_off = nullptr) = 0;
    // rank r's sizes[r] bytes at `send`, concatenated in rank order into recv (sizes known to all)
    virtual void allgatherv_dev(const void *send, void *recv, const uint64_t *sizes) = 0;
    // all-to-all of device segments: to each rank d this rank sends the segments send[d] in order;
    // from each rank s it receives the segments of byte sizes recv[s] (what s sends here), placed
    // back to back, sources in rank order, from `out`. No staging copy on the sending side
    // (round 5: pass A's L1 buckets go out from where pass A wrote them).
    struct Seg {
        const void *p;
        uint64_t bytes;
    };
    virtual void alltoallv_dev_segs(const std::vector<std::vector<Seg>> &send, void *out,
                                    const std::vector<std::vector<uint64_t>> &recv) = 0;

    // every rank's n 64-bit words from device memory, in rank order (a bulk-synchronous round's
    // counts): the default reads them to the host first; RCCL gathers them on the device and
    // reads the result once
    // (dev is written by work queued on the context's stream; the transports read it after that)
    virtual void allgather_dev_words(const uint64_t *dev, int n, std::vector<uint64_t> &out) = 0;

    // (round 6) fixed-size all-to-all of device blocks: block d of `send` (`bytes` each, N blocks)
    // goes to rank d and lands as block `rank` of rank d's `recv`; this rank's own block is not
    // moved. Queued on the context's stream: the RCCL transport returns without waiting for it
    // (a device-resident loop of exchanges, e.g. the per-shard region BFS, needs no host round
    // trip per exchange); the default runs it through alltoallv_dev, which does wait.
    virtual void alltoall_fixed(const void *send, uint64_t bytes, void *recv) {
        std::vector<uint64_t> sz(world, bytes), off(world);
        for (int q = 0; q < world; ++q) off[q] = (uint64_t)q * bytes;
        sz[rank] = 0;
        alltoallv_dev(send, sz.data(), recv, sz.data(), off.data(), off.data());
    }

    // typed helpers over allgatherv_host
    template <class T>
    std::vector<T> allgather_vec(const std::vector<T> &mine, std::vector<uint64_t> *counts = nullptr) {
        std::vector<uint8_t> raw;
        std::vector<uint64_t> sizes;
        allgatherv_host(mine.data(), mine.size() * sizeof(T), raw, sizes);
        std::vector<T> out(raw.size() / sizeof(T));
        if (!raw.empty()) memcpy(out.data(), raw.data(), raw.size());
        if (counts) {
            counts->resize(sizes.size());
            for (size_t r = 0; r < sizes.size(); ++r) (*counts)[r] = sizes[r] / sizeof(T);
        }
        return out;
    }
    template <class T>
    std::vector<T> allgather_one(T v) {
        return allgather_vec(std::vector<T>{v});
    }
};

// one piece of alltoallv_dev_segs' schedule: send side (segment index, offset in it, bytes) or
// receive side (seg -1, offset in the output, bytes)
struct SegPiece {
    int seg;
    uint64_t off, n;
};
void seg_schedule(int world, int rank, const std::vector<std::vector<uint64_t>> &send_sizes,
                  const std::vector<std::vector<uint64_t>> &recv_sizes, uint64_t piece,
                  std::vector<std::vector<SegPiece>> &sends, std::vector<std::vector<SegPiece>> &recvs, size_t &rounds);
uint64_t comm_schedule_check(int world, uint64_t seed, uint64_t piece);  // mcaat_comm_schedule_check

std::unique_ptr<Comm> comm_rccl(mcaat_ctx *ctx, int world, int rank, const uint8_t *unique_id);
std::unique_ptr<Comm> comm_shm(mcaat_ctx *ctx, int world, int rank, const char *name, uint64_t slot_bytes);
void comm_unique_id(uint8_t *out);  // 128 bytes (ncclGetUniqueId)

// dist.hip: the graph of the reads of all ranks (each passes its own slice), bit-identical
// to the single-GPU graph of all reads; every rank holds the whole graph afterwards
void build_graph_sharded(mcaat_ctx *ctx, Comm &comm, const mcaat_reads *r, int k, mcaat_graph *g);

}  // namespace mcaat

struct mcaat_comm {
    std::unique_ptr<mcaat::Comm> c;
};
