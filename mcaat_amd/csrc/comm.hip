// comm.hip — collectives between the ranks of a multi-GPU run (one process per GPU;
// SURVEY.md §8e). Two transports behind one interface (comm.h):
//   RCCL  device buffers move GPU to GPU over xGMI (ncclSend/ncclRecv groups for the
//         all-to-all, grouped ncclBroadcast for the exact-size all-gather). librccl is
//         opened on first use, so single-GPU runs never load it.
//   SHM   a POSIX shared-memory segment on the host: device buffers are staged through it
//         (ranks sharing one GPU, rehearsals, and host-only tests without a GPU).
// Every operation is collective. It returns once this rank's part is done, except the RCCL
// all-to-alls (alltoallv_dev, alltoall_fixed), which return once queued on the context stream:
// their results are for work ordered behind them on that stream (kernels, d2h).
#include <dlfcn.h>
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <cerrno>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "comm.h"

namespace mcaat {

namespace {

// exclusive prefix sums of per-rank byte counts
std::vector<uint64_t> offsets_of(const uint64_t *bytes, int n) {
    std::vector<uint64_t> o(n + 1, 0);
    for (int i = 0; i < n; ++i) o[i + 1] = o[i] + bytes[i];
    return o;
}

// ------------------------------------------------------------------ RCCL ----
struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *);
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int);
    ncclResult_t (*CommDestroy)(ncclComm_t);
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    ncclResult_t (*Broadcast)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*GroupStart)();
    ncclResult_t (*GroupEnd)();
    const char *(*GetErrorString)(ncclResult_t);
};

const Rccl &rccl() {
    static Rccl r = [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) throw Error(MCAAT_E_HIP, std::string("cannot load librccl: ") + dlerror());
        Rccl x{};
        auto sym = [&](const char *name) {
            void *p = dlsym(h, name);
            if (!p) throw Error(MCAAT_E_HIP, std::string("librccl lacks ") + name);
            return p;
        };
        x.GetUniqueId = (decltype(x.GetUniqueId))sym("ncclGetUniqueId");
        x.CommInitRank = (decltype(x.CommInitRank))sym("ncclCommInitRank");
        x.CommDestroy = (decltype(x.CommDestroy))sym("ncclCommDestroy");
        x.AllGather = (decltype(x.AllGather))sym("ncclAllGather");
        x.Broadcast = (decltype(x.Broadcast))sym("ncclBroadcast");
        x.Send = (decltype(x.Send))sym("ncclSend");
        x.Recv = (decltype(x.Recv))sym("ncclRecv");
        x.GroupStart = (decltype(x.GroupStart))sym("ncclGroupStart");
        x.GroupEnd = (decltype(x.GroupEnd))sym("ncclGroupEnd");
        x.GetErrorString = (decltype(x.GetErrorString))sym("ncclGetErrorString");
        return x;
    }();
    return r;
}

#define NCCL_OK(expr)                                                                              \
    do {                                                                                           \
        ncclResult_t r__ = (expr);                                                                 \
        if (r__ != ncclSuccess)                                                                    \
            throw ::mcaat::Error(MCAAT_E_HIP, std::string(#expr " failed: ") + rccl().GetErrorString(r__)); \
    } while (0)

// RCCL counts are size_t, but pieces of at most 1 GiB keep every message well inside the
// ranges all RCCL versions test
constexpr uint64_t kPiece = 1ULL << 30;

}  // namespace

// The op schedule of RcclComm::alltoallv_dev_segs on one rank: to each peer q the segments
// send_sizes[q] (in order) cut into pieces, from each peer q the segments recv_sizes[q] cut the
// same way and placed back to back from the start of q's block of `out` (sources in rank order).
// Round j of the exchange holds, per peer, the j-th send piece and the j-th receive piece, so the
// k-th operation between two ranks sits in the same round on both sides (one ncclGroupEnd per
// round: a round-agnostic split could wait on a peer's later round). Shared with
// mcaat_comm_schedule_check, which builds every rank's schedule and checks the pairing on the host.
void seg_schedule(int world, int rank, const std::vector<std::vector<uint64_t>> &send_sizes,
                  const std::vector<std::vector<uint64_t>> &recv_sizes, uint64_t piece,
                  std::vector<std::vector<SegPiece>> &sends, std::vector<std::vector<SegPiece>> &recvs, size_t &rounds) {
    sends.assign(world, {});
    recvs.assign(world, {});
    rounds = 0;
    uint64_t d = 0;  // receive offset in out
    for (int q = 0; q < world; ++q)
        for (const uint64_t n : recv_sizes[q]) {
            if (q != rank)
                for (uint64_t c0 = 0; c0 < n; c0 += piece) recvs[q].push_back({-1, d + c0, std::min(piece, n - c0)});
            d += n;
        }
    for (int q = 0; q < world; ++q) {
        if (q == rank) continue;
        for (size_t i = 0; i < send_sizes[q].size(); ++i)
            for (uint64_t c0 = 0; c0 < send_sizes[q][i]; c0 += piece)
                sends[q].push_back({(int)i, c0, std::min(piece, send_sizes[q][i] - c0)});
        rounds = std::max({rounds, sends[q].size(), recvs[q].size()});
    }
}

namespace {

struct RcclComm final : Comm {
    mcaat_ctx *ctx;
    ncclComm_t comm = nullptr;
    RcclComm(mcaat_ctx *c, int world_, int rank_, const uint8_t *id) : ctx(c) {
        world = world_;
        rank = rank_;
        ncclUniqueId u;
        memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
        mcaat::bind(ctx);
        NCCL_OK(rccl().CommInitRank(&comm, world, u, rank));
    }
    ~RcclComm() override {
        if (comm) (void)rccl().CommDestroy(comm);
        if (pin) (void)hipHostFree(pin);
    }
    // small host all-gathers (the routers' count exchanges, one per bulk-synchronous round): one
    // fixed-slot ncclAllGather through pinned staging — the slot carries the size and the payload —
    // instead of a size all-gather, a data all-gather and four pageable copies
    static constexpr uint64_t kSmallSlot = 1024;
    uint8_t *pin = nullptr;  // (world + 1) slots: this rank's, then everyone's
    const char *kind() const override { return "rccl"; }

    void sync() { HIP_OK(hipStreamSynchronize(ctx->stream)); }

    void barrier() override {
        Counted cc__(*this);
        DevBuf<uint64_t> a(1), b(world);
        HIP_OK(hipMemsetAsync(a.p, 0, 8, ctx->stream));
        NCCL_OK(rccl().AllGather(a.p, b.p, 8, ncclUint8, comm, ctx->stream));
        sync();
    }

    void allgather_u64(uint64_t v, std::vector<uint64_t> &out) {
        DevBuf<uint64_t> a(1), b(world);
        HIP_OK(hipMemcpyAsync(a.p, &v, 8, hipMemcpyHostToDevice, ctx->stream));
        NCCL_OK(rccl().AllGather(a.p, b.p, 8, ncclUint8, comm, ctx->stream));
        out.resize(world);
        HIP_OK(hipMemcpyAsync(out.data(), b.p, 8 * (uint64_t)world, hipMemcpyDeviceToHost, ctx->stream));
        sync();
    }

    void allgatherv_host(const void *send, uint64_t bytes, std::vector<uint8_t> &out,
                         std::vector<uint64_t> &sizes) override {
        Counted cc__(*this);
        // every rank takes the slot path or none: whether it fits is agreed in the slot itself
        // (a size past the slot sends the size only, and every rank then runs the general path)
        if (!pin) HIP_OK(hipHostMalloc((void **)&pin, (world + 1) * kSmallSlot, hipHostMallocDefault));
        {
            const bool fits = bytes + 8 <= kSmallSlot;
            memcpy(pin, &bytes, 8);
            if (fits && bytes) memcpy(pin + 8, send, bytes);
            DevBuf<uint8_t> a(kSmallSlot), b((uint64_t)world * kSmallSlot);
            HIP_OK(hipMemcpyAsync(a.p, pin, kSmallSlot, hipMemcpyHostToDevice, ctx->stream));
            NCCL_OK(rccl().AllGather(a.p, b.p, kSmallSlot, ncclUint8, comm, ctx->stream));
            HIP_OK(hipMemcpyAsync(pin + kSmallSlot, b.p, (uint64_t)world * kSmallSlot, hipMemcpyDeviceToHost, ctx->stream));
            sync();
            sizes.resize(world);
            bool all = true;
            for (int r = 0; r < world; ++r) {
                memcpy(&sizes[r], pin + (uint64_t)(r + 1) * kSmallSlot, 8);
                if (sizes[r] + 8 > kSmallSlot) all = false;
            }
            if (all) {
                const auto off = offsets_of(sizes.data(), world);
                out.resize(off[world]);
                for (int r = 0; r < world; ++r)
                    if (sizes[r]) memcpy(out.data() + off[r], pin + (uint64_t)(r + 1) * kSmallSlot + 8, sizes[r]);
                return;
            }
        }
        allgather_u64(bytes, sizes);
        const auto off = offsets_of(sizes.data(), world);
        out.resize(off[world]);
        if (!off[world]) return;
        DevBuf<uint8_t> s(bytes ? bytes : 1), r(off[world]);
        if (bytes) HIP_OK(hipMemcpyAsync(s.p, send, bytes, hipMemcpyHostToDevice, ctx->stream));
        allgatherv_dev(s.p, r.p, sizes.data());
        HIP_OK(hipMemcpyAsync(out.data(), r.p, off[world], hipMemcpyDeviceToHost, ctx->stream));
        sync();
    }

    void allgather_dev_words(const uint64_t *dev, int n, std::vector<uint64_t> &out) override {
        Counted cc__(*this);
        out.resize((size_t)world * n);
        if (!n) return;
        if (!pin) HIP_OK(hipHostMalloc((void **)&pin, (world + 1) * kSmallSlot, hipHostMallocDefault));
        if ((uint64_t)n * 8 > kSmallSlot) {  // larger than the pinned slots: through the host
            std::vector<uint64_t> mine(n);
            HIP_OK(hipMemcpyAsync(mine.data(), dev, 8 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
            sync();
            out = allgather_vec(mine);
            return;
        }
        DevBuf<uint64_t> b((uint64_t)world * n);
        NCCL_OK(rccl().AllGather(dev, b.p, 8 * (size_t)n, ncclUint8, comm, ctx->stream));
        HIP_OK(hipMemcpyAsync(pin, b.p, (uint64_t)world * n * 8, hipMemcpyDeviceToHost, ctx->stream));
        sync();
        memcpy(out.data(), pin, (uint64_t)world * n * 8);
    }

    void alltoallv_dev(const void *send, const uint64_t *send_bytes, void *recv, const uint64_t *recv_bytes,
                       const uint64_t *send_off, const uint64_t *recv_off) override {
        Counted cc__(*this);
        if (coll_depth == 1) ++n_queued;
        auto so = offsets_of(send_bytes, world), ro = offsets_of(recv_bytes, world);
        if (send_off) so.assign(send_off, send_off + world);
        if (recv_off) ro.assign(recv_off, recv_off + world);
        const uint8_t *s = (const uint8_t *)send;
        uint8_t *d = (uint8_t *)recv;
        if (send_bytes[rank] != recv_bytes[rank]) throw Error(MCAAT_E_INVALID, "alltoallv: self sizes differ");
        if (send_bytes[rank])
            HIP_OK(hipMemcpyAsync(d + ro[rank], s + so[rank], send_bytes[rank], hipMemcpyDeviceToDevice, ctx->stream));
        uint64_t most = 0;
        for (int p = 0; p < world; ++p)
            if (p != rank) most = std::max({most, send_bytes[p], recv_bytes[p]});
        // piece c of every peer's message in one group (matching send/recv order on all ranks)
        for (uint64_t c0 = 0; c0 < most; c0 += kPiece) {
            NCCL_OK(rccl().GroupStart());
            for (int p = 0; p < world; ++p) {
                if (p == rank) continue;
                if (send_bytes[p] > c0)
                    NCCL_OK(rccl().Send(s + so[p] + c0, std::min(kPiece, send_bytes[p] - c0), ncclUint8, p, comm,
                                        ctx->stream));
                if (recv_bytes[p] > c0)
                    NCCL_OK(rccl().Recv(d + ro[p] + c0, std::min(kPiece, recv_bytes[p] - c0), ncclUint8, p, comm,
                                        ctx->stream));
            }
            NCCL_OK(rccl().GroupEnd());
        }
        // (round 6) no synchronise: the exchange stays queued on the context stream, and every
        // consumer of `recv` (kernels, d2h) is ordered behind it on that stream, as every reuse of
        // `send` through the stream-ordered arena is; a routed round now waits on the host once,
        // for its count all-gather, instead of three times
    }

    // one ncclSend / ncclRecv per peer, grouped, left running on the stream (no synchronise)
    void alltoall_fixed(const void *send, uint64_t bytes, void *recv) override {
        Counted cc__(*this);
        if (coll_depth == 1) ++n_queued;
        if (world == 1 || !bytes) return;
        // blocks above 1 GiB in pieces, every peer's piece c in group c (as alltoallv_dev)
        for (uint64_t c0 = 0; c0 < bytes; c0 += kPiece) {
            const uint64_t n = std::min(kPiece, bytes - c0);
            NCCL_OK(rccl().GroupStart());
            for (int p = 0; p < world; ++p) {
                if (p == rank) continue;
                NCCL_OK(rccl().Send((const uint8_t *)send + (uint64_t)p * bytes + c0, n, ncclUint8, p, comm, ctx->stream));
                NCCL_OK(rccl().Recv((uint8_t *)recv + (uint64_t)p * bytes + c0, n, ncclUint8, p, comm, ctx->stream));
            }
            NCCL_OK(rccl().GroupEnd());
        }
    }

    // Segments in rounds: round j holds, for every peer, the j-th send segment and the j-th
    // receive segment (pieces of 1 GiB), so the k-th operation between two ranks sits in the
    // same round on both sides (ncclGroupEnd of one round completes before the next starts on
    // the stream; a round-agnostic split could wait on a peer's later round).
    void alltoallv_dev_segs(const std::vector<std::vector<Seg>> &send, void *out,
                            const std::vector<std::vector<uint64_t>> &recv) override {
        Counted cc__(*this);
        std::vector<std::vector<uint64_t>> ssz(world);
        for (int q = 0; q < world; ++q)
            for (const Seg &g : send[q]) ssz[q].push_back(g.bytes);
        std::vector<std::vector<SegPiece>> sends, recvs;
        size_t rounds = 0;
        seg_schedule(world, rank, ssz, recv, kPiece, sends, recvs, rounds);
        // own segments: copies on the stream, in place
        {
            uint8_t *o = (uint8_t *)out;
            for (int q = 0; q < rank; ++q)
                for (const uint64_t n : recv[q]) o += n;
            if (send[rank].size() != recv[rank].size()) throw Error(MCAAT_E_INVALID, "alltoallv_segs: self segments differ");
            for (size_t i = 0; i < send[rank].size(); ++i) {
                if (send[rank][i].bytes != recv[rank][i]) throw Error(MCAAT_E_INVALID, "alltoallv_segs: self sizes differ");
                if (send[rank][i].bytes)
                    HIP_OK(hipMemcpyAsync(o, send[rank][i].p, send[rank][i].bytes, hipMemcpyDeviceToDevice, ctx->stream));
                o += send[rank][i].bytes;
            }
        }
        uint8_t *d = (uint8_t *)out;
        for (size_t j = 0; j < rounds; ++j) {
            NCCL_OK(rccl().GroupStart());
            for (int q = 0; q < world; ++q) {
                if (q == rank) continue;
                if (j < sends[q].size()) {
                    const SegPiece &x = sends[q][j];
                    NCCL_OK(rccl().Send((const uint8_t *)send[q][x.seg].p + x.off, x.n, ncclUint8, q, comm, ctx->stream));
                }
                if (j < recvs[q].size())
                    NCCL_OK(rccl().Recv(d + recvs[q][j].off, recvs[q][j].n, ncclUint8, q, comm, ctx->stream));
            }
            NCCL_OK(rccl().GroupEnd());
        }
        sync();
    }

    // exact-size all-gather: one broadcast per root into its place in the output, grouped
    void allgatherv_dev(const void *send, void *recv, const uint64_t *sizes) override {
        Counted cc__(*this);
        const auto off = offsets_of(sizes, world);
        uint8_t *d = (uint8_t *)recv;
        uint64_t most = 0;
        for (int r = 0; r < world; ++r) most = std::max(most, sizes[r]);
        for (uint64_t c0 = 0; c0 < most; c0 += kPiece) {
            NCCL_OK(rccl().GroupStart());
            for (int r = 0; r < world; ++r) {
                if (sizes[r] <= c0) continue;
                const uint64_t n = std::min(kPiece, sizes[r] - c0);
                const void *src = r == rank ? (const uint8_t *)send + c0 : d + off[r] + c0;
                NCCL_OK(rccl().Broadcast(src, d + off[r] + c0, n, ncclUint8, r, comm, ctx->stream));
            }
            NCCL_OK(rccl().GroupEnd());
        }
        sync();
    }
};

// ------------------------------------------------------------------- SHM ----
constexpr int kMaxRanks = 64;

struct ShmHeader {
    std::atomic<uint32_t> arrived;
    std::atomic<uint32_t> generation;
    std::atomic<uint32_t> attached;
    uint32_t world;
    uint64_t slot_bytes;
    uint64_t pub[kMaxRanks];  // per-rank published value of the current operation
    int32_t pid[kMaxRanks];   // each rank's process (a rank that died ends the others' waits)
};
static_assert(std::atomic<uint32_t>::is_always_lock_free, "process-shared atomics must be lock-free");

struct ShmComm final : Comm {
    mcaat_ctx *ctx;  // may be null: host collectives only
    std::string name;
    ShmHeader *hdr = nullptr;
    uint8_t *slots = nullptr;
    size_t map_bytes = 0;
    uint64_t slot = 0;
    double timeout_s = 900.0;

    ShmComm(mcaat_ctx *c, int world_, int rank_, const char *nm, uint64_t slot_bytes) : ctx(c), name(nm) {
        world = world_;
        rank = rank_;
        slot = std::max<uint64_t>(4096, (slot_bytes + 4095) & ~4095ULL);
        if (const char *e = getenv("MCAAT_COMM_TIMEOUT")) timeout_s = std::max(1.0, atof(e));
        const uint64_t hb = (sizeof(ShmHeader) + 4095) & ~4095ULL;
        map_bytes = hb + slot * (uint64_t)world;
        int fd = -1;
        const auto t0 = std::chrono::steady_clock::now();
        if (rank == 0) {
            fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
            if (fd < 0) throw Error(MCAAT_E_IO, "shm_open(" + name + ") failed (name in use?)");
            if (ftruncate(fd, (off_t)map_bytes) != 0) {
                close(fd);
                shm_unlink(name.c_str());
                throw Error(MCAAT_E_NOMEM, "ftruncate of the shared segment failed");
            }
        } else {
            // rank 0 creates and sizes the segment; the others wait for it
            for (;;) {
                fd = shm_open(name.c_str(), O_RDWR, 0600);
                if (fd >= 0) {
                    struct stat st;
                    if (fstat(fd, &st) == 0 && (uint64_t)st.st_size == map_bytes) break;
                    close(fd);
                    fd = -1;
                }
                check_timeout(t0, "attach");
                std::this_thread::sleep_for(std::chrono::milliseconds(2));
            }
        }
        void *p = mmap(nullptr, map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) throw Error(MCAAT_E_NOMEM, "mmap of the shared segment failed");
        hdr = (ShmHeader *)p;
        slots = (uint8_t *)p + hb;
        if (rank == 0) {
            hdr->world = (uint32_t)world;
            hdr->slot_bytes = slot;
        }
        hdr->pid[rank] = (int32_t)getpid();
        hdr->attached.fetch_add(1, std::memory_order_acq_rel);
        while (hdr->attached.load(std::memory_order_acquire) < (uint32_t)world) {
            check_timeout(t0, "attach");
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
        barrier();
        if (rank == 0) shm_unlink(name.c_str());  // the mappings stay; nothing is left behind
    }
    ~ShmComm() override {
        if (hdr) munmap(hdr, map_bytes);
    }
    const char *kind() const override { return "shm"; }

    void check_timeout(std::chrono::steady_clock::time_point t0, const char *what) const {
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (s > timeout_s)
            throw Error(MCAAT_E_IO, std::string("shared-memory comm: ") + what + " timed out (a rank is missing?)");
    }
    // a rank whose process has exited (e.g. it failed an allocation) will never arrive: the first
    // such rank, or -1
    int dead_peer() const {
        if (!hdr || hdr->attached.load(std::memory_order_acquire) < (uint32_t)world) return -1;
        for (int r = 0; r < world; ++r)
            if (r != rank && hdr->pid[r] > 0 && !alive(hdr->pid[r])) return r;
        return -1;
    }
    // gone, or exited and not yet reaped by its parent (a zombie still answers kill(pid, 0))
    static bool alive(int32_t pid) {
        if (kill(pid, 0) != 0 && errno == ESRCH) return false;
        char path[64], buf[256];
        snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
        FILE *f = fopen(path, "r");
        if (!f) return true;  // no /proc: kill's answer stands
        const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
        fclose(f);
        buf[n] = 0;
        const char *p = strrchr(buf, ')');  // "pid (comm) state ..."
        return !(p && p[1] == ' ' && (p[2] == 'Z' || p[2] == 'X'));
    }

    void barrier() override {
        Counted cc__(*this);
        const uint32_t g = hdr->generation.load(std::memory_order_acquire);
        if (hdr->arrived.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)world - 1) {
            hdr->arrived.store(0, std::memory_order_relaxed);
            hdr->generation.fetch_add(1, std::memory_order_acq_rel);
            return;
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 0; hdr->generation.load(std::memory_order_acquire) == g; ++spin) {
            if (spin < 1024) continue;
            if ((spin & 1023) == 0) {
                check_timeout(t0, "barrier");
                // every other rank stops waiting for a rank that exited, instead of at the time
                // limit (the barrier may have completed just before that rank left: re-read it)
                if ((spin & 0xFFFFF) == 0) {
                    const int d = dead_peer();
                    if (d >= 0 && hdr->generation.load(std::memory_order_acquire) == g)
                        throw Error(MCAAT_E_IO, "shared-memory comm: rank " + std::to_string(d) + " exited (barrier)");
                }
            }
            sched_yield();
        }
    }

    // every rank publishes one value; returns all of them (rank order)
    std::vector<uint64_t> exchange(uint64_t v) {
        hdr->pub[rank] = v;
        barrier();
        std::vector<uint64_t> all(hdr->pub, hdr->pub + world);
        barrier();  // nobody overwrites pub before everyone has read it
        return all;
    }

    uint8_t *slot_of(int r) const { return slots + slot * (uint64_t)r; }

    // a device-to-device copy that has landed when this returns: ordered on the context's
    // stream (the caller's kernels run there) and waited for. A plain hipMemcpy between two
    // device buffers returns before the copy completes and runs on the null stream, which the
    // context's non-blocking stream does not wait for: with one rank (nothing but this copy in
    // an exchange) the next kernels read the buffer while it was still being written.
    void d2d(void *dst, const void *src, uint64_t n) {
        HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, ctx->stream));
        HIP_OK(hipStreamSynchronize(ctx->stream));
    }
    // copies between host or device memory and a slot (ctx null: host memory only)
    // (device sides on the context's stream and waited for: a host-to-device hipMemcpy from
    // pageable memory may return before its DMA has landed)
    void put(uint8_t *dst, const void *src, uint64_t n, bool dev) {
        if (!n) return;
        if (dev) {
            HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, ctx->stream));
            HIP_OK(hipStreamSynchronize(ctx->stream));
        } else {
            memcpy(dst, src, n);
        }
    }
    void get(void *dst, const uint8_t *src, uint64_t n, bool dev) {
        if (!n) return;
        if (dev) {
            HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, ctx->stream));
            HIP_OK(hipStreamSynchronize(ctx->stream));
        } else {
            memcpy(dst, src, n);
        }
    }

    // all-gather of sizes[r] bytes per rank (known to all) through the slots, in rounds
    void gather_through_slots(const void *send, void *recv, const uint64_t *sizes, bool dev) {
        const auto off = offsets_of(sizes, world);
        uint64_t most = 0;
        for (int r = 0; r < world; ++r) most = std::max(most, sizes[r]);
        for (uint64_t c0 = 0; c0 < most; c0 += slot) {
            if (sizes[rank] > c0) put(slot_of(rank), (const uint8_t *)send + c0, std::min(slot, sizes[rank] - c0), dev);
            barrier();
            for (int r = 0; r < world; ++r) {
                if (sizes[r] <= c0) continue;
                const uint64_t n = std::min(slot, sizes[r] - c0);
                uint8_t *dst = (uint8_t *)recv + off[r] + c0;
                if (r == rank) {
                    if (dev) d2d(dst, (const uint8_t *)send + c0, n);
                    else memcpy(dst, (const uint8_t *)send + c0, n);
                } else {
                    get(dst, slot_of(r), n, dev);
                }
            }
            barrier();
        }
    }

    void allgather_dev_words(const uint64_t *dev, int n, std::vector<uint64_t> &out) override {
        Counted cc__(*this);
        need_ctx();  // the stream's writes of dev are done
        std::vector<uint64_t> mine(n);
        if (n) HIP_OK(hipMemcpy(mine.data(), dev, 8 * (size_t)n, hipMemcpyDeviceToHost));
        out = allgather_vec(mine);
    }

    void allgatherv_host(const void *send, uint64_t bytes, std::vector<uint8_t> &out,
                         std::vector<uint64_t> &sizes) override {
        Counted cc__(*this);
        sizes = exchange(bytes);
        const auto off = offsets_of(sizes.data(), world);
        out.resize(off[world]);
        gather_through_slots(send, out.data(), sizes.data(), false);
    }

    void need_ctx() const {
        if (!ctx) throw Error(MCAAT_E_INVALID, "shared-memory comm without a context moves host memory only");
        mcaat::bind(ctx);
        HIP_OK(hipStreamSynchronize(ctx->stream));
    }

    void alltoallv_dev(const void *send, const uint64_t *send_bytes, void *recv, const uint64_t *recv_bytes,
                       const uint64_t *send_off, const uint64_t *recv_off) override {
        Counted cc__(*this);
        if (coll_depth == 1) ++n_queued;
        need_ctx();
        auto so = offsets_of(send_bytes, world), ro = offsets_of(recv_bytes, world);
        if (send_off) so.assign(send_off, send_off + world);
        if (recv_off) ro.assign(recv_off, recv_off + world);
        // shift s: this rank sends to rank+s and receives from rank-s
        for (int s = 0; s < world; ++s) {
            const int to = (rank + s) % world, from = (rank - s + world) % world;
            const uint8_t *src = (const uint8_t *)send + so[to];
            uint8_t *dst = (uint8_t *)recv + ro[from];
            if (s == 0) {
                if (send_bytes[rank] != recv_bytes[rank]) throw Error(MCAAT_E_INVALID, "alltoallv: self sizes differ");
                if (send_bytes[rank]) d2d(dst, src, send_bytes[rank]);
                continue;
            }
            const auto out_n = exchange(send_bytes[to]);
            uint64_t most = 0;
            for (int r = 0; r < world; ++r) most = std::max(most, out_n[r]);
            for (uint64_t c0 = 0; c0 < most; c0 += slot) {
                if (send_bytes[to] > c0) put(slot_of(rank), src + c0, std::min(slot, send_bytes[to] - c0), true);
                barrier();
                if (recv_bytes[from] > c0) get(dst + c0, slot_of(from), std::min(slot, recv_bytes[from] - c0), true);
                barrier();
            }
        }
    }

    void allgatherv_dev(const void *send, void *recv, const uint64_t *sizes) override {
        Counted cc__(*this);
        need_ctx();
        gather_through_slots(send, recv, sizes, true);
    }

    // bytes [a, a + n) of the concatenation of segments `sg` (device) into host memory
    void put_range(uint8_t *dst, const std::vector<Seg> &sg, uint64_t a, uint64_t n) {
        uint64_t o = 0;
        for (const Seg &g : sg) {
            if (n == 0) break;
            if (a < o + g.bytes) {
                const uint64_t off = a - o, m = std::min(n, g.bytes - off);
                HIP_OK(hipMemcpyAsync(dst, (const uint8_t *)g.p + off, m, hipMemcpyDeviceToHost, ctx->stream));
                dst += m;
                a += m;
                n -= m;
            }
            o += g.bytes;
        }
        HIP_OK(hipStreamSynchronize(ctx->stream));
    }

    // the segments go through the slots as the plain all-to-all's messages do (no device staging
    // copy: ranks sharing one GPU cannot afford a third copy of the descriptors)
    void alltoallv_dev_segs(const std::vector<std::vector<Seg>> &send, void *out,
                            const std::vector<std::vector<uint64_t>> &recv) override {
        Counted cc__(*this);
        need_ctx();
        std::vector<uint64_t> sb(world, 0), rb(world, 0);
        for (int q = 0; q < world; ++q) {
            for (const Seg &g : send[q]) sb[q] += g.bytes;
            for (const uint64_t n : recv[q]) rb[q] += n;
        }
        const auto ro = offsets_of(rb.data(), world);
        for (int s = 0; s < world; ++s) {
            const int to = (rank + s) % world, from = (rank - s + world) % world;
            uint8_t *dst = (uint8_t *)out + ro[from];
            if (s == 0) {
                if (sb[rank] != rb[rank]) throw Error(MCAAT_E_INVALID, "alltoallv_segs: self sizes differ");
                for (const Seg &g : send[rank]) {
                    if (g.bytes) HIP_OK(hipMemcpyAsync(dst, g.p, g.bytes, hipMemcpyDeviceToDevice, ctx->stream));
                    dst += g.bytes;
                }
                HIP_OK(hipStreamSynchronize(ctx->stream));
                continue;
            }
            const auto out_n = exchange(sb[to]);
            uint64_t most = 0;
            for (int r = 0; r < world; ++r) most = std::max(most, out_n[r]);
            for (uint64_t c0 = 0; c0 < most; c0 += slot) {
                if (sb[to] > c0) put_range(slot_of(rank), send[to], c0, std::min(slot, sb[to] - c0));
                barrier();
                if (rb[from] > c0) get(dst + c0, slot_of(from), std::min(slot, rb[from] - c0), true);
                barrier();
            }
        }
    }
};

}  // namespace

std::unique_ptr<Comm> comm_rccl(mcaat_ctx *ctx, int world, int rank, const uint8_t *id) {
    return std::make_unique<RcclComm>(ctx, world, rank, id);
}

std::unique_ptr<Comm> comm_shm(mcaat_ctx *ctx, int world, int rank, const char *name, uint64_t slot_bytes) {
    if (world > kMaxRanks) throw Error(MCAAT_E_INVALID, "shared-memory comm: at most 64 ranks");
    return std::make_unique<ShmComm>(ctx, world, rank, name, slot_bytes);
}

// every rank's schedule for random segment lists (world ranks, piece bytes): each pair's j-th send
// piece on one side equals the j-th receive piece on the other, pieces tile the segments in order,
// and the receive pieces tile each source's block of `out`; returns the most rounds of any rank
uint64_t comm_schedule_check(int world, uint64_t seed, uint64_t piece) {
    if (world < 1 || world > 64 || !piece) throw Error(MCAAT_E_INVALID, "schedule check: bad arguments");
    uint64_t x = seed * 0x9E3779B97F4A7C15ULL + 1;
    auto rnd = [&](uint64_t m) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        return m ? x % m : 0;
    };
    // sz[r][q]: the segment sizes rank r sends to q (empty lists, empty segments, and sizes around
    // multiples of the piece included)
    std::vector<std::vector<std::vector<uint64_t>>> sz(world, std::vector<std::vector<uint64_t>>(world));
    for (int r = 0; r < world; ++r)
        for (int q = 0; q < world; ++q) {
            const uint64_t ns = rnd(5);
            for (uint64_t i = 0; i < ns; ++i) {
                const uint64_t kind = rnd(4);
                sz[r][q].push_back(kind == 0 ? 0 : kind == 1 ? piece * (1 + rnd(3)) + rnd(3) - 1 : rnd(4 * piece) + 1);
            }
        }
    std::vector<std::vector<std::vector<SegPiece>>> S(world), Rv(world);
    uint64_t most = 0;
    for (int r = 0; r < world; ++r) {
        std::vector<std::vector<uint64_t>> recv(world);
        for (int q = 0; q < world; ++q) recv[q] = sz[q][r];
        size_t rounds = 0;
        seg_schedule(world, r, sz[r], recv, piece, S[r], Rv[r], rounds);
        most = std::max<uint64_t>(most, rounds);
        // receive pieces tile each source's block, in order
        uint64_t off = 0;
        for (int q = 0; q < world; ++q) {
            uint64_t tot = 0;
            for (uint64_t n : recv[q]) tot += n;
            if (q != r) {
                uint64_t at = off;
                for (const SegPiece &p : Rv[r][q]) {
                    if (p.off != at || p.n == 0 || p.n > piece) throw Error(MCAAT_E_INVALID, "schedule check: receive pieces do not tile");
                    at += p.n;
                }
                if (at != off + tot) throw Error(MCAAT_E_INVALID, "schedule check: receive pieces miss bytes");
            }
            off += tot;
        }
        // send pieces tile the segments in order
        for (int q = 0; q < world; ++q) {
            if (q == r) continue;
            size_t j = 0;
            for (size_t i = 0; i < sz[r][q].size(); ++i) {
                uint64_t at = 0;
                while (at < sz[r][q][i]) {
                    if (j >= S[r][q].size() || S[r][q][j].seg != (int)i || S[r][q][j].off != at)
                        throw Error(MCAAT_E_INVALID, "schedule check: send pieces do not tile");
                    at += S[r][q][j++].n;
                }
                if (at != sz[r][q][i]) throw Error(MCAAT_E_INVALID, "schedule check: send pieces overrun");
            }
            if (j != S[r][q].size()) throw Error(MCAAT_E_INVALID, "schedule check: extra send pieces");
        }
    }
    // pairing: the j-th piece r -> q is the j-th piece q receives from r, same size
    for (int r = 0; r < world; ++r)
        for (int q = 0; q < world; ++q) {
            if (q == r) continue;
            if (S[r][q].size() != Rv[q][r].size()) throw Error(MCAAT_E_INVALID, "schedule check: piece counts differ");
            for (size_t j = 0; j < S[r][q].size(); ++j)
                if (S[r][q][j].n != Rv[q][r][j].n) throw Error(MCAAT_E_INVALID, "schedule check: paired pieces differ");
        }
    return most;
}

void comm_unique_id(uint8_t *out) {
    ncclUniqueId u;
    NCCL_OK(rccl().GetUniqueId(&u));
    memcpy(out, u.internal, NCCL_UNIQUE_ID_BYTES);
}

}  // namespace mcaat
