// fastq_ingest.hip — FASTQ(.gz/.bz2) -> 2-bit read library in HBM.
//
// Replaces SDBGBuild::BuildLib / SequenceLibCollection::Build (sdbg_build.cpp:82-115, the
// MEGAHIT buildlib step) for FASTQ inputs, and builds in the same pass the mapping view that
// get_reads re-parses the FASTQ for (reads.cpp:20-52, 88-130). The host only moves bytes: a
// reader task fills pinned chunks (zlib / libbz2 inflate .gz / .bz2; plain files are copied straight into
// the chunk by four pread() threads) while the GPU parses the previous chunk:
//
//  1. k_fq_nlcount   one lane per 64-byte segment (4 x 16-B loads): number of '\n' bytes
//                    (SWAR zero-byte count); exclusive scan -> line index per segment.
//  2. k_fq_nlpos     the same segments again: position of every '\n' (line starts).
//                    Records are 4 lines (header '@', sequence, '+', quality); the bytes
//                    after the last complete record carry over to the next chunk.
//  3. k_fq_records   one lane per record: header check, sequence bounds ('\r' stripped),
//                    ACGT base count and maximal-run count (counting view: non-ACGT symbols
//                    split a read), sequence length (mapping view); three exclusive scans.
//  4. k_fq_emit      one lane per record: packs the counting view (runs -> reads, global
//                    read offsets) and the mapping view (second file reversed and
//                    complemented; A/C/G -> 0/1/2, anything else -> 3, reads.cpp:44-52) into
//                    the growing device streams; words shared with a neighbouring record are
//                    merged with atomicOr, whole words are stored.
//
// Bytes per chunk byte (roofline, HBM): ~2.5 B read (two newline passes + the record
// passes) + 0.25 B per sequence byte written per view. The ingest is PCIe/host-read bound
// (text crosses PCIe once); the parse runs at HBM speed. FASTA (multi-line records) stays
// on the host parser in capi.hip.
#include <hipcub/hipcub.hpp>
#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <atomic>
#include <future>
#include <memory>
#include <string>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <thread>

#include "internal.h"

namespace mcaat {
namespace {

constexpr int kBlock = 256;
constexpr uint32_t kSeg = 64;  // bytes per lane in the newline passes

// zero-byte mask of a 32-bit word: bit 7 of each byte that is zero (exact, no carries)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
    const uint32_t y = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    return ~(y | v | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t nl_mask(uint32_t v) { return zero_bytes(v ^ 0x0A0A0A0Au); }

__global__ void k_fq_nlcount(const uint8_t *buf, uint32_t nseg, uint32_t *cnt) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += stride) {
        const uint4 *p = reinterpret_cast<const uint4 *>(buf + (size_t)s * kSeg);
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = p[q];
            c += __popc(nl_mask(v.x)) + __popc(nl_mask(v.y)) + __popc(nl_mask(v.z)) + __popc(nl_mask(v.w));
        }
        cnt[s] = c;
    }
}

__global__ void k_fq_nlpos(const uint8_t *buf, uint32_t nseg, const uint32_t *first, uint32_t *nl) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += stride) {
        const uint4 *p = reinterpret_cast<const uint4 *>(buf + (size_t)s * kSeg);
        uint32_t o = first[s];
        const uint32_t base = s * kSeg;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = p[q];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t m = nl_mask(w[j]);
                while (m) {
                    const int b = __builtin_ctz(m) >> 3;
                    nl[o++] = base + 16 * q + 4 * j + b;
                    m &= m - 1;
                }
            }
        }
    }
}

// counting-view code: A/C/G/T in either case, -1 splits the read (capi.hip Packer)
__device__ __forceinline__ int count_code(uint8_t c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return -1;
    }
}
// mapping-view code (k_mer_to_node_id, reads.cpp:44-52)
__device__ __forceinline__ uint32_t map_code(uint8_t c) { return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : 3; }
// complement then code (reverse_pair_ends_sequence, reads.cpp:20-31: only A/C/G/T change)
__device__ __forceinline__ uint32_t map_code_rc(uint8_t c) { return c == 'T' ? 0 : c == 'G' ? 1 : c == 'C' ? 2 : 3; }

// a lane's sequential byte readers over the chunk (4-byte aligned loads instead of one load
// per byte; the chunk buffer is 256-B aligned and padded, so reading up to 3 bytes past the
// end is in bounds)
struct Fwd {
    const uint32_t *w;
    uint32_t cur;
    int avail;
    __device__ Fwd(const uint8_t *buf, uint32_t pos) {
        w = reinterpret_cast<const uint32_t *>(buf + (pos & ~3u));
        cur = *w++ >> (8 * (pos & 3));
        avail = 4 - (int)(pos & 3);
    }
    __device__ __forceinline__ uint8_t next() {
        if (!avail) {
            cur = *w++;
            avail = 4;
        }
        const uint8_t c = (uint8_t)cur;
        cur >>= 8;
        --avail;
        return c;
    }
};
struct Bwd {  // from pos downwards
    const uint32_t *w;
    uint32_t cur;
    int idx;
    __device__ Bwd(const uint8_t *buf, uint32_t pos) {
        w = reinterpret_cast<const uint32_t *>(buf + (pos & ~3u));
        cur = *w;
        idx = (int)(pos & 3);
    }
    __device__ __forceinline__ uint8_t next() {
        if (idx < 0) {
            cur = *--w;
            idx = 3;
        }
        return (uint8_t)(cur >> (8 * idx--));
    }
};

enum : uint32_t { kBadHeader = 1, kDiffer = 2 };

// per record: sequence start, length, counting-view bases and runs
__global__ void k_fq_records(const uint8_t *buf, const uint32_t *nl, uint32_t n_rec, uint32_t *sbeg, uint32_t *slen,
                             uint32_t *nbase, uint32_t *nrun, uint32_t *flags) {
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t fl = 0;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n_rec; r += stride) {
        const uint32_t h = r ? nl[4 * r - 1] + 1 : 0;
        if (buf[h] != '@') fl |= kBadHeader;
        const uint32_t s = nl[4 * r] + 1;
        uint32_t e = nl[4 * r + 1];
        if (e > s && buf[e - 1] == '\r') --e;
        // '+' line, and a quality line as long as the sequence: otherwise not 4-line FASTQ
        // (wrapped lines), which the host kseq-style reader takes
        const uint32_t qs = nl[4 * r + 2] + 1;
        uint32_t qe = nl[4 * r + 3];
        if (qe > qs && buf[qe - 1] == '\r') --qe;
        if (buf[nl[4 * r + 1] + 1] != '+' || qe - qs != e - s) fl |= kBadHeader;
        uint32_t bases = 0, runs = 0;
        bool in = false, differ = false;
        Fwd rd(buf, s);
        for (uint32_t i = s; i < e; ++i) {
            const uint8_t c = rd.next();
            if (count_code(c) >= 0) {
                ++bases;
                runs += !in;
                in = true;
            } else {
                in = false;
            }
            differ |= c != 'A' && c != 'C' && c != 'G' && c != 'T';
        }
        // the mapping view equals the counting view only if this record is one ACGT run
        if (differ || runs != 1) fl |= kDiffer;
        sbeg[r] = s;
        slen[r] = e - s;
        nbase[r] = bases;
        nrun[r] = runs;
    }
    if (fl) atomicOr(flags, fl);
}

// appends 2-bit symbols at consecutive stream positions; a word this lane does not fill
// completely may be shared with another record and is merged with atomicOr
struct PackWriter {
    uint64_t *out;
    uint64_t pos;
    uint64_t acc = 0;
    bool partial;
    __device__ PackWriter(uint64_t *o, uint64_t p) : out(o), pos(p), partial((p & 31) != 0) {}
    __device__ __forceinline__ void put(uint32_t b) {
        acc |= (uint64_t)b << (2 * (pos & 31));
        if ((++pos & 31) == 0) {
            uint64_t *w = out + ((pos - 1) >> 5);
            if (partial) {
                if (acc) atomicOr((unsigned long long *)w, (unsigned long long)acc);
            } else {
                *w = acc;
            }
            acc = 0;
            partial = false;
        }
    }
    __device__ __forceinline__ void finish() {
        if ((pos & 31) && acc) atomicOr((unsigned long long *)(out + (pos >> 5)), (unsigned long long)acc);
    }
};

__global__ void k_fq_emit(const uint8_t *buf, uint32_t n_rec, const uint32_t *sbeg, const uint32_t *slen,
                          const uint32_t *boff, const uint32_t *roff, const uint32_t *qoff, uint64_t g_base,
                          uint64_t g_read, uint64_t g_qbase, uint64_t g_rec, int reverse, uint64_t *packed,
                          uint64_t *offsets, uint64_t *qpacked, uint64_t *qoffsets) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n_rec; r += stride) {
        const uint32_t sb = sbeg[r];
        const uint32_t L = slen[r];
        // counting view: maximal ACGT runs are reads
        PackWriter pw(packed, g_base + boff[r]);
        uint64_t ri = g_read + roff[r];
        bool in = false;
        Fwd rd(buf, sb);
        for (uint32_t i = 0; i < L; ++i) {
            const int b = count_code(rd.next());
            if (b >= 0) {
                pw.put((uint32_t)b);
                in = true;
            } else if (in) {
                offsets[1 + ri++] = pw.pos;
                in = false;
            }
        }
        if (in) offsets[1 + ri] = pw.pos;
        pw.finish();
        // mapping view: one entry per record
        if (qpacked) {
            PackWriter qw(qpacked, g_qbase + qoff[r]);
            if (!reverse) {
                Fwd rq(buf, sb);
                for (uint32_t i = 0; i < L; ++i) qw.put(map_code(rq.next()));
            } else if (L) {
                Bwd rq(buf, sb + L - 1);
                for (uint32_t i = 0; i < L; ++i) qw.put(map_code_rc(rq.next()));
            }
            qw.finish();
            qoffsets[1 + g_rec + r] = qw.pos;
        }
    }
}

__global__ void k_fq_fixed_len(const uint64_t *off, uint64_t n, uint64_t L, uint32_t *bad) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    bool b = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) b |= off[i] != i * L;
    if (b) atomicOr(bad, 1u);
}

void scan_u32(mcaat_ctx *ctx, const uint32_t *in, uint32_t *out, uint64_t n, DevBuf<uint8_t> &tmp) {
    size_t need = 0;
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, in, out, (size_t)n, ctx->stream));
    if (need > tmp.bytes()) tmp.alloc(need);
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(tmp.p, need, in, out, (size_t)n, ctx->stream));
}

// grows a zero-filled device stream, keeping its first `used` elements
void grow(mcaat_ctx *ctx, DevBuf<uint64_t> &b, uint64_t used, uint64_t need) {
    if (need <= b.n) return;
    DevBuf<uint64_t> nb(std::max<uint64_t>(need, b.n + b.n / 2));
    HIP_OK(hipMemsetAsync(nb.p, 0, nb.bytes(), ctx->stream));
    if (used) HIP_OK(hipMemcpyAsync(nb.p, b.p, 8 * used, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    b = std::move(nb);
}

// Source of input bytes: InStream for compressed files (one inflate stream), parallel pread()
// for plain files (one thread copies page-cache data at ~13 GB/s; eight reach ~38 GB/s end to end).
struct Source {
    std::unique_ptr<InStream> z;  // gzip / bzip2
    int fd = -1;
    uint64_t off = 0;
    const char *path;
    uint64_t end = ~0ULL;  // plain files: read [off, end) only (a rank's part of the file)
    // [begin, end) of a plain file; a compressed file is read whole (begin = 0, end = ~0)
    explicit Source(const char *p, uint64_t begin = 0, uint64_t end_ = ~0ULL) : off(begin), path(p), end(end_) {
        if (is_compressed_file(p)) {
            if (begin != 0 || end_ != ~0ULL) throw Error(MCAAT_E_INVALID, "a compressed input cannot be split");
            z.reset(new InStream(p));
            return;
        }
        fd = open(p, O_RDONLY);
        if (fd < 0) throw Error(MCAAT_E_IO, std::string("cannot open ") + p);
        posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
    }
    ~Source() {
        if (fd >= 0) close(fd);
    }
    Source(const Source &) = delete;
    Source &operator=(const Source &) = delete;
    size_t read(uint8_t *dst, size_t n) {
        if (z) return z->read(dst, n);
        n = (size_t)std::min<uint64_t>(n, end > off ? end - off : 0);
        if (!n) return 0;
        // 8 by default: the C3 FASTQ (92 GB in tmpfs) reads at 38 GB/s end to end with 8 or 16
        // threads, 12.6 GB/s with 4; MCAAT_FASTQ_THREADS overrides (1..32)
        static const int kThreads = [] {
            const char *e = getenv("MCAAT_FASTQ_THREADS");
            const int v = e ? atoi(e) : 8;
            return v < 1 ? 1 : v > 32 ? 32 : v;
        }();
        const size_t piece = (n + kThreads - 1) / kThreads;
        size_t got[32] = {};
        bool err[32] = {};
        auto job = [&](int t) {
            const size_t a = std::min(n, t * piece), b = std::min(n, a + piece);
            size_t g = 0;
            while (a + g < b) {
                const ssize_t r = pread(fd, dst + a + g, b - a - g, (off_t)(off + a + g));
                if (r < 0) { err[t] = true; break; }
                if (r == 0) break;
                g += (size_t)r;
            }
            got[t] = g;
        };
        std::thread th[31];
        for (int t = 1; t < kThreads; ++t) th[t - 1] = std::thread(job, t);
        job(0);
        for (int t = 1; t < kThreads; ++t) th[t - 1].join();
        size_t total = 0;
        for (int t = 0; t < kThreads; ++t) {
            if (err[t]) throw Error(MCAAT_E_IO, std::string("read error in ") + path);
            const size_t a = std::min(n, t * piece), b = std::min(n, a + piece);
            total += got[t];
            if (got[t] < b - a) break;  // end of file inside piece t: later pieces read nothing
        }
        off += total;
        return total;
    }
};

bool is_space(uint8_t c) { return c == '\n' || c == '\r' || c == ' ' || c == '\t'; }

}  // namespace

size_t fastq_chunk_bytes() {
    if (const char *e = getenv("MCAAT_FASTQ_CHUNK")) {
        const long long v = atoll(e);
        // chunk positions are 32-bit: keep chunk + carry reserve well below 4 GiB
        if (v >= 256) return (size_t)std::min<long long>(v, 1LL << 30);
    }
    return size_t(256) << 20;
}

// All inputs are FASTQ (checked by the caller). Files are concatenated; records of files
// after the first are reversed and complemented in the mapping view (paired-end R2).
void ingest_fastq(mcaat_ctx *ctx, const char *const *files, int n_files, mcaat_reads *r,
                  const std::vector<std::pair<uint64_t, uint64_t>> *ranges) {
    // plain files of well-formed upper-case ACGT records: packed by host threads (PCIe carries
    // 2 bits per base); any other input falls through to the text parser below
    if (fastq_hostpack(ctx, files, n_files, ranges, r)) return;
    const size_t CH = fastq_chunk_bytes();
    const size_t R = std::max<size_t>(CH / 4, 4096);  // carry reserve: the longest record that fits
    const size_t cap = R + CH + 2 * kSeg;

    uint64_t est = 0;  // stream capacity estimate from the input sizes (grown on demand)
    for (int i = 0; i < n_files; ++i) {
        struct stat st;
        const std::string path(files[i]);
        const bool gz = (path.size() > 3 && path.compare(path.size() - 3, 3, ".gz") == 0) ||
                        (path.size() > 4 && path.compare(path.size() - 4, 4, ".bz2") == 0);
        if (stat(files[i], &st) == 0) {
            uint64_t sz = (uint64_t)st.st_size;
            if (ranges) sz = std::min(sz, (*ranges)[i].second) - std::min(sz, (*ranges)[i].first);
            est += sz * (gz ? 4 : 1);
        }
    }
    DevBuf<uint64_t> packed(est / 64 + 1024), offsets(est / 256 + 1024);
    DevBuf<uint64_t> qpacked(est / 64 + 1024), qoffsets(est / 256 + 1024);
    for (auto *b : {&packed, &offsets, &qpacked, &qoffsets}) HIP_OK(hipMemsetAsync(b->p, 0, b->bytes(), ctx->stream));
    uint64_t n_bases = 0, n_reads = 0, q_bases = 0, n_rec = 0;
    uint32_t flags_all = 0;

    if (ctx->pinned_bytes < cap) {
        for (auto *&p : ctx->pinned) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
        }
        ctx->pinned_bytes = 0;
        for (auto *&p : ctx->pinned) HIP_OK(hipHostMalloc((void **)&p, cap, hipHostMallocDefault));
        ctx->pinned_bytes = cap;
    }
    uint8_t *hb[2] = {ctx->pinned[0], ctx->pinned[1]};
    DevBuf<uint8_t> dbufs[2];
    dbufs[0].alloc(cap);
    dbufs[1].alloc(cap);
    struct CopyStream {  // uploads overlap the parse of the previous chunk
        hipStream_t s = nullptr;
        hipEvent_t ev[2] = {nullptr, nullptr};    // upload into dbufs[x] complete
        hipEvent_t done[2] = {nullptr, nullptr};  // the parse of dbufs[x] complete (buffer free)
        CopyStream() {
            HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            for (auto &e : ev) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            for (auto &e : done) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        ~CopyStream() {
            if (s) (void)hipStreamSynchronize(s);
            for (auto &e : ev)
                if (e) (void)hipEventDestroy(e);
            for (auto &e : done)
                if (e) (void)hipEventDestroy(e);
            if (s) (void)hipStreamDestroy(s);
        }
    } cs;
    for (auto &e : cs.done) HIP_OK(hipEventRecord(e, ctx->stream));
    hipEvent_t *up_ev = cs.ev;
    const uint64_t max_seg = cap / kSeg + 1;
    DevBuf<uint32_t> cnt(max_seg + 1), first(max_seg + 1), nl(cap + 16);  // every byte may be a newline
    DevBuf<uint32_t> sbeg, slen, nbase, nrun, boff, roff, qoff;
    DevBuf<uint32_t> meta(8);
    DevBuf<uint8_t> tmp(1 << 20);
    uint32_t *hmeta = nullptr;
    HIP_OK(hipHostMalloc((void **)&hmeta, 64, hipHostMallocDefault));
    struct MetaFree {
        uint32_t *p;
        ~MetaFree() { (void)hipHostFree(p); }
    } meta_free{hmeta};

    // chunk x: host bytes [start, start+total) of hb[x] (carry + new data, blank lines trimmed
    // at the file's ends) uploaded on the copy stream into dbufs[x]; up_ev[x] marks completion
    auto prepare = [&](int x, size_t carry_x, size_t n_x, bool eof_x, bool first_x, uint8_t *&start_x,
                       size_t &total_x) {
        start_x = hb[x] + R - carry_x;
        total_x = carry_x + n_x;
        if (first_x)  // leading blank lines
            while (total_x && is_space(*start_x)) ++start_x, --total_x;
        if (eof_x) {  // trailing blank lines; the last line gets its newline
            while (total_x && is_space(start_x[total_x - 1])) --total_x;
            if (total_x) start_x[total_x++] = '\n';
        }
        if (total_x) {
            const size_t padded = (total_x + kSeg - 1) / kSeg * kSeg + kSeg;
            // dbufs[x] is free once the kernels of the chunk it held last have run
            HIP_OK(hipStreamWaitEvent(cs.s, cs.done[x], 0));
            HIP_OK(hipMemcpyAsync(dbufs[x].p, start_x, total_x, hipMemcpyHostToDevice, cs.s));
            HIP_OK(hipMemsetAsync(dbufs[x].p + total_x, 0, padded - total_x, cs.s));
            HIP_OK(hipEventRecord(up_ev[x], cs.s));
        }
    };
    std::vector<uint64_t> file_records;
    for (int fi = 0; fi < n_files; ++fi) {
        const uint64_t rec_before = n_rec;
        struct FileDone {  // records of this file, however the loop below is left
            std::vector<uint64_t> &v;
            const uint64_t &n, before;
            ~FileDone() { v.push_back(n - before); }
        } file_done{file_records, n_rec, rec_before};
        if (ranges && (*ranges)[fi].first >= (*ranges)[fi].second) continue;  // no part of this file
        Source src(files[fi], ranges ? (*ranges)[fi].first : 0, ranges ? (*ranges)[fi].second : ~0ULL);
        int cur = 0;
        size_t n = src.read(hb[cur] + R, CH);
        bool eof = n < CH;
        uint8_t *start = nullptr;
        size_t total = 0;
        prepare(cur, 0, n, eof, true, start, total);
        std::future<size_t> next;
        if (!eof) {
            uint8_t *dst = hb[cur ^ 1] + R;
            next = std::async(std::launch::async, [&src, dst, CH] { return src.read(dst, CH); });
        }
        for (;;) {
            // ---- newline passes (after this chunk's upload)
            const uint32_t nseg = (uint32_t)((total + kSeg - 1) / kSeg);
            if (total) {
                HIP_OK(hipStreamWaitEvent(ctx->stream, up_ev[cur], 0));
                KernelTimer kt(ctx, "fq_parse", 2.0 * (double)total);
                HIP_OK(hipMemsetAsync(cnt.p + nseg, 0, 4, ctx->stream));
                hipLaunchKernelGGL(k_fq_nlcount, dim3(grid_for(nseg, kBlock)), dim3(kBlock), 0, ctx->stream,
                                   dbufs[cur].p, nseg, cnt.p);
                LAUNCH_OK();
                scan_u32(ctx, cnt.p, first.p, (uint64_t)nseg + 1, tmp);
                hipLaunchKernelGGL(k_fq_nlpos, dim3(grid_for(nseg, kBlock)), dim3(kBlock), 0, ctx->stream,
                                   dbufs[cur].p, nseg, first.p, nl.p);
                LAUNCH_OK();
                HIP_OK(hipMemcpyAsync(hmeta, first.p + nseg, 4, hipMemcpyDeviceToHost, ctx->stream));
                HIP_OK(hipStreamSynchronize(ctx->stream));
                kt.stop();
            }
            const uint32_t NL = total ? hmeta[0] : 0;
            const uint32_t nrec = NL / 4;
            if (eof && NL % 4)
                throw FormatError(std::string("not 4-line FASTQ (truncated record, blank or wrapped line): ") + files[fi]);
            size_t consumed = 0;
            if (nrec) {
                HIP_OK(hipMemcpyAsync(hmeta, nl.p + 4 * (uint64_t)nrec - 1, 4, hipMemcpyDeviceToHost, ctx->stream));
                HIP_OK(hipStreamSynchronize(ctx->stream));
                consumed = (size_t)hmeta[0] + 1;
            }
            if (!eof && total - consumed > R)
                throw FormatError(std::string("FASTQ record longer than the chunk reserve (") + std::to_string(R) +
                                  " bytes): " + files[fi]);
            // ---- the next chunk: its carry is known now, so it uploads while this chunk's
            // records are parsed; this chunk's host buffer is free again for the reader
            const bool have_next = !eof;
            uint8_t *nstart = nullptr;
            size_t ntotal = 0;
            bool neof = true;
            if (have_next) {
                const size_t nn = next.get();
                neof = nn < CH;
                const size_t ncarry = total - consumed;
                memcpy(hb[cur ^ 1] + R - ncarry, start + consumed, ncarry);
                prepare(cur ^ 1, ncarry, nn, neof, false, nstart, ntotal);
                if (!neof) {
                    uint8_t *dst = hb[cur] + R;
                    next = std::async(std::launch::async, [&src, dst, CH] { return src.read(dst, CH); });
                }
            }
            // ---- records
            if (nrec) {
                KernelTimer kt(ctx, "fq_records", (double)consumed + 16.0 * nrec);
                if (sbeg.n < (uint64_t)nrec + 1) {
                    const uint64_t m = std::max<uint64_t>((uint64_t)nrec + 1, cap / 64);
                    for (auto *b : {&sbeg, &slen, &nbase, &nrun, &boff, &roff, &qoff}) b->alloc(m);
                }
                HIP_OK(hipMemsetAsync(meta.p, 0, 4, ctx->stream));
                for (auto *b : {&nbase, &nrun, &slen}) HIP_OK(hipMemsetAsync(b->p + nrec, 0, 4, ctx->stream));
                hipLaunchKernelGGL(k_fq_records, dim3(grid_for(nrec, kBlock)), dim3(kBlock), 0, ctx->stream, dbufs[cur].p,
                                   nl.p, nrec, sbeg.p, slen.p, nbase.p, nrun.p, meta.p);
                LAUNCH_OK();
                scan_u32(ctx, nbase.p, boff.p, (uint64_t)nrec + 1, tmp);
                scan_u32(ctx, nrun.p, roff.p, (uint64_t)nrec + 1, tmp);
                scan_u32(ctx, slen.p, qoff.p, (uint64_t)nrec + 1, tmp);
                HIP_OK(hipMemcpyAsync(hmeta + 0, boff.p + nrec, 4, hipMemcpyDeviceToHost, ctx->stream));
                HIP_OK(hipMemcpyAsync(hmeta + 1, roff.p + nrec, 4, hipMemcpyDeviceToHost, ctx->stream));
                HIP_OK(hipMemcpyAsync(hmeta + 2, qoff.p + nrec, 4, hipMemcpyDeviceToHost, ctx->stream));
                HIP_OK(hipMemcpyAsync(hmeta + 3, meta.p, 4, hipMemcpyDeviceToHost, ctx->stream));
                HIP_OK(hipStreamSynchronize(ctx->stream));
                kt.stop();
                const uint32_t cb = hmeta[0], cr = hmeta[1], cq = hmeta[2], fl = hmeta[3];
                if (fl & kBadHeader) throw FormatError(std::string("not 4-line FASTQ (header or '+' line): ") + files[fi]);
                flags_all |= fl;
                if (fi > 0) flags_all |= kDiffer;  // second file: reverse-complemented records
                grow(ctx, packed, (n_bases + 31) / 32 + 1, (n_bases + cb + 31) / 32 + 17);
                grow(ctx, offsets, n_reads + 1, n_reads + cr + 2);
                grow(ctx, qpacked, (q_bases + 31) / 32 + 1, (q_bases + cq + 31) / 32 + 17);
                grow(ctx, qoffsets, n_rec + 1, n_rec + nrec + 2);
                KernelTimer ke(ctx, "fq_emit", (double)consumed + 0.5 * (double)(cb + cq) + 8.0 * (cr + nrec));
                hipLaunchKernelGGL(k_fq_emit, dim3(grid_for(nrec, kBlock)), dim3(kBlock), 0, ctx->stream, dbufs[cur].p, nrec,
                                   sbeg.p, slen.p, boff.p, roff.p, qoff.p, n_bases, n_reads, q_bases, n_rec, fi > 0 ? 1 : 0,
                                   packed.p, offsets.p, qpacked.p, qoffsets.p);
                HIP_OK(hipGetLastError());
                ke.stop();
                n_bases += cb;
                n_reads += cr;
                q_bases += cq;
                n_rec += nrec;
            }
            HIP_OK(hipEventRecord(cs.done[cur], ctx->stream));
            if (!have_next) break;
            cur ^= 1;
            start = nstart;
            total = ntotal;
            eof = neof;
        }
    }
    HIP_OK(hipStreamSynchronize(ctx->stream));

    r->ctx = ctx;
    r->n_reads = n_reads;
    r->n_bases = n_bases;
    r->n_words = (n_bases + 31) / 32;
    r->fixed_len = 0;
    if (n_reads > 0) {
        uint64_t L = 0;
        HIP_OK(hipMemcpy(&L, offsets.p + 1, 8, hipMemcpyDeviceToHost));
        HIP_OK(hipMemsetAsync(meta.p, 0, 4, ctx->stream));
        hipLaunchKernelGGL(k_fq_fixed_len, dim3(grid_for(n_reads + 1, kBlock)), dim3(kBlock), 0, ctx->stream,
                           offsets.p, n_reads, L, meta.p);
        HIP_OK(hipMemcpyAsync(hmeta, meta.p, 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_OK(hipStreamSynchronize(ctx->stream));
        if (!hmeta[0] && L > 0) r->fixed_len = L;
    }
    r->packed = std::move(packed);
    r->offsets = std::move(offsets);
    r->n_records = n_rec;
    r->file_records = file_records;
    r->has_records = (flags_all & kDiffer) != 0;
    if (r->has_records) {
        r->rec_packed = std::move(qpacked);
        r->rec_offsets = std::move(qoffsets);
    }
}

}  // namespace mcaat

namespace mcaat {

// The counting view as 4-line FASTQ ("@r", sequence, "+", all-'I' qualities): record i
// starts at byte 2*offsets[i] + 7*i, so host threads format disjoint read ranges and pwrite
// them independently. Used to make FASTQ inputs of the synthetic configs (bench, tests).
void write_fastq(const mcaat_reads *r, const char *path, int threads) {
    std::vector<uint64_t> packed(r->n_words + 1, 0), offs(r->n_reads + 1);
    if (r->n_words) HIP_OK(hipMemcpy(packed.data(), r->packed.p, 8 * r->n_words, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(offs.data(), r->offsets.p, 8 * (r->n_reads + 1), hipMemcpyDeviceToHost));
    const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) throw Error(MCAAT_E_IO, std::string("cannot create ") + path);
    const uint64_t n = r->n_reads;
    const uint64_t total = 2 * (offs[n] - offs[0]) + 7 * n;
    if (ftruncate(fd, (off_t)total) != 0) {
        close(fd);
        throw Error(MCAAT_E_IO, std::string("cannot size ") + path);
    }
    if (threads < 1) threads = 1;
    std::atomic<bool> failed{false};
    auto work = [&](uint64_t a, uint64_t b) {
        std::vector<char> buf;
        buf.reserve(8u << 20);
        uint64_t pos = 2 * (offs[a] - offs[0]) + 7 * a;
        auto flush = [&]() {
            size_t done = 0;
            while (done < buf.size()) {
                const ssize_t w = pwrite(fd, buf.data() + done, buf.size() - done, (off_t)(pos + done));
                if (w <= 0) { failed = true; return; }
                done += (size_t)w;
            }
            pos += buf.size();
            buf.clear();
        };
        for (uint64_t i = a; i < b && !failed; ++i) {
            const uint64_t s = offs[i], L = offs[i + 1] - s;
            const size_t at = buf.size();
            buf.resize(at + 2 * L + 7);
            char *o = buf.data() + at;
            *o++ = '@'; *o++ = 'r'; *o++ = '\n';
            for (uint64_t j = 0; j < L; ++j) o[j] = "ACGT"[(packed[(s + j) >> 5] >> (2 * ((s + j) & 31))) & 3];
            o += L;
            *o++ = '\n'; *o++ = '+'; *o++ = '\n';
            memset(o, 'I', L);
            o[L] = '\n';
            if (buf.size() >= (8u << 20)) flush();
        }
        flush();
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) {
        const uint64_t a = n * t / threads, b = n * (t + 1) / threads;
        if (a < b) pool.emplace_back(work, a, b);
    }
    for (auto &th : pool) th.join();
    close(fd);
    if (failed) throw Error(MCAAT_E_IO, std::string("write failed: ") + path);
}

}  // namespace mcaat

namespace mcaat {

bool is_compressed_file(const char *path) {
    unsigned char m[4] = {0, 0, 0, 0};
    const int fd = open(path, O_RDONLY);
    if (fd < 0) throw Error(MCAAT_E_IO, std::string("cannot open ") + path);
    const ssize_t n = pread(fd, m, 4, 0);
    close(fd);
    const bool gz = n >= 2 && m[0] == 0x1f && m[1] == 0x8b;
    const bool bz = n >= 4 && m[0] == 'B' && m[1] == 'Z' && m[2] == 'h' && m[3] >= '1' && m[3] <= '9';
    return gz || bz;
}

// A line start q >= pos begins a record when line q starts with '@', line q+2 with '+', and
// lines q+1 and q+3 (sequence, quality) have the same length. A quality line that starts
// with '@' is followed by a header and a sequence line, never by '+', so it is not taken.
// The window grows until four whole lines follow a candidate (records up to 64 MiB).
uint64_t fastq_record_start(const char *path, uint64_t pos) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) throw Error(MCAAT_E_IO, std::string("cannot open ") + path);
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        throw Error(MCAAT_E_IO, std::string("cannot stat ") + path);
    }
    const uint64_t size = (uint64_t)st.st_size;
    if (pos == 0 || pos >= size) {
        close(fd);
        return std::min(pos, size);
    }
    std::vector<uint8_t> buf;
    uint64_t result = size;
    // the window starts one byte early so a record starting exactly at pos is seen
    const uint64_t w0 = pos - 1;
    for (uint64_t win = 1 << 16;; win *= 2) {
        const uint64_t n = std::min<uint64_t>(win, size - w0);
        buf.resize(n);
        uint64_t got = 0;
        while (got < n) {
            const ssize_t r = pread(fd, buf.data() + got, n - got, (off_t)(w0 + got));
            if (r <= 0) break;
            got += (uint64_t)r;
        }
        buf.resize(got);
        const bool at_eof = w0 + got >= size;
        // line starts at or after pos (index 0 is byte pos - 1)
        std::vector<uint64_t> ls;
        for (uint64_t i = 0; i + 1 < got; ++i)
            if (buf[i] == '\n') ls.push_back(i + 1);
        auto line_len = [&](size_t li) -> int64_t {  // -1: line not complete in the window
            const uint64_t b = ls[li];
            const uint64_t e = li + 1 < ls.size() ? ls[li + 1] - 1 : (at_eof ? got : ~0ULL);
            if (e == ~0ULL) return -1;
            uint64_t len = e - b;
            if (len && buf[b + len - 1] == '\n') --len;
            if (len && buf[b + len - 1] == '\r') --len;
            return (int64_t)len;
        };
        bool undecided = false;
        for (size_t li = 0; li < ls.size(); ++li) {
            if (buf[ls[li]] != '@') continue;
            if (li + 3 >= ls.size()) {  // the record's four lines are not all in the window
                if (!at_eof) undecided = true;
                break;
            }
            if (buf[ls[li + 2]] != '+') continue;
            const int64_t a = line_len(li + 1), b = line_len(li + 3);
            if (a < 0 || b < 0) { undecided = true; break; }
            if (a != b) continue;
            result = w0 + ls[li];
            break;
        }
        if (result != size || !undecided || at_eof || win >= (64ULL << 20)) break;
    }
    close(fd);
    return result;
}

}  // namespace mcaat
