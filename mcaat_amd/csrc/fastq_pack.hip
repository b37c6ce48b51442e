// fastq_pack.hip — BuildLib's fast path: host threads pack 4-line FASTQ straight to 2 bits.
//
// Replaces the text upload of the GPU parser (fastq_ingest.hip) for plain files whose records
// are all well-formed 4-line records with non-empty, upper-case A/C/G/T sequences and LF line
// ends — the form simulators and most pipelines write. Such a record is exactly one read of the
// counting view and one record of the mapping view (oracle/fastx.py), so the library is the
// packed sequences in file order. PCIe then carries 2 bits per base instead of ~16 bits of
// text per base (C3: 11.5 GB instead of 92 GB), and the bound moves to the host threads' read
// of the page cache. Any other input (N or IUPAC symbols, lower case, CR line ends, blank or
// wrapped lines, empty sequences, compressed files) declines before anything is returned, and
// the caller runs the GPU text parser, which handles all of them.
//
// Each file is cut into one part per thread at record starts (fastq_record_start). A thread
// reads its part with pread() into a private block, checks and packs every record (AVX2 + BMI2
// where the CPU has them: 32 bases per compare/shift/multiply-add step), and uploads its packed
// stream from two pinned staging buffers on a stream of its own into a region of device memory
// reserved for it. One kernel then concatenates the regions (they start at arbitrary base
// offsets, so every output word is a funnel shift of at most a few region words); the offsets
// are i * L when every read has length L, else uploaded; the mapping view of paired inputs
// (files after the first reverse-complemented, reads.cpp:20-31) is built on the device from
// the counting view.
#include <chrono>
#include <fcntl.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <memory>
#include <thread>

#include "internal.h"

namespace mcaat {

namespace {

// bytes read per pread() block (MCAAT_PACK_BLOCK_KB). Round 5: 512 KB, so the block a thread
// parses is still in its core's cache after the copy into it (C3 BuildLib, one box: 16 MB
// 1.15 / 1.19 s, 4 MB 1.00, 1 MB 0.99 / 0.98, 512 KB 0.95, 256 KB 0.95 / 0.97)
size_t pack_block() {
    static const size_t b = [] {
        const char *e = getenv("MCAAT_PACK_BLOCK_KB");
        const long v = e ? atol(e) : 0;
        return v > 0 ? (size_t)std::min(v, 1L << 20) << 10 : (size_t)512 << 10;
    }();
    return b;
}
constexpr size_t kMaxRecord = 1u << 20;   // longest record the fast path takes
// packed words per pinned staging buffer (2 MB; round 3's 8 MB made the first call pin 256 MB
// for 16 threads, 52 ms inside the span, for no faster upload)
constexpr size_t kStageWords = 1u << 18;
// upload streams shared by the threads (thread t uses stream t % kUpStreams; 0: the context's
// own stream). Round 3 created one per thread, ~4.5 ms each (77 ms for 16, inside the span);
// the uploads (~10 GB/s in all) need no more than one: 0 / 2 / 4 streams measured build_lib
// 1.15-1.19 / 1.24-1.29 / 1.23-1.24 s at C3 (the packing itself unchanged)
constexpr int kUpStreams = 0;
constexpr int kPB = 256;

// ---------------------------------------------------------------- packing
// 2-bit code of an upper-case A/C/G/T byte: ((c >> 1) ^ (c >> 2)) & 3 maps A C G T -> 0 1 2 3.
inline bool scalar_pack(const uint8_t *s, uint32_t n, uint64_t &v) {
    v = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t c = s[i];
        if (c != 'A' && c != 'C' && c != 'G' && c != 'T') return false;
        v |= (uint64_t)(((c >> 1) ^ (c >> 2)) & 3) << (2 * i);
    }
    return true;
}

// 32 bytes (the first n valid) -> 64 bits of codes; false if one of the n is not A/C/G/T
__attribute__((target("avx2,bmi2"))) inline bool avx2_pack32(const uint8_t *s, uint32_t n, uint64_t &v) {
    const __m256i x = _mm256_loadu_si256((const __m256i *)s);
    const __m256i ok = _mm256_or_si256(_mm256_or_si256(_mm256_cmpeq_epi8(x, _mm256_set1_epi8('A')),
                                                       _mm256_cmpeq_epi8(x, _mm256_set1_epi8('C'))),
                                       _mm256_or_si256(_mm256_cmpeq_epi8(x, _mm256_set1_epi8('G')),
                                                       _mm256_cmpeq_epi8(x, _mm256_set1_epi8('T'))));
    const uint32_t m = (uint32_t)_mm256_movemask_epi8(ok);
    const uint32_t need = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1);
    if ((m & need) != need) return false;
    const __m256i c = _mm256_and_si256(_mm256_xor_si256(_mm256_srli_epi16(x, 1), _mm256_srli_epi16(x, 2)),
                                       _mm256_set1_epi8(3));
    // byte pairs -> 4 bits, then 16-bit pairs -> 8 bits: each 32-bit lane holds 4 codes in its low byte
    const __m256i t = _mm256_maddubs_epi16(c, _mm256_set1_epi16(0x0401));
    const __m256i u = _mm256_madd_epi16(t, _mm256_set1_epi32(0x00100001));
    const __m256i g = _mm256_shuffle_epi8(u, _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                                                              -1, 0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                                                              -1, -1));
    const __m256i h = _mm256_permutevar8x32_epi32(g, _mm256_setr_epi32(0, 4, 1, 1, 1, 1, 1, 1));
    v = (uint64_t)_mm_cvtsi128_si64(_mm256_castsi256_si128(h));
    if (n < 32) v &= (1ULL << (2 * n)) - 1;
    return true;
}

bool cpu_has_avx2() {
    static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("bmi2");
    return ok;
}

// ---------------------------------------------------------------- one thread's part
struct PartOut {
    uint64_t region = 0;  // first word of this part's device region
    uint64_t cap = 0;     // words in the region
    uint64_t bases = 0, reads = 0;
    uint32_t L0 = 0;      // length of every read so far (fixed-length input), 0 = none yet
    bool varlen = false;
    std::vector<uint32_t> lengths;  // every read's length once lengths differ
    std::string error;
};

struct Shared {
    std::atomic<bool> decline{false};
};

class PartPacker {
   public:
    PartPacker(uint64_t *dregion, uint64_t *stage0, uint64_t *stage1, hipStream_t st, PartOut &o)
        : dst_(dregion), st_(st), o_(o) {
        stage_[0] = stage0;
        stage_[1] = stage1;
        for (auto &e : ev_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        stage_[0][0] = 0;
    }
    ~PartPacker() {
        for (auto &e : ev_) {
            (void)hipEventSynchronize(e);
            (void)hipEventDestroy(e);
        }
    }

    // record sequence of n bases -> the stream; false: not upper-case ACGT (declines)
    bool append(const uint8_t *s, uint32_t n) {
        if ((pos_ + n) / 32 + 2 >= w0_ + kStageWords) flush(false);
        if ((pos_ + n) / 32 + 2 > o_.cap) return fail("part region full");
        const bool simd = cpu_has_avx2();
        for (uint32_t i = 0; i < n; i += 32) {
            const uint32_t m = std::min<uint32_t>(32, n - i);
            uint64_t v;
            const bool ok = simd ? avx2_pack32(s + i, m, v) : scalar_pack(s + i, m, v);
            if (!ok) return false;
            const uint64_t w = (pos_ >> 5) - w0_;
            const int sh = 2 * (int)(pos_ & 31);
            uint64_t *q = stage_[cur_];
            q[w] |= v << sh;
            q[w + 1] = sh ? v >> (64 - sh) : 0;
            pos_ += m;
        }
        ++o_.reads;
        if (!o_.varlen) {
            if (o_.L0 == 0) o_.L0 = n;
            if (n != o_.L0) {
                o_.varlen = true;
                o_.lengths.assign(o_.reads - 1, o_.L0);
            }
        }
        if (o_.varlen) o_.lengths.push_back(n);
        return true;
    }

    void finish() {
        flush(true);
        for (auto &e : ev_) HIP_OK(hipEventSynchronize(e));
        o_.bases = pos_;
    }

   private:
    bool fail(const char *why) {
        o_.error = why;
        return false;
    }
    // uploads the complete words [w0_, pos_/32) (and the partial last one at the end); the
    // partial word moves to the front of the other staging buffer
    void flush(bool last) {
        const uint64_t wend = last ? (pos_ + 31) / 32 : pos_ / 32;
        const uint64_t nw = wend - w0_;
        if (nw) {
            HIP_OK(hipMemcpyAsync(dst_ + w0_, stage_[cur_], 8 * nw, hipMemcpyHostToDevice, st_));
            HIP_OK(hipEventRecord(ev_[cur_], st_));
        }
        if (last) return;
        const int nx = cur_ ^ 1;
        HIP_OK(hipEventSynchronize(ev_[nx]));  // its previous upload is done
        stage_[nx][0] = stage_[cur_][nw];      // the partial word (0 when pos_ is word-aligned)
        cur_ = nx;
        w0_ = wend;
    }

    uint64_t *dst_;
    hipStream_t st_;
    PartOut &o_;
    uint64_t *stage_[2];
    hipEvent_t ev_[2] = {nullptr, nullptr};
    int cur_ = 0;
    uint64_t pos_ = 0, w0_ = 0;
};

// parse [b, e) of a plain file: 4-line records, each sequence packed; false = declined
// MCAAT_PACK_MMAP=1: the part is mapped (page-cache pages read in place, no copy) and its page
// tables are filled a window ahead by madvise(MADV_POPULATE_READ) instead of one fault per page
bool pack_mmap() {
    const char *e = getenv("MCAAT_PACK_MMAP");
    return e && e[0] == '1';
}
#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif
constexpr size_t kWin = 32u << 20;

bool pack_part(const char *path, uint64_t b, uint64_t e, bool file_end, PartPacker &pk, Shared &sh, PartOut &o) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) {
        o.error = std::string("cannot open ") + path;
        return false;
    }
    struct Fd {
        int fd;
        ~Fd() { close(fd); }
    } guard{fd};
    const bool mapped = pack_mmap() && e > b;
    const size_t kBlk = pack_block();
    std::vector<uint8_t> buf(mapped ? 0 : kBlk + kMaxRecord + 64);
    uint8_t *B = buf.data();
    size_t have = 0;  // bytes in B
    uint64_t off = b;
    size_t i = 0;     // parse position in B
    bool eof = b >= e;
    // mapped: [map_off, e) with B at byte b; the whole part is "read" at once
    uint8_t *map = nullptr;
    size_t map_len = 0, populated = 0;
    struct Unmap {
        uint8_t *&p;
        size_t &n;
        ~Unmap() {
            if (p) munmap(p, n);
        }
    } unmap_guard{map, map_len};
    if (mapped) {
        const uint64_t map_off = b & ~(uint64_t)4095;
        map_len = (size_t)(e - map_off);
        void *m = mmap(nullptr, map_len, PROT_READ, MAP_SHARED, fd, (off_t)map_off);
        if (m == MAP_FAILED) {
            o.error = "mmap failed";
            return false;
        }
        map = (uint8_t *)m;
        B = map + (b - map_off);
        have = (size_t)(e - b);
        off = e;
        eof = true;
    }
    auto populate = [&](size_t upto) {  // page tables of B[0, upto) filled ahead of the parse
        if (!mapped) return;
        while (populated < upto && populated < have) {
            const size_t n = std::min(kWin, have - populated);
            // page-aligned start inside the mapping
            const size_t a0 = (size_t)(B - map) + populated, a = a0 & ~(size_t)4095;
            (void)madvise(map + a, n + (a0 - a), MADV_POPULATE_READ);
            populated += n;
        }
    };
    std::vector<uint8_t> tail;  // a sequence too close to the end of the mapping for 32-B loads
    auto refill = [&]() -> bool {
        // keep the unparsed tail, read the next block behind it
        if (i) {
            memmove(B, B + i, have - i);
            have -= i;
            i = 0;
        }
        const size_t want = (size_t)std::min<uint64_t>(kBlk, e - off);
        size_t got = 0;
        while (got < want) {
            const ssize_t r = pread(fd, B + have + got, want - got, (off_t)(off + got));
            if (r < 0) return false;
            if (r == 0) break;
            got += (size_t)r;
        }
        have += got;
        off += got;
        eof = off >= e || got < want;
        memset(B + have, 0, 64);  // the packer reads up to 31 bytes past a line
        return true;
    };
    if (!mapped && !refill()) return false;
    auto line_end = [&](size_t from) -> size_t {  // index of the '\n' ending the line at from, or ~0
        const void *p = memchr(B + from, '\n', have - from);
        return p ? (size_t)((const uint8_t *)p - B) : ~(size_t)0;
    };
    for (;;) {
        if (sh.decline.load(std::memory_order_relaxed)) return false;
        if (mapped && i + kMaxRecord > populated) populate(i + kMaxRecord + kWin);
        if (i == have) {
            if (eof) break;
            if (!refill()) return false;
            continue;
        }
        // one record: header, sequence, '+', quality
        size_t h = line_end(i), s = h == ~(size_t)0 ? h : line_end(h + 1);
        size_t p = s == ~(size_t)0 ? s : line_end(s + 1);
        size_t q = p == ~(size_t)0 ? p : line_end(p + 1);
        if (q == ~(size_t)0) {
            // the record continues past the block (or the file ends without a final newline)
            if (!eof) {
                if (have - i > kMaxRecord) return false;
                if (!refill()) return false;
                continue;
            }
            if (p != ~(size_t)0 && file_end && e == off) {
                q = have;  // last record of the file, no final newline
                if (q == p + 1) return false;
            } else {
                return false;  // truncated record
            }
        }
        if (B[i] != '@' || B[h + 1] == '\n' || B[s + 1] != '+') return false;
        const size_t n = s - (h + 1);
        if (n == 0 || q - (p + 1) != n) return false;
        if (B[s - 1] == '\r' || B[h - 1] == '\r' || B[q - 1] == '\r' || B[p - 1] == '\r') return false;
        if (mapped && h + 1 + n + 32 > have) {  // the 32-B loads would leave the mapping
            tail.assign(B + h + 1, B + h + 1 + n);
            tail.resize(n + 64, 0);
            if (!pk.append(tail.data(), (uint32_t)n)) return false;
        } else if (!pk.append(B + h + 1, (uint32_t)n)) {
            return false;
        }
        i = q < have ? q + 1 : have;
    }
    return true;
}

// ---------------------------------------------------------------- device kernels
// part tables of k_concat_parts held in LDS up to this many parts ((2P + 1) x 8 B = 32 KB)
constexpr int kConcatLdsParts = 2047;
// out word W = bases [32W, 32W + 32) of the concatenation of the parts (part t: n_t bases at
// base offset start[t], stored from word region[t] of src)
__global__ void k_concat_parts(const uint64_t *src, const uint64_t *region_g, const uint64_t *start_g, int T,
                               uint64_t n_words, uint64_t total, uint64_t *out) {
    // (round 4) the parts' starts and regions in LDS, and each thread's part carried from its
    // previous word (its words ascend): 16.7 -> 6.3 ms at C3 (11.5 GB), from a scan of the
    // global start table per word
    // Above kConcatLdsParts parts (many files x many threads) the tables stay in global memory:
    // the launch then asks for no dynamic LDS (64 KB per workgroup is the limit)
    extern __shared__ uint64_t sh_parts[];
    const uint64_t *start = start_g, *region = region_g;
    if (T <= kConcatLdsParts) {
        for (int i = threadIdx.x; i <= T; i += blockDim.x) sh_parts[i] = start_g[i];
        for (int i = threadIdx.x; i < T; i += blockDim.x) sh_parts[T + 1 + i] = region_g[i];
        __syncthreads();
        start = sh_parts;
        region = sh_parts + T + 1;
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    int t = 0;
    for (uint64_t W = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; W < n_words; W += stride) {
        uint64_t j = 32 * W;
        const uint64_t jend = min(j + 32, total);
        while (t + 1 < T && start[t + 1] <= j) ++t;
        uint64_t v = 0;
        int filled = 0;
        while (j < jend) {
            while (start[t + 1] <= j) ++t;
            const uint64_t lp = j - start[t];           // position inside part t
            const uint64_t take = min(jend, start[t + 1]) - j;
            const uint64_t w = region[t] + (lp >> 5);
            const int sh = 2 * (int)(lp & 31);
            uint64_t x = src[w] >> sh;
            if (sh) x |= src[w + 1] << (64 - sh);
            if (take < 32) x &= (1ULL << (2 * take)) - 1;
            v |= x << (2 * filled);
            filled += (int)take;
            j += take;
        }
        out[W] = v;
    }
}

__global__ void k_offsets_fixed(uint64_t *off, uint64_t n, uint64_t L) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) off[i] = i * L;
}

// mapping view of paired inputs: reads before first_rc as they are, the others reversed and
// complemented (one record per read in this path)
__global__ void k_mapping_view(const uint64_t *packed, const uint64_t *off, uint64_t n_reads, uint64_t first_rc,
                               uint64_t n_words, uint64_t total, uint64_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t W = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; W < n_words; W += stride) {
        const uint64_t j0 = 32 * W, j1 = min(j0 + 32, total);
        // the read holding j0: last i with off[i] <= j0
        uint64_t lo = 0, hi = n_reads;
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) / 2;
            if (off[mid] <= j0) lo = mid;
            else hi = mid;
        }
        uint64_t i = lo, v = 0;
        for (uint64_t j = j0; j < j1; ++j) {
            while (off[i + 1] <= j) ++i;
            uint64_t src = j, flip = 0;
            if (i >= first_rc) {
                src = off[i] + off[i + 1] - 1 - j;
                flip = 3;
            }
            const uint64_t b = ((packed[src >> 5] >> (2 * (src & 31))) & 3) ^ flip;
            v |= b << (2 * (j - j0));
        }
        out[W] = v;
    }
}

// bases per byte and the read length of a file's first records (up to 1 MB of them), for
// the pass-A-ahead estimate; false when the sample's reads differ in length or none is whole
bool sample_records(const char *path, uint64_t b, uint64_t e, double &bases_per_byte, uint32_t &L) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return false;
    std::vector<uint8_t> buf((size_t)std::min<uint64_t>(e - b, 1u << 20));
    const ssize_t got = pread(fd, buf.data(), buf.size(), (off_t)b);
    close(fd);
    if (got <= 0) return false;
    size_t i = 0, line = 0, rec_end = 0;
    uint64_t bases = 0, n = 0;
    L = 0;
    for (size_t j = 0; j < (size_t)got; ++j) {
        if (buf[j] != '\n') continue;
        if (line % 4 == 1) {
            const uint64_t len = j - i;
            if (L && len != L) return false;
            L = (uint32_t)len;
        }
        if (line % 4 == 3) {
            bases += L;
            ++n;
            rec_end = j + 1;
        }
        ++line;
        i = j + 1;
    }
    if (!n || !rec_end) return false;
    bases_per_byte = (double)bases / (double)rec_end;
    return true;
}

int pack_threads() {
    if (const char *e = getenv("MCAAT_PACK_THREADS")) return std::max(1, std::min(64, atoi(e)));
    if (const char *e = getenv("OMP_NUM_THREADS")) {
        const int v = atoi(e);
        if (v > 0) return std::min(64, v);
    }
    return (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

}  // namespace

bool fastq_hostpack(mcaat_ctx *ctx, const char *const *files, int n_files,
                    const std::vector<std::pair<uint64_t, uint64_t>> *ranges, mcaat_reads *r) {
    if (const char *e = getenv("MCAAT_HOSTPACK"))
        if (e[0] == '0') return false;
    if (knob(ctx, "fq.hostpack", 1) == 0) return false;
    for (int f = 0; f < n_files; ++f)
        if (is_compressed_file(files[f])) return false;
    const int T = pack_threads();
    hipStream_t st = ctx->stream;

    // parts: per file, T x K byte ranges cut at record starts (MCAAT_PACK_SPLIT = K), taken by
    // min(parts, T) worker threads from a shared counter. The threads read the page cache at
    // different speeds (C3, one part each: busy 0.83-1.10 s), so parts of ~1/256 of the file
    // let the fast ones take more: K = 1 / 8 / 16 -> pack 1.04-1.10 / 1.01-1.07 / 0.99-1.03 s
    int K = 16;
    if (const char *e = getenv("MCAAT_PACK_SPLIT")) K = std::max(1, std::min(16, atoi(e)));
    // keep the part tables of the concatenation in LDS where the file and thread counts allow
    K = std::max(1, std::min(K, kConcatLdsParts / std::max(1, n_files * T)));
    struct Part {
        int file;
        uint64_t b, e;
        bool file_end;
    };
    std::vector<Part> parts;
    for (int f = 0; f < n_files; ++f) {
        struct stat sb;
        if (stat(files[f], &sb) != 0) throw Error(MCAAT_E_IO, std::string("cannot stat ") + files[f]);
        const uint64_t S = (uint64_t)sb.st_size;
        const uint64_t b = ranges ? std::min(S, (*ranges)[f].first) : 0;
        const uint64_t e = ranges ? std::min(S, (*ranges)[f].second) : S;
        if (b >= e) continue;
        // a file must start with a record (leading blank lines: the GPU parser trims them)
        std::vector<uint64_t> cut{b};
        const int TK = T * K;
        for (int t = 1; t < TK; ++t) {
            const uint64_t c = fastq_record_start(files[f], b + (uint64_t)((unsigned __int128)(e - b) * t / TK));
            cut.push_back(std::max(cut.back(), std::min(c, e)));
        }
        cut.push_back(e);
        for (int t = 0; t < TK; ++t)
            if (cut[t + 1] > cut[t]) parts.push_back({f, cut[t], cut[t + 1], cut[t + 1] == S});
    }
    if (parts.empty()) return false;  // empty inputs: the GPU path's conventions
    const int P = (int)parts.size();

    // device regions (bases <= bytes / 2 for 4-line records) and pinned staging on the context
    std::vector<PartOut> outs(P);
    uint64_t rw = 0;
    for (int t = 0; t < P; ++t) {
        outs[t].region = rw;
        outs[t].cap = (parts[t].e - parts[t].b) / 64 + 64;
        rw += outs[t].cap;
    }
    verbose_mark(ctx, "fq.parts");
    // written by the upload streams, which the arena does not watch: taken with no allocation
    // stream, so the host waits for every fence still pending on the block (alloc.hip); the
    // stream guard below synchronises those streams before the block is freed
    DevBuf<uint64_t> regions;
    {
        AllocStreamScope foreign(nullptr);
        regions.alloc(rw);
    }
    verbose_mark(ctx, "fq.regions");
    const int NW = K > 1 ? std::min(P, T) : P;  // worker threads (K = 1: one per part, as round 3)
    const size_t stage_bytes = (size_t)NW * 2 * kStageWords * 8;
    if (ctx->pack_pinned_bytes < stage_bytes) {
        if (ctx->pack_pinned) HIP_OK(hipHostFree(ctx->pack_pinned));
        ctx->pack_pinned = nullptr;
        ctx->pack_pinned_bytes = 0;
        HIP_OK(hipHostMalloc((void **)&ctx->pack_pinned, stage_bytes, hipHostMallocDefault));
        ctx->pack_pinned_bytes = stage_bytes;
    }
    verbose_mark(ctx, "fq.pinned");
    // MCAAT_UP_STREAMS (A/B): upload streams; 0 = the context's own stream, none created
    int ns = kUpStreams;
    if (const char *e = getenv("MCAAT_UP_STREAMS")) ns = std::max(0, atoi(e));
    std::vector<hipStream_t> streams(std::min(P, std::max(ns, 1)), nullptr);
    struct Streams {
        std::vector<hipStream_t> &s;
        hipStream_t own;
        ~Streams() {
            for (auto x : s)
                if (x && x != own) {
                    (void)hipStreamSynchronize(x);
                    (void)hipStreamDestroy(x);
                }
        }
    } sguard{streams, st};
    if (ns == 0) {
        streams[0] = st;  // not destroyed: the guard below skips it
    } else {
        for (auto &s : streams) HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }

    verbose_mark(ctx, "fq.streams");
    // mcaat_count_ahead: pass A for k on each part as it lands (node_counter.hip nc_ahead_*),
    // sized from the first records of the first part
    std::shared_ptr<NcAhead> ahead;
    uint32_t ahead_L = 0;
    int ahead_k = 0;
    if (const int ak = ctx->ahead_k) {
        ctx->ahead_k = 0;
        double bpb = 0;
        if (knob(ctx, "nc.ahead", 1) && sample_records(files[parts[0].file], parts[0].b, parts[0].e, bpb, ahead_L) &&
            ahead_L > (uint32_t)ak) {
            uint64_t bytes = 0;
            for (auto &pt : parts) bytes += pt.e - pt.b;
            const double reads = (double)bytes * bpb / ahead_L * 1.02 + 64.0 * P;
            const uint64_t npos = ahead_L - (uint32_t)ak;  // (k+1)-mers per read
            // the buckets are live beside the part regions and the packed reads: if they cannot be
            // had, the read goes on without the ahead run (pass A then runs after it, as when a
            // part does not fit) instead of failing
            try {
                ahead = nc_ahead_begin(ctx, ak, (uint64_t)(reads * (double)npos),
                                       (uint64_t)(reads * (double)((npos + kNcItem - 1) / kNcItem)));
                ahead_k = ak;
            } catch (const Error &x) {
                (void)hipGetLastError();
                ahead.reset();
                if (getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1')
                    fprintf(stderr, "[mcaat] fq: count ahead skipped (%s)\n", x.what());
            }
            verbose_mark(ctx, "fq.ahead_begin");
        }
    }
    Shared sh;
    std::vector<int> ok(P, 0);
    std::vector<std::string> err(P);
    std::atomic<int> next{0};
    std::vector<double> busy(NW, 0.0);
    auto job = [&](int wk) {
        const auto t0 = std::chrono::steady_clock::now();
        // the HIP current device is per thread: a worker's events must belong to the
        // context's device, as its stream does
        (void)hipSetDevice(ctx->device);
        uint64_t *s0 = (uint64_t *)ctx->pack_pinned + (size_t)wk * 2 * kStageWords;
        for (int t = next.fetch_add(1); t < P; t = next.fetch_add(1)) {
            try {
                PartPacker pk(regions.p + outs[t].region, s0, s0 + kStageWords, streams[wk % streams.size()], outs[t]);
                const bool good = pack_part(files[parts[t].file], parts[t].b, parts[t].e, parts[t].file_end, pk, sh, outs[t]);
                if (good) pk.finish();  // the part is in HBM when this returns
                if (good && ahead) {
                    if (outs[t].varlen || (outs[t].reads && outs[t].L0 != ahead_L)) nc_ahead_fail(*ahead);
                    else nc_ahead_part(*ahead, regions.p + outs[t].region, outs[t].reads, outs[t].L0);
                }
                ok[t] = good;
                if (!good) sh.decline.store(true);
            } catch (const std::exception &x) {
                err[t] = x.what();
                sh.decline.store(true);
            }
        }
        busy[wk] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    {
        std::vector<std::thread> pool;
        for (int w = 1; w < NW; ++w) pool.emplace_back(job, w);
        job(0);
        for (auto &th : pool) th.join();
    }
    static const bool verbose = getenv("MCAAT_VERBOSE") && getenv("MCAAT_VERBOSE")[0] == '1';
    if (verbose) {
        const auto mm = std::minmax_element(busy.begin(), busy.end());
        fprintf(stderr, "[mcaat] fq: %d parts, %d workers, busy %.3f .. %.3f s\n", P, NW, *mm.first, *mm.second);
    }
    verbose_mark(ctx, "fq.pack");
    for (int t = 0; t < P; ++t)
        if (!err[t].empty()) throw Error(MCAAT_E_HIP, "FASTQ packing: " + err[t]);
    for (int t = 0; t < P; ++t)
        if (!ok[t]) return false;  // not the fast path's input: the GPU text parser takes it
    // (the ahead run, if any, ends below, after the concatenation is queued beside it)

    // concatenate the parts
    std::vector<uint64_t> start(P + 1, 0), region(P);
    uint64_t n_reads = 0;
    bool fixed = true;
    uint32_t L = 0;
    std::vector<uint64_t> file_records(n_files, 0);
    for (int t = 0; t < P; ++t) {
        start[t + 1] = start[t] + outs[t].bases;
        region[t] = outs[t].region;
        n_reads += outs[t].reads;
        file_records[parts[t].file] += outs[t].reads;
        if (outs[t].reads) {
            if (outs[t].varlen || (L && outs[t].L0 != L)) fixed = false;
            if (!L) L = outs[t].L0;
        }
    }
    const uint64_t n_bases = start[P], n_words = (n_bases + 31) / 32;
    DevBuf<uint64_t> dstart(P + 1), dregion(P);
    HIP_OK(hipMemcpyAsync(dstart.p, start.data(), 8 * (P + 1), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(dregion.p, region.data(), 8 * P, hipMemcpyHostToDevice, st));
    r->packed.alloc(n_words + 64);
    HIP_OK(hipMemsetAsync(r->packed.p + n_words, 0, 8 * 64, st));
    if (n_words) {
        KernelTimer kt(ctx, "fq_concat", 16.0 * (double)n_words);
        hipLaunchKernelGGL(k_concat_parts, dim3(grid_for(n_words, kPB, (unsigned)ctx->n_cu * 8)), dim3(kPB),
                           P <= kConcatLdsParts ? (size_t)(2 * P + 1) * 8 : (size_t)0, st, regions.p, dregion.p, dstart.p, P, n_words, n_bases, r->packed.p);
        LAUNCH_OK();
        kt.stop();
    }
    r->offsets.alloc(n_reads + 1);
    if (fixed) {
        hipLaunchKernelGGL(k_offsets_fixed, dim3(grid_for(n_reads + 1, kPB)), dim3(kPB), 0, st, r->offsets.p, n_reads,
                           (uint64_t)L);
        LAUNCH_OK();
    } else {
        std::vector<uint64_t> off(n_reads + 1, 0);
        uint64_t k = 0;
        for (int t = 0; t < P; ++t) {
            for (uint64_t j = 0; j < outs[t].reads; ++j, ++k)
                off[k + 1] = off[k] + (outs[t].varlen ? outs[t].lengths[j] : outs[t].L0);
        }
        h2d(ctx, r->offsets.p, off.data(), 8 * off.size());
    }
    if (ahead) {  // its last launches read the parts' regions: ended before they are released
        r->ahead = nc_ahead_end(*ahead);
        r->ahead_k = r->ahead ? ahead_k : 0;
        ahead.reset();
        verbose_mark(ctx, r->ahead ? "fq.ahead_end" : "fq.ahead_dropped");
    }
    HIP_OK(hipStreamSynchronize(st));
    verbose_mark(ctx, "fq.concat");
    regions.release();
    r->ctx = ctx;
    r->n_reads = n_reads;
    r->n_bases = n_bases;
    r->n_words = n_words;
    r->fixed_len = fixed && n_reads ? L : 0;
    r->n_records = n_reads;
    r->file_records = file_records;
    r->has_records = n_files > 1;
    if (r->has_records) {
        r->rec_packed.alloc(n_words + 64);
        HIP_OK(hipMemsetAsync(r->rec_packed.p + n_words, 0, 8 * 64, st));
        if (n_words) {
            hipLaunchKernelGGL(k_mapping_view, dim3(grid_for(n_words, kPB)), dim3(kPB), 0, st, r->packed.p,
                               r->offsets.p, n_reads, file_records[0], n_words, n_bases, r->rec_packed.p);
            LAUNCH_OK();
        }
        r->rec_offsets.alloc(n_reads + 1);
        HIP_OK(hipMemcpyAsync(r->rec_offsets.p, r->offsets.p, 8 * (n_reads + 1), hipMemcpyDeviceToDevice, st));
        HIP_OK(hipStreamSynchronize(st));
    }
    return true;
}

// loads this file's code object now (HIP defers it to the first launch of one of its kernels)
void preload_fastq_pack() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, (const void *)k_offsets_fixed);
}

}  // namespace mcaat
