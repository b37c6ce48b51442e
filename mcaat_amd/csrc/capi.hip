// capi.hip — extern "C" boundary of libmcaat_gpu.so (include/mcaat_gpu.h).
// Every entry point converts internal exceptions into a negative status plus a
// thread-local message (mcaat_last_error), the way the host mirror expects.
#include <sys/stat.h>
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "internal.h"
#include "comm.h"
#include "synth.h"

using namespace mcaat;

namespace {

thread_local std::string g_last_error;

template <class F>
int guarded(F &&f) {
    try {
        f();
        return MCAAT_OK;
    } catch (const Error &e) {
        g_last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc &) {
        g_last_error = "host allocation failed";
        return MCAAT_E_NOMEM;
    } catch (const std::exception &e) {
        g_last_error = e.what();
        return MCAAT_E_INVALID;
    }
}

void require(bool c, const char *msg) {
    if (!c) throw Error(MCAAT_E_INVALID, msg);
}

constexpr int kBlock = 256;

__global__ void k_synth(mcaat_synth_spec s, const uint64_t *genome, uint64_t *packed, uint64_t n_words,
                        uint64_t first, uint64_t count) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n_words; w += stride)
        packed[w] = synth_word(s, genome, w, first, count);
}

__global__ void k_fixed_offsets(uint64_t *off, uint64_t n, uint64_t L) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) off[i] = i * L;
}

void check_spec(const mcaat_synth_spec &s) {
    require(s.n_genomes > 0 && s.genome_len > 0 && s.read_len > 0, "synth: empty genome or read length");
    require(s.read_len <= s.genome_len, "synth: read longer than genome");
    require(s.repeat_len_min <= s.repeat_len_max && s.spacer_len_min <= s.spacer_len_max, "synth: bad length range");
    if (s.arrays_per_genome) {
        const uint64_t worst = (uint64_t)(s.spacers_per_array + 1) * s.repeat_len_max +
                               (uint64_t)s.spacers_per_array * s.spacer_len_max;
        require(worst * s.arrays_per_genome <= s.genome_len, "synth: arrays do not fit the genome");
    }
}

void upload_reads(mcaat_ctx *ctx, const uint64_t *packed, uint64_t n_words, const uint64_t *offsets,
                  uint64_t n_reads, mcaat_reads *r) {
    r->ctx = ctx;
    r->n_reads = n_reads;
    r->n_bases = offsets[n_reads];
    r->n_words = n_words;
    require((r->n_bases + 31) / 32 <= n_words, "reads: packed stream shorter than the offsets say");
    r->fixed_len = 0;
    if (n_reads > 0) {
        const uint64_t L = offsets[1] - offsets[0];
        bool fixed = offsets[0] == 0 && L > 0;
        for (uint64_t i = 0; fixed && i <= n_reads; ++i) fixed = offsets[i] == i * L;
        if (fixed) r->fixed_len = L;
    }
    r->packed.alloc(n_words + 16);
    r->offsets.alloc(n_reads + 1);
    HIP_OK(hipMemsetAsync(r->packed.p, 0, r->packed.bytes(), ctx->stream));
    HIP_OK(hipMemcpyAsync(r->packed.p, packed, 8 * n_words, hipMemcpyHostToDevice, ctx->stream));
    HIP_OK(hipMemcpyAsync(r->offsets.p, offsets, 8 * (n_reads + 1), hipMemcpyHostToDevice, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
}

// FASTQ/FASTA(.gz) -> packed reads. Counting view: records are split at non-ACGT symbols.
// Mapping view (reads.cpp:88-130): one entry per record; records of the second file are
// reversed and complemented (reverse_pair_ends_sequence, reads.cpp:20-31: only A/C/G/T
// are complemented), then coded as k_mer_to_node_id does (reads.cpp:44-52: 'A','C','G' ->
// 0,1,2 and every other character -> 3).
struct Stream {
    std::vector<uint64_t> words;
    std::vector<uint64_t> offsets{0};
    uint64_t n = 0;
    void put(int b) {
        if ((n >> 5) >= words.size()) words.push_back(0);
        words[n >> 5] |= (uint64_t)b << (2 * (n & 31));
        ++n;
    }
};

struct Packer {
    Stream reads;    // counting view
    Stream records;  // mapping view
    bool records_differ = false;
    int file = 0;    // 0: first input file, >0: second (paired) file
    void end_read() {
        if (reads.n != reads.offsets.back()) reads.offsets.push_back(reads.n);
    }
    static int map_code(char ch) { return ch == 'A' ? 0 : ch == 'C' ? 1 : ch == 'G' ? 2 : 3; }
    void add_sequence(const std::string &s) {
        for (char ch : s) {
            int b;
            switch (ch) {
                case 'A': case 'a': b = 0; break;
                case 'C': case 'c': b = 1; break;
                case 'G': case 'g': b = 2; break;
                case 'T': case 't': b = 3; break;
                default: b = -1;
            }
            if (b < 0) end_read();
            else reads.put(b);
            if (ch != 'A' && ch != 'C' && ch != 'G' && ch != 'T') records_differ = true;
        }
        end_read();
        if (file == 0) {
            for (char ch : s) records.put(map_code(ch));
        } else {
            records_differ = true;
            for (size_t i = s.size(); i-- > 0;) {
                const char ch = s[i];
                records.put(map_code(ch == 'A' ? 'T' : ch == 'T' ? 'A' : ch == 'C' ? 'G' : ch == 'G' ? 'C' : ch));
            }
        }
        records.offsets.push_back(records.n);
    }
};

void upload_records(mcaat_ctx *ctx, const Stream &rec, mcaat_reads *r) {
    r->n_records = rec.offsets.size() - 1;
    r->has_records = true;
    r->rec_packed.alloc(rec.words.size() + 16);
    r->rec_offsets.alloc(rec.offsets.size());
    HIP_OK(hipMemsetAsync(r->rec_packed.p, 0, r->rec_packed.bytes(), ctx->stream));
    if (!rec.words.empty())
        HIP_OK(hipMemcpyAsync(r->rec_packed.p, rec.words.data(), 8 * rec.words.size(), hipMemcpyHostToDevice,
                              ctx->stream));
    HIP_OK(hipMemcpyAsync(r->rec_offsets.p, rec.offsets.data(), 8 * rec.offsets.size(), hipMemcpyHostToDevice,
                          ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
}

// first non-blank byte of a (possibly compressed) file: '@' FASTQ, '>' FASTA
int sniff_format(const char *path) {
    InStream f(path);
    uint8_t buf[4096];
    for (;;) {
        const size_t n = f.read(buf, sizeof buf);
        for (size_t i = 0; i < n; ++i)
            if (buf[i] != '\n' && buf[i] != '\r' && buf[i] != ' ' && buf[i] != '\t') return buf[i];
        if (n < sizeof buf) return -1;
    }
}

// Host reader with the reference's kseq semantics (klib kseq_read, as MEGAHIT buildlib and
// kseq++ in reads.cpp read records): FASTA, and the FASTQ inputs the 4-line GPU parser hands
// back (blank lines between records, wrapped sequence/quality lines, records longer than its
// carry reserve). A record starts at the next '>' or '@'; its header line is skipped; sequence
// lines are concatenated (blank lines skipped, one trailing '\r' dropped) up to a line that
// starts with '>', '@' or '+'; after '+' the rest of that line is skipped and quality lines are
// read until they hold at least as many characters as the sequence (at least one line); any
// other count is an error. Restated for the tests in oracle/fastx.py kseq_sequences.
struct GzChars {  // characters of a plain, gzip or bzip2 input
    InStream f;
    std::vector<uint8_t> buf = std::vector<uint8_t>(1 << 20);
    size_t pos = 0, len = 0;
    explicit GzChars(const char *p) : f(p) {}
    int peek() {
        if (pos == len) {
            len = f.read(buf.data(), buf.size());
            pos = 0;
            if (len == 0) return -1;
        }
        return buf[pos];
    }
    int get() {
        const int c = peek();
        if (c >= 0) ++pos;
        return c;
    }
    // the rest of the current line (one trailing '\r' dropped), appended to out if given
    void line(std::string *out) {
        const size_t at = out ? out->size() : 0;
        for (int c; (c = get()) >= 0 && c != '\n';)
            if (out) out->push_back((char)c);
        if (out && out->size() > at && out->back() == '\r') out->pop_back();
    }
};

void read_fastx_host(const char *path, Packer &pk) {
    GzChars in(path);
    std::string seq, qual;
    bool have_header = false;
    for (;;) {
        if (!have_header) {
            int c;
            while ((c = in.get()) >= 0 && c != '>' && c != '@') {
            }
            if (c < 0) return;
        }
        in.line(nullptr);  // header
        seq.clear();
        int c = -1;
        while ((c = in.peek()) >= 0) {
            if (c == '>' || c == '@' || c == '+') break;
            if (c == '\n') {
                in.get();
                continue;
            }
            in.line(&seq);
        }
        if (c < 0) {
            pk.add_sequence(seq);
            return;
        }
        if (c == '>' || c == '@') {
            pk.add_sequence(seq);
            in.get();
            have_header = true;
            continue;
        }
        in.line(nullptr);  // the '+' line
        qual.clear();
        while (in.peek() >= 0) {
            in.line(&qual);
            if (qual.size() >= seq.size()) break;
        }
        if (qual.size() != seq.size())
            throw Error(MCAAT_E_IO, std::string("malformed FASTQ (quality length differs from sequence length): ") + path);
        pk.add_sequence(seq);
        have_header = false;
    }
}

}  // namespace

namespace mcaat {

// genome of the synthetic community: iid bases, arrays R S1 R S2 ... R Sn R written
// into disjoint slots (one slot per array) of each genome
// the planted arrays of the community (what synth_genome_host writes into each slot): per
// array its genome, index, repeat and spacers as base codes 0..3
struct PlantedArray {
    uint64_t g;
    uint32_t a;
    std::vector<int> repeat;
    std::vector<std::vector<int>> spacers;
};
static void synth_arrays(const mcaat_synth_spec &s, std::vector<PlantedArray> *arrays, std::vector<uint64_t> *pos_out) {
    for (uint64_t g = 0; g < s.n_genomes; ++g) {
        for (uint32_t a = 0; a < s.arrays_per_genome; ++a) {
            const uint64_t h0 = hash3(s.seed ^ 0xC415, g, a);
            const uint32_t lr = s.repeat_len_min + (uint32_t)(h0 % (s.repeat_len_max - s.repeat_len_min + 1));
            const uint32_t ls_max = s.spacer_len_max;
            const uint64_t slot = s.genome_len / s.arrays_per_genome;
            uint64_t len = (uint64_t)(s.spacers_per_array + 1) * lr + (uint64_t)s.spacers_per_array * ls_max;
            const uint64_t room = slot > len ? slot - len : 0;
            PlantedArray pa;
            pa.g = g;
            pa.a = a;
            pa.repeat.resize(lr);
            for (uint32_t i = 0; i < lr; ++i) pa.repeat[i] = (int)(hash3(s.seed ^ 0x4e9, g * 1000003 + a, i) & 3);
            for (uint32_t c = 0; c < s.spacers_per_array; ++c) {
                const uint64_t hs = hash3(s.seed ^ 0x5ACE, g * 1000003 + a, c);
                const uint32_t ls = s.spacer_len_min + (uint32_t)(hs % (s.spacer_len_max - s.spacer_len_min + 1));
                std::vector<int> sp(ls);
                for (uint32_t i = 0; i < ls; ++i) sp[i] = (int)(hash3(hs, c, i) & 3);
                pa.spacers.push_back(std::move(sp));
            }
            if (pos_out) pos_out->push_back(g * s.genome_len + a * slot + (room ? hash3(s.seed ^ 0x9051, g, a) % room : 0));
            arrays->push_back(std::move(pa));
        }
    }
}

void synth_genome_host(const mcaat_synth_spec &s, std::vector<uint64_t> &genome) {
    check_spec(s);
    const uint64_t total = (uint64_t)s.n_genomes * s.genome_len;
    genome.assign((total + 31) / 32 + 1, 0);
    auto setb = [&](uint64_t j, int b) {
        uint64_t &w = genome[j >> 5];
        const int sh = 2 * (int)(j & 31);
        w = (w & ~(3ULL << sh)) | ((uint64_t)b << sh);
    };
    for (uint64_t g = 0; g < s.n_genomes; ++g)
        for (uint64_t i = 0; i < s.genome_len; ++i) setb(g * s.genome_len + i, (int)(hash3(s.seed, g, i ^ 0xA11) & 3));
    // arrays R S1 R S2 ... R Sn R, one per slot
    std::vector<PlantedArray> arrays;
    std::vector<uint64_t> starts;
    synth_arrays(s, &arrays, &starts);
    for (size_t j = 0; j < arrays.size(); ++j) {
        uint64_t pos = starts[j];
        const PlantedArray &pa = arrays[j];
        for (size_t c = 0; c <= pa.spacers.size(); ++c) {
            for (int b : pa.repeat) setb(pos++, b);
            if (c == pa.spacers.size()) break;
            for (int b : pa.spacers[c]) setb(pos++, b);
        }
    }
}

void synth_reads(mcaat_ctx *ctx, const mcaat_synth_spec &s, mcaat_reads *out, uint64_t first, uint64_t count) {
    std::vector<uint64_t> genome;
    synth_genome_host(s, genome);
    hipStream_t st = ctx->stream;
    DevBuf<uint64_t> dg(genome.size());
    HIP_OK(hipMemcpyAsync(dg.p, genome.data(), 8 * genome.size(), hipMemcpyHostToDevice, st));
    out->ctx = ctx;
    out->n_reads = count;
    out->n_bases = count * s.read_len;
    out->n_words = (out->n_bases + 31) / 32;
    out->fixed_len = s.read_len;
    out->packed.alloc(out->n_words + 16);
    out->offsets.alloc(s.n_reads + 1);
    HIP_OK(hipMemsetAsync(out->packed.p, 0, out->packed.bytes(), st));
    hipLaunchKernelGGL(k_synth, dim3(grid_for(out->n_words, kBlock)), dim3(kBlock), 0, st, s, dg.p, out->packed.p,
                       out->n_words, first, count);
    LAUNCH_OK();
    hipLaunchKernelGGL(k_fixed_offsets, dim3(grid_for(count + 1, kBlock)), dim3(kBlock), 0, st,
                       out->offsets.p, count, (uint64_t)s.read_len);
    LAUNCH_OK();
    HIP_OK(hipStreamSynchronize(st));
}

}  // namespace mcaat

extern "C" {

const char *mcaat_last_error(void) { return g_last_error.c_str(); }

int mcaat_device_count(int *n) {
    return guarded([&] {
        require(n != nullptr, "null argument");
        int c = 0;
        hipError_t e = hipGetDeviceCount(&c);
        if (e != hipSuccess) { (void)hipGetLastError(); c = 0; }
        *n = c;
    });
}

int mcaat_preload(int device) {
    return guarded([&] {
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess || device < 0 || device >= c) {
            (void)hipGetLastError();
            throw Error(MCAAT_E_HIP, "no such HIP device");
        }
        HIP_OK(hipSetDevice(device));
        mcaat::preload_fastq_pack();
        mcaat::preload_node_counter();
        mcaat::preload_sdbg_build();
        mcaat::preload_cycle_finder();
        mcaat::preload_read_mapping();
        mcaat::preload_shard();
        mcaat::preload_shard_cf();
        mcaat::preload_sdbg_succinct();
        (void)hipGetLastError();
    });
}

int mcaat_init(int device, mcaat_ctx **out) {
    return guarded([&] {
        require(out != nullptr, "null argument");
        int c = 0;
        hipError_t e = hipGetDeviceCount(&c);
        if (e != hipSuccess || c == 0) {
            (void)hipGetLastError();
            throw Error(MCAAT_E_HIP, "no HIP device available");
        }
        require(device >= 0 && device < c, "device index out of range");
        HIP_OK(hipSetDevice(device));
        auto *ctx = new mcaat_ctx;
        ctx->device = device;
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
            ctx->n_cu = ncu;
        hipError_t se = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
        // the side stream of the counter's pass B / pass C overlap, created with the context
        // rather than inside the first count (~4.5 ms per stream)
        if (se == hipSuccess) se = hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking);
        if (se != hipSuccess) {
            if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
            delete ctx;
            throw Error(MCAAT_E_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(se));
        }
        // frees fence these streams while they have work queued (stream-ordered arena, alloc.hip)
        mcaat::watch_stream(device, ctx->stream);
        mcaat::watch_stream(device, ctx->side);
        *out = ctx;
    });
}

void mcaat_finalize(mcaat_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    mcaat::dev_trim();
    mcaat::unwatch_stream(ctx->device, ctx->side);
    mcaat::unwatch_stream(ctx->device, ctx->stream);
    if (mcaat::alloc_stream() == ctx->stream) mcaat::set_alloc_stream(nullptr);
    for (auto *&p : ctx->pinned)
        if (p) (void)hipHostFree(p);
    for (hipEvent_t e : ctx->events) (void)hipEventDestroy(e);
    if (ctx->bounce) (void)hipHostFree(ctx->bounce);
    if (ctx->pack_pinned) (void)hipHostFree(ctx->pack_pinned);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int mcaat_reads_from_host(mcaat_ctx *ctx, const uint64_t *packed, uint64_t n_words, const uint64_t *offsets,
                          uint64_t n_reads, mcaat_reads **out) {
    return guarded([&] {
        require(ctx && out && offsets && (packed || n_words == 0), "null argument");
        mcaat::bind(ctx);
        auto *r = new mcaat_reads;
        try {
            upload_reads(ctx, packed, n_words, offsets, n_reads, r);
        } catch (...) {
            delete r;
            throw;
        }
        *out = r;
    });
}

int mcaat_count_ahead(mcaat_ctx *ctx, int k) {
    return guarded([&] {
        require(ctx, "null argument");
        require(k == 0 || (k >= 2 && k <= kMaxK), "k must be 0 or in [2, 30]");
        ctx->ahead_k = k;
    });
}

int mcaat_reads_from_fastx(mcaat_ctx *ctx, const char *const *files, int n_files, mcaat_reads **out) {
    struct AheadOnce {  // one read uses a mcaat_count_ahead request, whichever path it takes
        mcaat_ctx *c;
        ~AheadOnce() {
            if (c) c->ahead_k = 0;
        }
    } once{ctx};
    return guarded([&] {
        require(ctx && out && files && n_files > 0, "null argument");
        mcaat::bind(ctx);
        // empty (or blank) files go with either format: they hold no records, and keep their
        // place in the file order (a second file's records are reverse-complemented)
        int n_fastq = 0, n_fasta = 0;
        for (int i = 0; i < n_files; ++i) {
            const int c = sniff_format(files[i]);
            if (c == '@') ++n_fastq;
            else if (c == '>') ++n_fasta;
            else if (c != -1) throw Error(MCAAT_E_IO, std::string("not FASTA/FASTQ: ") + files[i]);
        }
        auto *r = new mcaat_reads;
        auto host_path = [&] {
            Packer pk;
            std::vector<uint64_t> per_file;
            for (int i = 0; i < n_files; ++i) {
                pk.file = i;
                const uint64_t before = pk.records.offsets.size();
                read_fastx_host(files[i], pk);
                per_file.push_back(pk.records.offsets.size() - before);
            }
            *r = mcaat_reads{};
            upload_reads(ctx, pk.reads.words.data(), pk.reads.words.size(), pk.reads.offsets.data(),
                         pk.reads.offsets.size() - 1, r);
            if (pk.records_differ) upload_records(ctx, pk.records, r);
            r->file_records = per_file;
        };
        try {
            if (n_fastq > 0 && n_fasta == 0) {
                // 4-line FASTQ on the GPU; inputs it does not take (blank lines between records,
                // wrapped lines, records above its carry reserve) are read again on the host
                try {
                    ingest_fastq(ctx, files, n_files, r);
                } catch (const FormatError &) {
                    host_path();
                }
            } else {
                host_path();  // FASTA, FASTA + FASTQ, or only empty files
            }
        } catch (...) {
            delete r;
            throw;
        }
        *out = r;
    });
}

/* mapping view (the counting view itself when not separate) */
int mcaat_reads_records_download(const mcaat_reads *r, uint64_t *packed, uint64_t *offsets) {
    return guarded([&] {
        require(r != nullptr, "null argument");
        const uint64_t n = r->has_records ? r->n_records : r->n_reads;
        const auto &pk = r->has_records ? r->rec_packed : r->packed;
        const auto &of = r->has_records ? r->rec_offsets : r->offsets;
        uint64_t nb = 0;
        HIP_OK(hipMemcpy(&nb, of.p + n, 8, hipMemcpyDeviceToHost));
        if (packed && nb) HIP_OK(hipMemcpy(packed, pk.p, 8 * ((nb + 31) / 32), hipMemcpyDeviceToHost));
        if (offsets) HIP_OK(hipMemcpy(offsets, of.p, 8 * (n + 1), hipMemcpyDeviceToHost));
    });
}

int mcaat_reads_info(const mcaat_reads *r, uint64_t *n_reads, uint64_t *n_bases) {
    return guarded([&] {
        require(r != nullptr, "null argument");
        if (n_reads) *n_reads = r->n_reads;
        if (n_bases) *n_bases = r->n_bases;
    });
}

int mcaat_reads_download(const mcaat_reads *r, uint64_t *packed, uint64_t *offsets) {
    return guarded([&] {
        require(r != nullptr, "null argument");
        mcaat::bind(r->ctx);
        if (packed) HIP_OK(hipMemcpy(packed, r->packed.p, 8 * r->n_words, hipMemcpyDeviceToHost));
        if (offsets) HIP_OK(hipMemcpy(offsets, r->offsets.p, 8 * (r->n_reads + 1), hipMemcpyDeviceToHost));
    });
}

int mcaat_reads_write_fastq(const mcaat_reads *r, const char *path, int threads) {
    return guarded([&] {
        require(r && path, "null argument");
        mcaat::bind(r->ctx);
        write_fastq(r, path, threads);
    });
}

void mcaat_reads_free(mcaat_reads *r) { delete r; }

int mcaat_reads_synth(mcaat_ctx *ctx, const mcaat_synth_spec *spec, mcaat_reads **out) {
    return guarded([&] {
        require(ctx && spec && out, "null argument");
        check_spec(*spec);
        mcaat::bind(ctx);
        auto *r = new mcaat_reads;
        try {
            synth_reads(ctx, *spec, r, 0, spec->n_reads);
        } catch (...) {
            delete r;
            throw;
        }
        *out = r;
    });
}

int mcaat_reads_synth_range(mcaat_ctx *ctx, const mcaat_synth_spec *spec, uint64_t first, uint64_t count,
                            mcaat_reads **out) {
    return guarded([&] {
        require(ctx && spec && out, "null argument");
        check_spec(*spec);
        require(first <= spec->n_reads && count <= spec->n_reads - first, "read range outside the spec");
        mcaat::bind(ctx);
        auto *r = new mcaat_reads;
        try {
            synth_reads(ctx, *spec, r, first, count);
        } catch (...) {
            delete r;
            throw;
        }
        *out = r;
    });
}

int mcaat_synth_host(const mcaat_synth_spec *spec, uint64_t *packed, uint64_t *offsets) {
    return guarded([&] {
        require(spec && packed && offsets, "null argument");
        std::vector<uint64_t> genome;
        synth_genome_host(*spec, genome);
        const uint64_t nb = spec->n_reads * spec->read_len, nw = (nb + 31) / 32;
        for (uint64_t w = 0; w < nw; ++w) packed[w] = synth_word(*spec, genome.data(), w);
        for (uint64_t i = 0; i <= spec->n_reads; ++i) offsets[i] = i * spec->read_len;
    });
}

int mcaat_synth_genome_host(const mcaat_synth_spec *spec, uint64_t *packed) {
    return guarded([&] {
        require(spec && packed, "null argument");
        std::vector<uint64_t> genome;
        synth_genome_host(*spec, genome);
        const uint64_t total = (uint64_t)spec->n_genomes * spec->genome_len;
        memcpy(packed, genome.data(), 8 * ((total + 31) / 32));
    });
}

int mcaat_synth_arrays_host(const mcaat_synth_spec *spec, char *text, uint64_t cap, uint64_t *len) {
    return guarded([&] {
        require(spec && len, "null argument");
        check_spec(*spec);
        std::vector<PlantedArray> arrays;
        synth_arrays(*spec, &arrays, nullptr);
        std::string t;
        auto seq = [&](const std::vector<int> &v) {
            for (int b : v) t += "ACGT"[b];
        };
        for (const auto &pa : arrays) {
            t += std::to_string(pa.g) + "\t" + std::to_string(pa.a) + "\t";
            seq(pa.repeat);
            t += "\t";
            for (size_t c = 0; c < pa.spacers.size(); ++c) {
                if (c) t += ",";
                seq(pa.spacers[c]);
            }
            t += "\n";
        }
        *len = t.size();
        if (text && cap) {
            const size_t n = std::min<size_t>(cap - 1, t.size());
            memcpy(text, t.data(), n);
            text[n] = 0;
        }
    });
}

void mcaat_trim(mcaat_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    mcaat::dev_trim();
}

int mcaat_count_edges(mcaat_ctx *ctx, const mcaat_reads *r, int k, uint64_t *n_distinct, uint64_t **keys,
                      uint32_t **counts) {
    return guarded([&] {
        require(ctx && r && n_distinct && keys && counts, "null argument");
        require(k >= 2 && k <= kMaxK, "k must be in [2, 30]");
        mcaat::bind(ctx);
        CountResult c;
        node_counter(ctx, r, k, c);
        sort_counts(ctx, c, k);
        *n_distinct = c.n;
        *keys = (uint64_t *)malloc(8 * (c.n ? c.n : 1));
        *counts = (uint32_t *)malloc(4 * (c.n ? c.n : 1));
        if (!*keys || !*counts) throw std::bad_alloc();
        if (c.n) {
            HIP_OK(hipMemcpy(*keys, c.keys.p, 8 * c.n, hipMemcpyDeviceToHost));
            HIP_OK(hipMemcpy(*counts, c.counts.p, 4 * c.n, hipMemcpyDeviceToHost));
        }
    });
}

void mcaat_free(void *p) { free(p); }

int mcaat_build_graph(mcaat_ctx *ctx, const mcaat_reads *r, int k, mcaat_graph **out) {
    return guarded([&] {
        require(ctx && r && out, "null argument");
        require(k >= 2 && k <= kMaxK, "k must be in [2, 30]");
        mcaat::bind(ctx);
        verbose_mark(ctx, "build.enter");
        auto *g = new mcaat_graph;
        g->ctx = ctx;
        try {
            verbose_mark(ctx, "build.new");
            StageTimer timer(ctx);
            verbose_mark(ctx, "build.timer");
            CountResult c;
            node_counter(ctx, r, k, c);
            timer.mark("node_counter");
            sdbg_build(ctx, c, k, g);
            timer.mark("sdbg_build");
            HIP_OK(hipStreamSynchronize(ctx->stream));
            timer.finish();
        } catch (...) {
            delete g;
            throw;
        }
        *out = g;
    });
}

int mcaat_count_local(mcaat_ctx *ctx, const mcaat_reads *r, int k, mcaat_counts **out) {
    return guarded([&] {
        require(ctx && r && out, "null argument");
        require(k >= 2 && k <= kMaxK, "k must be in [2, 30]");
        mcaat::bind(ctx);
        auto *c = new mcaat_counts;
        c->ctx = ctx;
        c->k = k;
        try {
            StageTimer timer(ctx);
            node_counter(ctx, r, k, c->c);
            timer.mark("node_counter");
            HIP_OK(hipStreamSynchronize(ctx->stream));
            timer.finish();
        } catch (...) {
            delete c;
            throw;
        }
        *out = c;
    });
}

int mcaat_counts_info(const mcaat_counts *c, uint64_t *n_canonical) {
    return guarded([&] {
        require(c && n_canonical, "null argument");
        *n_canonical = c->c.n;
    });
}

int mcaat_counts_histogram(const mcaat_counts *c, int bits, uint64_t *hist) {
    return guarded([&] {
        require(c && hist, "null argument");
        require(bits >= 1 && bits <= 13 && bits <= 2 * (c->k + 1), "histogram bits must be in [1, min(13, 2(k+1))]");
        mcaat::bind(c->ctx);
        counts_histogram(c->ctx, c->c, c->k, bits, hist);
    });
}

int mcaat_counts_partition(const mcaat_counts *c, int n_owners, const uint64_t *splits, uint64_t *sizes,
                           uint64_t *keys_dev, uint32_t *counts_dev, uint64_t cap) {
    return guarded([&] {
        require(c && sizes && (n_owners == 1 || splits), "null argument");
        require(n_owners >= 1 && n_owners <= 64, "n_owners must be in [1, 64]");
        for (int i = 1; i + 1 < n_owners; ++i) require(splits[i - 1] <= splits[i], "splits must be ascending");
        mcaat::bind(c->ctx);
        counts_partition(c->ctx, c->c, c->k, n_owners, splits, sizes, keys_dev, counts_dev, cap);
    });
}

// handles may outlive their context (its buffers remember their device's arena)
void mcaat_counts_free(mcaat_counts *c) { delete c; }

int mcaat_edges_reduce(mcaat_ctx *ctx, int k, const uint64_t *keys_dev, const uint32_t *counts_dev, uint64_t n,
                       uint64_t *keys_out_dev, uint16_t *mult_out_dev, uint64_t *n_out) {
    return guarded([&] {
        require(ctx && n_out && (n == 0 || (keys_dev && counts_dev && keys_out_dev && mult_out_dev)), "null argument");
        require(k >= 2 && k <= kMaxK, "k must be in [2, 30]");
        mcaat::bind(ctx);
        *n_out = edges_reduce(ctx, k, keys_dev, counts_dev, n, keys_out_dev, mult_out_dev);
    });
}

int mcaat_graph_from_sorted(mcaat_ctx *ctx, int k, const uint64_t *keys_dev, const uint16_t *mult_dev, uint64_t D,
                            mcaat_graph **out) {
    return guarded([&] {
        require(ctx && out && (D == 0 || (keys_dev && mult_dev)), "null argument");
        require(k >= 2 && k <= kMaxK, "k must be in [2, 30]");
        mcaat::bind(ctx);
        verbose_mark(ctx, "build.enter");
        auto *g = new mcaat_graph;
        g->ctx = ctx;
        try {
            StageTimer timer(ctx);
            graph_from_sorted(ctx, k, keys_dev, mult_dev, D, g);
            timer.mark("sdbg_build");
            HIP_OK(hipStreamSynchronize(ctx->stream));
            timer.finish();
        } catch (...) {
            delete g;
            throw;
        }
        *out = g;
    });
}

// entry points that read the whole graph: a sharded graph (each rank its range) is gathered first
static void require_whole(const mcaat_graph *g) {
    if (g->sharded)
        throw Error(MCAAT_E_INVALID, "the graph is sharded over the ranks: call mcaat_graph_unshard first");
}

int mcaat_graph_shard_info(const mcaat_graph *g, int *sharded, uint64_t *first, uint64_t *n_local) {
    return guarded([&] {
        require(g != nullptr, "null argument");
        if (sharded) *sharded = g->sharded ? 1 : 0;
        if (first) *first = g->sharded ? g->id_lo : 0;
        if (n_local) *n_local = g->sharded ? g->D_local : g->D;
    });
}

int mcaat_graph_unshard(mcaat_graph *g, mcaat_comm *comm) {
    return guarded([&] {
        require(g != nullptr, "null argument");
        if (!g->sharded) return;
        require(comm != nullptr, "a sharded graph is gathered over its communicator");
        mcaat::bind(g->ctx);
        graph_unshard(g, *comm->c);
    });
}

int mcaat_graph_info(const mcaat_graph *g, int *k, uint64_t *n_edges) {
    return guarded([&] {
        require(g != nullptr, "null argument");
        if (k) *k = g->k;
        if (n_edges) *n_edges = g->D;
    });
}

int mcaat_graph_download(const mcaat_graph *g, uint64_t *keys, uint16_t *mult, uint8_t *valid) {
    return guarded([&] {
        require(g != nullptr, "null argument");
        require_whole(g);
        mcaat::bind(g->ctx);
        if (keys && g->D) HIP_OK(hipMemcpy(keys, g->key.p, 8 * g->D, hipMemcpyDeviceToHost));
        if (mult && g->D) HIP_OK(hipMemcpy(mult, g->mult.p, 2 * g->D, hipMemcpyDeviceToHost));
        if (valid) graph_download_valid(g, valid);
    });
}

int mcaat_graph_valid_words(const mcaat_graph *g, uint64_t *words) {
    return guarded([&] {
        require(g != nullptr && (words || g->D == 0), "null argument");
        require_whole(g);
        mcaat::bind(g->ctx);
        if (g->D) HIP_OK(hipMemcpy(words, g->valid.p, 8 * g->n_words(), hipMemcpyDeviceToHost));
    });
}

int mcaat_graph_download_range(const mcaat_graph *g, uint64_t first, uint64_t count, uint64_t *keys, uint16_t *mult,
                               uint8_t *valid) {
    return guarded([&] {
        require(g != nullptr, "null argument");
        require(first <= g->D && count <= g->D - first, "edge range out of bounds");
        if (!count) return;
        require_whole(g);
        mcaat::bind(g->ctx);
        if (keys) HIP_OK(hipMemcpy(keys, g->key.p + first, 8 * count, hipMemcpyDeviceToHost));
        if (mult) HIP_OK(hipMemcpy(mult, g->mult.p + first, 2 * count, hipMemcpyDeviceToHost));
        if (valid) {
            const uint64_t w0 = first / 64, w1 = (first + count + 63) / 64;
            std::vector<uint64_t> bits(w1 - w0);
            HIP_OK(hipMemcpy(bits.data(), g->valid.p + w0, 8 * (w1 - w0), hipMemcpyDeviceToHost));
            for (uint64_t i = 0; i < count; ++i) {
                const uint64_t e = first + i;
                valid[i] = (uint8_t)((bits[e / 64 - w0] >> (e & 63)) & 1);
            }
        }
    });
}

int mcaat_graph_set_valid(mcaat_graph *g, const uint64_t *ids, size_t n, int valid) {
    return guarded([&] {
        require(g && (ids || n == 0), "null argument");
        require_whole(g);
        mcaat::bind(g->ctx);
        graph_set_valid(g, ids, n, valid);
    });
}

int mcaat_graph_neighbors(const mcaat_graph *g, const uint64_t *ids, size_t n, int incoming, uint64_t *out,
                          int32_t *counts) {
    return guarded([&] {
        require(g && (n == 0 || (ids && out && counts)), "null argument");
        for (size_t i = 0; i < n; ++i) require(ids[i] < g->D, "edge id out of range");
        require_whole(g);
        mcaat::bind(g->ctx);
        graph_neighbors(g, ids, n, incoming, out, counts);
    });
}

int mcaat_graph_gather(const mcaat_graph *g, const uint64_t *ids, size_t n, uint64_t *keys, uint16_t *mult) {
    return guarded([&] {
        require(g && (n == 0 || ids), "null argument");
        for (size_t i = 0; i < n; ++i) require(ids[i] < g->D, "edge id out of range");
        require_whole(g);
        mcaat::bind(g->ctx);
        graph_gather(g, ids, n, keys, mult);
    });
}

int mcaat_graph_keep_only(mcaat_graph *g, const uint64_t *ids, size_t n) {
    return guarded([&] {
        require(g && (ids || n == 0), "null argument");
        require_whole(g);
        mcaat::bind(g->ctx);
        graph_keep_only(g, ids, n);
    });
}
int mcaat_graph_valid_subgraph(const mcaat_graph *g, uint64_t *n_valid, uint64_t *ids, uint32_t *nbr, uint8_t *counts) {
    return guarded([&] {
        require(g != nullptr && n_valid != nullptr, "null argument");
        require((ids == nullptr) == (nbr == nullptr) && (ids == nullptr) == (counts == nullptr), "all outputs or none");
        require_whole(g);
        mcaat::bind(g->ctx);
        *n_valid = graph_valid_out_ranks(g, ids, nbr, counts);
    });
}

int mcaat_graph_keep_region(mcaat_graph *g, const uint64_t *seeds, size_t n, uint64_t hops) {
    return guarded([&] {
        require(g != nullptr && (n == 0 || seeds), "null argument");
        require_whole(g);
        mcaat::bind(g->ctx);
        graph_keep_region(g, seeds, n, hops);
    });
}

int mcaat_graph_succinct_check(mcaat_graph *g, int check, uint64_t *out, double *ms) {
    return guarded([&] {
        require(g && out && ms, "null argument");
        require_whole(g);
        mcaat::bind(g->ctx);
        graph_succinct_check(g, check != 0, out, ms);
    });
}

int mcaat_graph_save(const mcaat_graph *g, const char *path) {
    return guarded([&] {
        require(g && path, "null argument");
        require_whole(g);
        mcaat::bind(g->ctx);
        graph_save(g, path);
    });
}

int mcaat_graph_load(mcaat_ctx *ctx, const char *path, mcaat_graph **out) {
    return guarded([&] {
        require(ctx && path && out, "null argument");
        mcaat::bind(ctx);
        auto *g = new mcaat_graph;
        try {
            graph_load(ctx, path, g);
        } catch (...) {
            delete g;
            throw;
        }
        *out = g;
    });
}

void mcaat_graph_free(mcaat_graph *g) {
    mcaat_ctx *ctx = g ? g->ctx : nullptr;
    if (ctx) verbose_mark(ctx, "graph.enter_free");
    delete g;
    if (ctx) verbose_mark(ctx, "graph.free");
}

int mcaat_reads_records_info(const mcaat_reads *r, uint64_t *n_records, int *separate) {
    return guarded([&] {
        require(r != nullptr, "null argument");
        if (n_records) *n_records = r->has_records ? r->n_records : r->n_reads;
        if (separate) *separate = r->has_records ? 1 : 0;
    });
}

int mcaat_map_reads(const mcaat_graph *g, const mcaat_reads *r, const uint64_t *cycle_nodes, size_t n_nodes,
                    uint64_t max_batch_ids, mcaat_mapped **out) {
    return guarded([&] {
        require(g && r && out && (cycle_nodes || n_nodes == 0), "null argument");
        require(g->ctx == r->ctx, "graph and reads belong to different contexts");
        require_whole(g);
        mcaat::bind(g->ctx);
        auto *m = new mcaat_mapped;
        try {
            map_reads(g, r, cycle_nodes, n_nodes, max_batch_ids ? max_batch_ids : (uint64_t)1 << 28, m);
        } catch (...) {
            delete m;
            throw;
        }
        *out = m;
    });
}

int mcaat_mapped_get(const mcaat_mapped *m, uint64_t *n_reads, const uint64_t **ids, const uint64_t **offsets,
                     const uint64_t **records) {
    return guarded([&] {
        require(m != nullptr, "null argument");
        if (n_reads) *n_reads = m->offsets.size() - 1;
        if (ids) *ids = m->ids.data();
        if (offsets) *offsets = m->offsets.data();
        if (records) *records = m->records.data();
    });
}

void mcaat_mapped_free(mcaat_mapped *m) { delete m; }

void mcaat_cf_default_params(mcaat_cf_params *p) {
    if (!p) return;
    p->threshold_multiplicity = 20;
    p->low_abundance = 1;
    p->cycle_max_length = 77;
    p->cycle_min_length = 27;
    p->cluster_bound = 500;
    p->step_cap = 10000000;
}

int mcaat_cycle_finder(mcaat_graph *g, const mcaat_cf_params *p, mcaat_cycles **out) {
    return mcaat_cycle_finder_comm(g, nullptr, p, out);
}

int mcaat_cycles_count(const mcaat_cycles *c, size_t *n) {
    return guarded([&] {
        require(c && n, "null argument");
        *n = c->starts.size();
    });
}

int mcaat_cycles_get(const mcaat_cycles *c, size_t i, uint64_t *start, const uint64_t **flat,
                     const uint64_t **offsets, size_t *n_cycles) {
    return guarded([&] {
        require(c != nullptr, "null argument");
        require(i < c->starts.size(), "entry index out of range");
        if (start) *start = c->starts[i];
        if (flat) *flat = c->flat[i].data();
        if (offsets) *offsets = c->offsets[i].data();
        if (n_cycles) *n_cycles = c->offsets[i].size() - 1;
    });
}

int mcaat_cycles_export(const mcaat_cycles *c, uint64_t *sizes, uint64_t *starts, uint64_t *entry_offsets,
                        uint64_t *cycle_offsets, uint64_t *nodes) {
    return guarded([&] {
        require(c && sizes, "null argument");
        const size_t n = c->starts.size();
        uint64_t ncyc = 0, nnodes = 0;
        for (size_t i = 0; i < n; ++i) {
            ncyc += c->offsets[i].size() - 1;
            nnodes += c->flat[i].size();
        }
        sizes[0] = n;
        sizes[1] = ncyc;
        sizes[2] = nnodes;
        if (!starts || !entry_offsets || !cycle_offsets || !nodes) return;  // sizing call
        uint64_t e = 0, q = 0;
        entry_offsets[0] = 0;
        cycle_offsets[0] = 0;
        for (size_t i = 0; i < n; ++i) {
            starts[i] = c->starts[i];
            const auto &of = c->offsets[i];
            for (size_t j = 1; j < of.size(); ++j) cycle_offsets[++e] = q + of[j];
            entry_offsets[i + 1] = e;
            if (!c->flat[i].empty()) memcpy(nodes + q, c->flat[i].data(), 8 * c->flat[i].size());
            q += c->flat[i].size();
        }
    });
}

int mcaat_cycles_stats(const mcaat_cycles *c, uint64_t *stats) {
    return guarded([&] {
        require(c && stats, "null argument");
        for (int i = 0; i < 8; ++i) stats[i] = c->stats[i];
    });
}

int mcaat_cycles_candidates(const mcaat_cycles *c, size_t *n, const uint64_t **ids, const int32_t **buckets) {
    return guarded([&] {
        require(c && n, "null argument");
        *n = c->cand_ids.size();
        if (ids) *ids = c->cand_ids.data();
        if (buckets) *buckets = c->cand_bucket.data();
    });
}

void mcaat_cycles_free(mcaat_cycles *c) { delete c; }

int mcaat_stage_times(const mcaat_ctx *ctx, int max, const char **names, double *ms, int *n) {
    return guarded([&] {
        require(ctx && n, "null argument");
        int m = 0;
        for (auto &s : ctx->stages) {
            if (m < max) {
                if (names) names[m] = s.first;
                if (ms) ms[m] = s.second;
            }
            ++m;
        }
        *n = m;
    });
}

int mcaat_kernel_timing(const mcaat_ctx *ctx, const char *kernel, double *avg_ms, uint64_t *launches,
                        double *bytes_per_launch) {
    return guarded([&] {
        require(ctx && kernel, "null argument");
        auto it = ctx->kstats.find(kernel);
        const KernelStat s = it == ctx->kstats.end() ? KernelStat{} : it->second;
        if (avg_ms) *avg_ms = s.launches ? s.total_ms / s.launches : 0.0;
        if (launches) *launches = s.launches;
        if (bytes_per_launch) *bytes_per_launch = s.launches ? s.total_bytes / s.launches : 0.0;
    });
}

void mcaat_reset_timing(mcaat_ctx *ctx) {
    if (ctx) ctx->kstats.clear();
}

int mcaat_set_knob(mcaat_ctx *ctx, const char *name, int64_t value) {
    static const char *const known[] = {
        "nc.group_budget", "nc.fallback_budget", "nc.out_cap", "nc.l1_slots", "nc.fine_bits",
        "nc.edge_cap",     "nc.desc_cap",        "sort.msd",   "sort.wave_limit", "sort.mid_limit",
        "sort.block_limit", "cf.dls_stack",      "cf.dls_visited", "cf.fc_lock", "cf.fc_relax",
        "cf.fc_out",       "cf.fc_window",       "cf.walk_budget", "sdbg.adj_lds",   "sdbg.adj_cap",       "cf.ruler_mask",
        "nc.overlap",      "sort.l3_counting",   "cf.peel_list_div", "cf.peel_list_cap", "cf.cand_cap",
        "fq.hostpack",     "sort.mid_counting", "nc.big_table", "cf.fused_init", "sort.mid_occ", "cf.scan_u", "cf.prep_batch", "cf.dls_lanes", "dist.oriented",
        "sort.small_mid", "sort.small_limit", "cf.recount", "cf.dls_host",
        "dist.desc",      "cf.compact",         "cf.fresh",   "cf.dls_persist", "nc.split_first", "nc.split_max", "cf.pull_flags", "cf.dls_budget", "nc.grow_early",
        "nc.free_sync", "dist.shard_cf", "dist.ruler_mask", "dist.adj_chunk", "dist.dir_edges", "nc.ahead", "dist.adj_ranges", "dist.win_ranges", "cf.dls_lds", "cf.dls_lds_cap", "dist.segs_at_one", "nc.a_mini", "dist.bfs_sync", "cf.compact_pct", "dist.bfs_block", "dist.bfs_frontier", "dist.res_fixed", "dist.res_batch", "dist.res_block_mb", "dist.walk_block", "dist.walk_batch"};
    return guarded([&] {
        require(ctx && name, "null argument");
        bool ok = false;
        for (const char *k : known) ok = ok || strcmp(k, name) == 0;
        if (!ok) throw Error(MCAAT_E_INVALID, std::string("unknown knob: ") + name);
        if (value < 0) ctx->knobs.erase(name);
        else ctx->knobs[name] = value;
    });
}

/* ---- multi-GPU: communicators and the native sharded path ----------------------- */
int mcaat_comm_unique_id(uint8_t *id) {
    return guarded([&] {
        require(id != nullptr, "null argument");
        comm_unique_id(id);
    });
}

int mcaat_comm_schedule_check(int world, uint64_t seed, uint64_t piece_bytes, uint64_t *rounds) {
    return guarded([&] {
        const uint64_t r = comm_schedule_check(world, seed, piece_bytes);
        if (rounds) *rounds = r;
    });
}

int mcaat_comm_init_rccl(mcaat_ctx *ctx, int world, int rank, const uint8_t *id, mcaat_comm **out) {
    return guarded([&] {
        require(ctx && id && out, "null argument");
        require(world >= 1 && rank >= 0 && rank < world, "rank must be in [0, world)");
        mcaat::bind(ctx);
        auto *c = new mcaat_comm;
        try {
            c->c = comm_rccl(ctx, world, rank, id);
        } catch (...) {
            delete c;
            throw;
        }
        *out = c;
    });
}

int mcaat_comm_init_shm(mcaat_ctx *ctx, int world, int rank, const char *name, uint64_t slot_bytes,
                        mcaat_comm **out) {
    return guarded([&] {
        require(name && out, "null argument");
        require(name[0] == '/' && !strchr(name + 1, '/'), "shared-memory name must be \"/name\"");
        require(world >= 1 && rank >= 0 && rank < world, "rank must be in [0, world)");
        if (ctx) mcaat::bind(ctx);
        auto *c = new mcaat_comm;
        try {
            c->c = comm_shm(ctx, world, rank, name, slot_bytes ? slot_bytes : (256ULL << 20));
        } catch (...) {
            delete c;
            throw;
        }
        *out = c;
    });
}

int mcaat_comm_info(const mcaat_comm *c, int *world, int *rank) {
    return guarded([&] {
        require(c != nullptr, "null argument");
        if (world) *world = c->c->world;
        if (rank) *rank = c->c->rank;
    });
}

int mcaat_comm_barrier(mcaat_comm *c) {
    return guarded([&] {
        require(c != nullptr, "null argument");
        c->c->barrier();
    });
}

int mcaat_comm_allgather_sizes(mcaat_comm *c, uint64_t bytes, uint64_t *sizes) {
    return guarded([&] {
        require(c && sizes, "null argument");
        const std::vector<uint64_t> all = c->c->allgather_one(bytes);
        std::copy(all.begin(), all.end(), sizes);
    });
}

int mcaat_comm_allgatherv(mcaat_comm *c, const void *send, uint64_t bytes, void *recv, const uint64_t *sizes) {
    return guarded([&] {
        require(c && sizes && (send || !bytes), "null argument");
        require(sizes[c->c->rank] == bytes, "sizes[rank] differs from bytes");
        std::vector<uint8_t> all;
        std::vector<uint64_t> got;
        c->c->allgatherv_host(send, bytes, all, got);
        for (int r = 0; r < c->c->world; ++r) require(got[r] == sizes[r], "sizes differ from the ranks' byte counts");
        require(recv || all.empty(), "null argument");
        if (!all.empty()) memcpy(recv, all.data(), all.size());
    });
}

void mcaat_comm_free(mcaat_comm *c) { delete c; }

int mcaat_reads_from_fastx_part(mcaat_ctx *ctx, const char *const *files, int n_files, int part, int n_parts,
                                mcaat_reads **out) {
    if (n_parts == 1 && part == 0) return mcaat_reads_from_fastx(ctx, files, n_files, out);
    return guarded([&] {
        require(n_parts >= 1 && part >= 0 && part < n_parts, "part must be in [0, n_parts)");
        require(ctx && out && files && n_files > 0, "null argument");
        mcaat::bind(ctx);
        std::vector<std::pair<uint64_t, uint64_t>> ranges;
        for (int i = 0; i < n_files; ++i) {
            const int c = sniff_format(files[i]);
            if (c == '>') throw Error(MCAAT_E_IO, std::string("FASTA inputs are not split over ranks: ") + files[i]);
            if (is_compressed_file(files[i])) {
                // one compressed stream cannot be split: part 0 reads the whole file
                ranges.push_back(part == 0 ? std::make_pair(0ULL, ~0ULL) : std::make_pair(0ULL, 0ULL));
                continue;
            }
            struct stat st;
            if (stat(files[i], &st) != 0) throw Error(MCAAT_E_IO, std::string("cannot stat ") + files[i]);
            const uint64_t S = (uint64_t)st.st_size;
            const uint64_t b = fastq_record_start(files[i], (uint64_t)((unsigned __int128)S * part / n_parts));
            const uint64_t e = part + 1 == n_parts
                                   ? S
                                   : fastq_record_start(files[i], (uint64_t)((unsigned __int128)S * (part + 1) / n_parts));
            ranges.push_back({b, std::max(b, e)});
        }
        auto *r = new mcaat_reads;
        try {
            ingest_fastq(ctx, files, n_files, r, &ranges);
        } catch (const FormatError &e) {
            delete r;
            throw Error(MCAAT_E_IO, std::string("input not split over ranks (read it whole): ") + e.what());
        } catch (...) {
            delete r;
            throw;
        }
        *out = r;
    });
}

int mcaat_reads_file_records(const mcaat_reads *r, int file, uint64_t *n_records) {
    return guarded([&] {
        require(r && n_records, "null argument");
        require(file >= 0, "file index out of range");
        if (r->file_records.empty()) {  // reads not loaded from files: one source, file 0
            *n_records = file == 0 ? (r->has_records ? r->n_records : r->n_reads) : 0;
            return;
        }
        require((size_t)file < r->file_records.size(), "file index out of range");
        *n_records = r->file_records[file];
    });
}

int mcaat_build_graph_sharded(mcaat_ctx *ctx, mcaat_comm *comm, const mcaat_reads *r, int k, mcaat_graph **out) {
    return guarded([&] {
        require(ctx && comm && r && out, "null argument");
        require(k >= 2 && k <= kMaxK, "k must be in [2, 30]");
        mcaat::bind(ctx);
        auto *g = new mcaat_graph;
        g->ctx = ctx;
        try {
            build_graph_sharded(ctx, *comm->c, r, k, g);
        } catch (...) {
            delete g;
            throw;
        }
        *out = g;
    });
}

int mcaat_cycle_finder_comm(mcaat_graph *g, mcaat_comm *comm, const mcaat_cf_params *p, mcaat_cycles **out) {
    return guarded([&] {
        require(g && p && out, "null argument");
        require(p->cycle_max_length >= 2 && p->cycle_max_length <= 250, "cycle_max_length must be in [2, 250]");
        require(p->cluster_bound >= 1 && p->cluster_bound <= 65535, "cluster_bound must be in [1, 65535]");
        require(p->step_cap >= 1, "step_cap must be positive");
        mcaat::bind(g->ctx);
        require(!g->sharded || comm, "a sharded graph runs CycleFinder over its communicator");
        auto *c = new mcaat_cycles;
        try {
            if (g->sharded) cycle_finder_sharded(g, *p, c, *comm->c);
            else cycle_finder(g, *p, c, comm ? comm->c.get() : nullptr);
            verbose_mark(g->ctx, "cf.return");
        } catch (...) {
            delete c;
            throw;
        }
        *out = c;
    });
}

}  // extern "C"

int mcaat_arena_check(mcaat_ctx *ctx, int64_t *out) {
    return guarded([&] {
        require(ctx && out, "null argument");
        mcaat::bind(ctx);
        mcaat::arena_check(ctx, out);
    });
}

int mcaat_arena_usage(mcaat_ctx *ctx, int reset_peak, uint64_t *in_use, uint64_t *peak, uint64_t *reserved) {
    return guarded([&] {
        require(ctx != nullptr, "null argument");
        mcaat::bind(ctx);
        mcaat::arena_usage(in_use, peak, reserved, reset_peak != 0);
    });
}
