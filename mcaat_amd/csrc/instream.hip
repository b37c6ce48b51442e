// instream.hip — sequential byte stream of an input file, decompressed: gzip through zlib
// (plain files read through gzread are passed through unchanged), bzip2 through libbz2 opened
// at run time (the reference links BZip2 for MEGAHIT's buildlib and kseq, CMakeLists.txt:38).
// Concatenated gzip members and concatenated bzip2 streams (pbzip2) are read in sequence.
#include <dlfcn.h>
#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <string>

#include "internal.h"

namespace mcaat {

namespace {

// libbz2's low-level stream interface (bzlib.h 1.0: the structure layout is part of the ABI)
struct BzStream {
    char *next_in;
    unsigned int avail_in, total_in_lo32, total_in_hi32;
    char *next_out;
    unsigned int avail_out, total_out_lo32, total_out_hi32;
    void *state;
    void *(*bzalloc)(void *, int, int);
    void (*bzfree)(void *, void *);
    void *opaque;
};
constexpr int kBzOk = 0, kBzStreamEnd = 4;

struct Bz2 {
    int (*init)(BzStream *, int, int) = nullptr;
    int (*decompress)(BzStream *) = nullptr;
    int (*end)(BzStream *) = nullptr;
};

const Bz2 &bz2() {
    static Bz2 b = [] {
        Bz2 x;
        void *h = dlopen("libbz2.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libbz2.so.1.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) throw Error(MCAAT_E_IO, "bzip2 input needs libbz2.so.1, which is not installed");
        x.init = (int (*)(BzStream *, int, int))dlsym(h, "BZ2_bzDecompressInit");
        x.decompress = (int (*)(BzStream *))dlsym(h, "BZ2_bzDecompress");
        x.end = (int (*)(BzStream *))dlsym(h, "BZ2_bzDecompressEnd");
        if (!x.init || !x.decompress || !x.end) throw Error(MCAAT_E_IO, "libbz2 lacks the decompression interface");
        return x;
    }();
    return b;
}

}  // namespace

struct InStream::Impl {
    std::string path;
    gzFile gz = nullptr;
    FILE *bf = nullptr;  // bzip2: the compressed file
    BzStream bs{};
    bool bs_open = false, bz_done = false;
    std::vector<char> in;

    ~Impl() {
        if (gz) gzclose(gz);
        if (bs_open) bz2().end(&bs);
        if (bf) fclose(bf);
    }
    void bz_start() {  // keeps the pending input (the next concatenated stream's first bytes)
        char *ni = bs.next_in;
        const unsigned ai = bs.avail_in;
        memset(&bs, 0, sizeof bs);
        bs.next_in = ni;
        bs.avail_in = ai;
        if (bz2().init(&bs, 0, 0) != kBzOk) throw Error(MCAAT_E_IO, "bzip2 init failed for " + path);
        bs_open = true;
    }
    size_t bz_read(uint8_t *dst, size_t n) {
        size_t got = 0;
        while (got < n && !bz_done) {
            if (bs.avail_in == 0) {
                const size_t r = fread(in.data(), 1, in.size(), bf);
                if (r == 0) {
                    if (ferror(bf)) throw Error(MCAAT_E_IO, "read error in " + path);
                    // input exhausted: complete only at a stream boundary
                    if (bs_open) throw Error(MCAAT_E_IO, "truncated bzip2 stream in " + path);
                    bz_done = true;
                    break;
                }
                bs.next_in = in.data();
                bs.avail_in = (unsigned)r;
            }
            if (!bs_open) bz_start();  // the next concatenated stream
            bs.next_out = (char *)dst + got;
            const size_t want = std::min<size_t>(n - got, 1u << 30);
            bs.avail_out = (unsigned)want;
            const int rc = bz2().decompress(&bs);
            got += want - bs.avail_out;
            if (rc == kBzStreamEnd) {
                bz2().end(&bs);
                bs_open = false;
            } else if (rc != kBzOk) {
                throw Error(MCAAT_E_IO, "corrupt bzip2 data in " + path);
            }
        }
        return got;
    }
};

InStream::InStream(const char *path) : impl_(new Impl) {
    impl_->path = path;
    FILE *f = fopen(path, "rb");
    if (!f) {
        delete impl_;
        throw Error(MCAAT_E_IO, std::string("cannot open ") + path);
    }
    unsigned char m[4] = {0, 0, 0, 0};
    const size_t nm = fread(m, 1, 4, f);
    fseek(f, 0, SEEK_SET);
    kind_ = nm >= 4 && m[0] == 'B' && m[1] == 'Z' && m[2] == 'h' && m[3] >= '1' && m[3] <= '9' ? Kind::Bzip2
            : nm >= 2 && m[0] == 0x1f && m[1] == 0x8b                                         ? Kind::Gzip
                                                                                               : Kind::Plain;
    try {
        if (kind_ == Kind::Bzip2) {
            impl_->bf = f;
            impl_->in.resize(1 << 20);
            (void)bz2();  // fail here, at open, when libbz2 is missing
            impl_->bz_start();
        } else {
            fclose(f);
            impl_->gz = gzopen(path, "rb");
            if (!impl_->gz) throw Error(MCAAT_E_IO, std::string("cannot open ") + path);
            gzbuffer(impl_->gz, 1u << 20);
        }
    } catch (...) {
        delete impl_;
        throw;
    }
}

InStream::~InStream() { delete impl_; }

size_t InStream::read(uint8_t *dst, size_t n) {
    if (kind_ == Kind::Bzip2) return impl_->bz_read(dst, n);
    size_t got = 0;
    while (got < n) {
        const unsigned want = (unsigned)std::min<size_t>(n - got, 1u << 30);
        const int r = gzread(impl_->gz, dst + got, want);
        if (r < 0) {
            int errnum = 0;
            throw Error(MCAAT_E_IO, "read error in " + impl_->path + ": " + gzerror(impl_->gz, &errnum));
        }
        if (r == 0) break;
        got += (size_t)r;
    }
    return got;
}

}  // namespace mcaat
