// hostreg_probe.cpp — how fast can FASTQ bytes in the page cache reach HBM?
// (a) pread into pinned chunks + hipMemcpyAsync (what fastq_ingest does, threads copy)
// (b) mmap the file, hipHostRegister each window, DMA straight from the page cache
// usage: hostreg_probe <file> <window MiB> <threads>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    const char *path = argv[1];
    const size_t W = (size_t)atoll(argv[2]) << 20;
    const int T = atoi(argv[3]);
    const int fd = open(path, O_RDONLY);
    struct stat st;
    fstat(fd, &st);
    const size_t S = (size_t)st.st_size;
    void *dev = nullptr;
    CK(hipMalloc(&dev, 2 * W));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // (a) pread + pinned + copy (double-buffered: read the next while the last uploads)
    {
        unsigned char *pin[2];
        CK(hipHostMalloc((void **)&pin[0], W, 0));
        CK(hipHostMalloc((void **)&pin[1], W, 0));
        const double t0 = now();
        int cur = 0;
        for (size_t off = 0; off < S; off += W, cur ^= 1) {
            const size_t n = std::min(W, S - off);
            CK(hipStreamSynchronize(s));  // the buffer about to be overwritten is free
            std::vector<std::thread> th;
            const size_t piece = (n + T - 1) / T;
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    const size_t a = std::min(n, t * piece), b = std::min(n, a + piece);
                    size_t g = 0;
                    while (a + g < b) {
                        const ssize_t r = pread(fd, pin[cur] + a + g, b - a - g, (off_t)(off + a + g));
                        if (r <= 0) break;
                        g += (size_t)r;
                    }
                });
            for (auto &x : th) x.join();
            CK(hipMemcpyAsync((char *)dev + cur * W, pin[cur], n, hipMemcpyHostToDevice, s));
        }
        CK(hipStreamSynchronize(s));
        const double t1 = now();
        printf("pread+pinned  %zu MiB windows, %d threads: %.2f GB/s\n", W >> 20, T, S / (t1 - t0) / 1e9);
    }
    // (b) mmap + hipHostRegister per window
    {
        unsigned char *m = (unsigned char *)mmap(nullptr, S, PROT_READ, MAP_SHARED, fd, 0);
        if (m == MAP_FAILED) return 3;
        double reg = 0, t0 = now();
        int cur = 0;
        std::vector<void *> regd;
        for (size_t off = 0; off < S; off += W, cur ^= 1) {
            const size_t n = std::min(W, S - off);
            const double r0 = now();
            CK(hipHostRegister(m + off, n, hipHostRegisterReadOnly));
            reg += now() - r0;
            CK(hipMemcpyAsync((char *)dev + cur * W, m + off, n, hipMemcpyHostToDevice, s));
            regd.push_back(m + off);
            if (regd.size() > 2) {
                CK(hipStreamSynchronize(s));
                for (size_t q = 0; q + 1 < regd.size(); ++q) CK(hipHostUnregister(regd[q]));
                regd.erase(regd.begin(), regd.end() - 1);
            }
        }
        CK(hipStreamSynchronize(s));
        for (void *p : regd) CK(hipHostUnregister(p));
        const double t1 = now();
        printf("mmap+register %zu MiB windows: %.2f GB/s (register %.3f s of %.3f s)\n", W >> 20, S / (t1 - t0) / 1e9,
               reg, t1 - t0);
    }
    return 0;
}
