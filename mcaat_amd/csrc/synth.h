// synth.h — counter-based synthetic metagenome reads (SURVEY.md §8d "Synthetic inputs").
// Identical on host and device: every read base is a pure function of (spec, read, pos),
// so any shard or rank can regenerate exactly the same reads without communication.
#pragma once
#include "common.h"
#include "../../include/mcaat_gpu.h"

namespace mcaat {

struct ReadPlace {
    uint64_t g, start;  // genome and first genome base of the read's segment
    int rc;             // 1: read is the reverse complement of the segment
};

MCAAT_HD uint64_t synth_frag_len(const mcaat_synth_spec &s, uint64_t pair) {
    uint64_t F = 270 + hash3(s.seed, pair, 11) % 61;  // 300 +- 30
    if (F < s.read_len) F = s.read_len;
    if (F > s.genome_len) F = s.genome_len;
    return F;
}

MCAAT_HD ReadPlace synth_place(const mcaat_synth_spec &s, uint64_t r) {
    ReadPlace p;
    const uint64_t L = s.read_len;
    if (!s.paired) {
        p.g = hash3(s.seed, r, 1) % s.n_genomes;
        p.rc = (int)(hash3(s.seed, r, 2) & 1);
        p.start = hash3(s.seed, r, 3) % (s.genome_len - L + 1);
        return p;
    }
    const uint64_t pair = r >> 1;
    const uint64_t F = synth_frag_len(s, pair);
    p.g = hash3(s.seed, pair, 1) % s.n_genomes;
    const int fstrand = (int)(hash3(s.seed, pair, 2) & 1);
    const uint64_t fs = hash3(s.seed, pair, 3) % (s.genome_len - F + 1);
    const int mate = (int)(r & 1);
    // fstrand 0: R1 = fwd head of fragment, R2 = rc of tail; fstrand 1: mirrored
    const int head = (mate == fstrand);
    p.start = head ? fs : fs + F - L;
    p.rc = head ? 0 : 1;
    return p;
}

MCAAT_HD int genome_base(const uint64_t *genome, uint64_t genome_len, uint64_t g, uint64_t i) {
    const uint64_t j = g * genome_len + i;
    return (int)((genome[j >> 5] >> (2 * (j & 31))) & 3);
}

MCAAT_HD int synth_base(const mcaat_synth_spec &s, const uint64_t *genome, const ReadPlace &p,
                        uint64_t r, uint64_t pos) {
    const uint64_t L = s.read_len;
    int b = p.rc ? 3 - genome_base(genome, s.genome_len, p.g, p.start + L - 1 - pos)
                 : genome_base(genome, s.genome_len, p.g, p.start + pos);
    if (s.error_rate > 0) {
        const uint64_t h = hash3(s.seed ^ 0xE77E77ULL, r, pos);
        const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
        if (u < s.error_rate) b = (b + 1 + (int)((h & 0xFF) % 3)) & 3;
    }
    return b;
}

// packed word w of the stream of reads [first, first + count) (fixed length L: the slice's
// read i = bases [i*L, i*L+L)); read indices stay global, so a rank's slice is exactly that
// part of the single-stream reads
MCAAT_HD uint64_t synth_word(const mcaat_synth_spec &s, const uint64_t *genome, uint64_t w, uint64_t first,
                             uint64_t count) {
    const uint64_t L = s.read_len, total = count * L;
    uint64_t v = 0;
    uint64_t j = w * 32;
    uint64_t r = j / L, pos = j - r * L;
    ReadPlace p = synth_place(s, first + r);
    for (int i = 0; i < 32 && j < total; ++i, ++j) {
        v |= (uint64_t)synth_base(s, genome, p, first + r, pos) << (2 * i);
        if (++pos == L) {
            pos = 0;
            ++r;
            if (r < count) p = synth_place(s, first + r);
        }
    }
    return v;
}
MCAAT_HD uint64_t synth_word(const mcaat_synth_spec &s, const uint64_t *genome, uint64_t w) {
    return synth_word(s, genome, w, 0, s.n_reads);
}

}  // namespace mcaat
