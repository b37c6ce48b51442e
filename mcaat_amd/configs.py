"""Workload configs of BASELINE.json: the synthetic communities the bench,
the full-size GPU tests and the multi-rank checks share, so every one of them names the same
input. Each entry: spec (the whole dataset), k, thr (threshold_multiplicity), name, and a
coverage-matched CPU-baseline sample in the same D/N_occ regime."""
from __future__ import annotations

from .lib import SynthSpec

CONFIGS = {
    # C3: 300 Mbp community (200 genomes x 1.5 Mbp, 2 arrays each), 300M SE reads, k=27
    "c3": dict(spec=SynthSpec(seed=3, n_genomes=200, genome_len=1_500_000, arrays_per_genome=2,
                                spacers_per_array=12, repeat_len_min=30, repeat_len_max=36, spacer_len_min=30,
                                spacer_len_max=36, read_len=150, n_reads=300_000_000, error_rate=2.0e-4),
               k=27, thr=20, name="C3 1B-node synthetic metagenome (300M x 150bp SE, k=27, thr=20)",
               # CPU-baseline sample in the same regime: 150x coverage, D/N_occ ~ 0.027 as at C3
               sample=SynthSpec(seed=3, n_genomes=20, genome_len=100_000, arrays_per_genome=2, spacers_per_array=12,
                                  repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36,
                                  read_len=150, n_reads=2_000_000, error_rate=2.0e-4)),
    # C2: 50M PE reads (25M pairs) over a 400 Mbp community with 500 CRISPR arrays, 0.5 % errors
    # (250 genomes x 1.6 Mbp x 2 arrays: the generator places whole arrays per genome)
    "c2": dict(spec=SynthSpec(seed=2, n_genomes=250, genome_len=1_600_000, arrays_per_genome=2,
                                spacers_per_array=12, repeat_len_min=30, repeat_len_max=36, spacer_len_min=30,
                                spacer_len_max=36, read_len=150, n_reads=50_000_000, error_rate=5.0e-3, paired=True),
               k=27, thr=20, name="C2 50M PE synthetic metagenome (400 Mbp, 500 arrays, e=0.5%, k=27)",
               sample=SynthSpec(seed=2, n_genomes=40, genome_len=200_000, arrays_per_genome=2, spacers_per_array=12,
                                  repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36,
                                  read_len=150, n_reads=1_000_000, error_rate=5.0e-3, paired=True)),
    # C5: the low-abundance regime (include/settings.h:33-38 with threshold_multiplicity=2,
    # low_abundance=true, cycle min/max 27/77) on the C3 community, substitution errors raised
    # until the graph passes 2^31 edges (D ~ 4e9 is BASELINE's 8-GPU figure; this is the
    # largest D one GPU's 288 GB holds through the build)
    "c5": dict(spec=SynthSpec(seed=5, n_genomes=200, genome_len=1_500_000, arrays_per_genome=2,
                                spacers_per_array=12, repeat_len_min=30, repeat_len_max=36, spacer_len_min=30,
                                spacer_len_max=36, read_len=150, n_reads=300_000_000, error_rate=1.7e-3),
               k=27, thr=2, name="C5 low-abundance regime on one GPU (300M x 150bp SE, e=0.17%, k=27, thr=2, "
                                 "low_abundance, 27/77)",
               sample=SynthSpec(seed=5, n_genomes=20, genome_len=100_000, arrays_per_genome=2, spacers_per_array=12,
                                  repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36,
                                  read_len=150, n_reads=2_000_000, error_rate=1.7e-3)),
    "tiny": dict(spec=SynthSpec(), k=27, thr=20, name="C1 tiny (10k x 150bp, 50 kbp genome, k=27)",
                 sample=SynthSpec()),
}
