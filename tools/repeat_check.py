"""Determinism check: build the C3 graph several times in one process (arena reuse)."""
import hashlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mcaat_amd as M
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
spec = M.SynthSpec(seed=3, n_genomes=200, genome_len=1_500_000, arrays_per_genome=2, spacers_per_array=12,
                   repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36, read_len=150,
                   n_reads=n, error_rate=2.0e-4)
with M.Context(0) as ctx:
    r = M.Reads.synth(ctx, spec)
    for i in range(reps):
        g = M.Graph.build(ctx, r, 27)
        k, m, v = g.download()
        print(i, "graph", len(k), hashlib.md5(k.tobytes()).hexdigest(), hashlib.md5(m.tobytes()).hexdigest(), flush=True)
        g.free()
