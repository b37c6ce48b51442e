"""Minimal driver for rocprofv3 runs: synth reads -> build -> cycle_finder, with progress."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mcaat_amd as M  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
stage = sys.argv[2] if len(sys.argv) > 2 else "all"
spec = M.SynthSpec(seed=3, n_genomes=200, genome_len=1_500_000, arrays_per_genome=2, spacers_per_array=12,
                   repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36, read_len=150,
                   n_reads=n, error_rate=2.0e-4)
t = time.time()
with M.Context(0) as ctx:
    print("ctx", time.time() - t, flush=True)
    reads = M.Reads.synth(ctx, spec)
    print("synth", time.time() - t, flush=True)
    g = M.Graph.build(ctx, reads, 27)
    print("build", time.time() - t, g.size, flush=True)
    if stage == "all":
        r = g.cycle_finder(M.CfParams())
        print("cf", time.time() - t, len(r.entries), flush=True)
    g.free()
    reads.free()
print("done", time.time() - t, flush=True)
