"""Regenerate tests/golden/*.json — oracle outputs on seeded synthetic inputs.

These are regression pins of the CPU restatement (the reference's own hot path cannot
be built here and ships no vectors). Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import mcaat_amd as M  # noqa: E402
import oracle as O  # noqa: E402

CASES = {
    "c1_k23": (dict(), 23, dict()),
    "c1_k27": (dict(), 27, dict()),
    "pe_err_k23": (dict(seed=7, n_genomes=4, genome_len=20_000, arrays_per_genome=2, spacers_per_array=8,
                        repeat_len_min=32, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36,
                        n_reads=24_000, error_rate=0.002, paired=True), 23, dict(threshold_multiplicity=5)),
    "low_thr_k23": (dict(seed=11, n_genomes=3, genome_len=15_000, arrays_per_genome=2, spacers_per_array=10,
                         repeat_len_min=30, repeat_len_max=34, spacer_len_min=30, spacer_len_max=34,
                         n_reads=12_000, error_rate=0.004), 23, dict(threshold_multiplicity=2)),
    "cluster5_k23": (dict(seed=21, n_genomes=1, genome_len=30_000, arrays_per_genome=1, spacers_per_array=40,
                          repeat_len_min=30, repeat_len_max=30, spacer_len_min=30, spacer_len_max=34,
                          n_reads=30_000), 23, dict(cluster_bound=5)),
}


def main():
    out_dir = os.path.dirname(os.path.abspath(__file__))
    for name, (spec_kw, k, params) in CASES.items():
        spec = M.SynthSpec(**spec_kw)
        packed, offs = M.synth_host(spec)
        g = O.OGraph.build(packed, offs, k, threads=4)
        keys, mult = g.arrays()
        res = g.cycle_finder(threads=1, **params)
        gold = {
            "spec": spec.__dict__,
            "k": k,
            "params": params,
            "D": int(g.size),
            "keys_xor": int(np.bitwise_xor.reduce(keys)),
            "mult_sum": int(mult.astype(np.uint64).sum()),
            "stats": res["stats"],
            "candidates": res["candidates"],
            "buckets": res["buckets"],
            "entries": [[s, c] for s, c in res["entries"]],
            "map_order": res["map_order"],
        }
        with open(os.path.join(out_dir, name + ".json"), "w") as f:
            json.dump(gold, f, separators=(",", ":"))
        print(name, gold["D"], gold["stats"])


if __name__ == "__main__":
    main()
