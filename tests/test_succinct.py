"""The succinct (BOSS) view of the graph (csrc/sdbg_succinct.hip, mcaat_graph_succinct_check):
W / last / W-minus nibbles per edge, sink and has-in bits per node, rank and select samples.
Every edge's valid out-neighbours (descending ids) and in-neighbours (ascending ids) by
rank/select equal those of the arrays the path runs on (out_info / in_info, themselves pinned
against the oracle in test_gpu_parity.py / test_scale_parity.py), on fresh graphs and after
CycleFinder has cleared valid bits; the out- and in-degree scans agree on both layouts."""
import pytest

import mcaat_amd as M
from mcaat_amd.configs import CONFIGS

pytestmark = pytest.mark.gpu

CASES = {
    "c1_k23": (M.SynthSpec(), 23, M.CfParams()),
    "c1_k27": (M.SynthSpec(), 27, M.CfParams()),
    "pe_err": (M.SynthSpec(seed=7, n_genomes=4, genome_len=20_000, arrays_per_genome=2, spacers_per_array=8,
                           repeat_len_min=32, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36,
                           n_reads=24_000, error_rate=0.002, paired=True), 23, M.CfParams(threshold_multiplicity=5)),
    "low_thr": (M.SynthSpec(seed=11, n_genomes=3, genome_len=15_000, arrays_per_genome=2, spacers_per_array=10,
                            repeat_len_min=30, repeat_len_max=34, spacer_len_min=30, spacer_len_max=34,
                            n_reads=12_000, error_rate=0.004), 23,
                M.CfParams(threshold_multiplicity=2, low_abundance=True)),
    # short k: many nodes with several out-edges, minus edges and multi-edge groups
    "k9_err": (M.SynthSpec(seed=13, n_genomes=2, genome_len=30_000, arrays_per_genome=1, spacers_per_array=6,
                           n_reads=8_000, error_rate=0.01), 9, M.CfParams(threshold_multiplicity=1000)),
    "c3_sample": (CONFIGS["c3"]["sample"], 27, M.CfParams(threshold_multiplicity=20)),
    "c5_sample": (CONFIGS["c5"]["sample"], 27, M.CfParams(threshold_multiplicity=2)),
}


@pytest.mark.parametrize("case", list(CASES))
def test_succinct_view_neighbours_equal_the_arrays(gpu_ctx, case):
    spec, k, prm = CASES[case]
    r = M.Reads.synth(gpu_ctx, spec)
    g = M.Graph.build(gpu_ctx, r, k)
    r.free()
    try:
        s = g.succinct_check()
        assert s["out_mismatch"] == 0 and s["in_mismatch"] == 0, s
        # every valid (edge, out-neighbour) pair counted once from each side
        assert s["outdeg_sum"] == s["indeg_sum"] > 0, s
        assert s["nodes"] >= s["sinks"] and s["view_bytes"] * 4 < s["array_bytes"], s
        g.cycle_finder(prm)  # clears valid bits (filter, peel)
        s2 = g.succinct_check()
        assert s2["out_mismatch"] == 0 and s2["in_mismatch"] == 0, s2
        assert s2["outdeg_sum"] == s2["indeg_sum"] < s["outdeg_sum"], (s, s2)
    finally:
        g.free()
