"""Spacer ordering (spacer_ordering.cpp:460-754) with the constraints as (distinct pair,
multiplicity) in first-occurrence order (mcaat_amd/host/array_order.cpp, the CLI's path) against
the reference's list form (MCAAT_ORDER_REF=1): the same CRISPR_Arrays.txt and the same printed
orders, constraint counts and confidences, on multi-array read sets with sequencing errors."""
import os

import numpy as np
import pytest

import mcaat_amd as M
import mcaat_amd.downstream as DS
import oracle as O
from tests.helpers import unpack_read

CASES = [
    M.SynthSpec(seed=21, n_genomes=3, genome_len=20_000, arrays_per_genome=1, spacers_per_array=9,
                repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36, n_reads=15_000,
                error_rate=0.001),
    M.SynthSpec(seed=5, n_genomes=4, genome_len=30_000, arrays_per_genome=2, spacers_per_array=12,
                repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36, n_reads=30_000,
                error_rate=0.002),
    M.SynthSpec(seed=8, n_genomes=2, genome_len=40_000, arrays_per_genome=3, spacers_per_array=20,
                repeat_len_min=28, repeat_len_max=32, spacer_len_min=30, spacer_len_max=34, n_reads=30_000,
                error_rate=0.0),
]


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_weighted_constraints_equal_list_form(tmp_path, capfd, ci):
    spec = CASES[ci]
    k, thr = 23, 5
    packed, offs = M.synth_host(spec)
    og = O.OGraph.build(packed, offs, k, threads=4)
    res = og.cycle_finder(threshold_multiplicity=thr, threads=1)
    ent = res["entries"]
    cycles = [c for i in res["map_order"] for c in ent[i][1]]
    assert cycles, "the fixture must yield cycles"
    nodes = sorted({x for c in cycles for x in c})
    seqs = [unpack_read(packed, int(offs[i]), int(offs[i + 1])) for i in range(len(offs) - 1)]
    reads = og.get_reads(seqs, len(seqs), nodes)
    keys, mult = og.arrays()
    outs = {}
    for ref in ("1", "0"):
        os.environ["MCAAT_ORDER_REF"] = ref
        try:
            valid = og.valid().astype(np.uint8).copy()
            path = tmp_path / f"arrays_{ref}.txt"
            capfd.readouterr()
            n = DS.crispr_arrays(k, keys, mult, valid, cycles, reads, str(path))
            printed = [ln for ln in capfd.readouterr().out.splitlines()
                       if "order is" in ln or "constraints" in ln or "confidence" in ln]
            outs[ref] = (n, path.read_text(), printed)
        finally:
            os.environ.pop("MCAAT_ORDER_REF", None)
    assert outs["0"] == outs["1"]
    assert outs["0"][2], "no subproblem was solved"


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_step7_threads_equal_serial(tmp_path, capfd, ci):
    """Step 7 solves its independent subproblems on host threads; everything it prints and the
    CRISPR_Arrays.txt it leads to (all_systems' insertion order) equal the serial loop's."""
    spec = CASES[ci]
    k, thr = 23, 5
    packed, offs = M.synth_host(spec)
    og = O.OGraph.build(packed, offs, k, threads=4)
    res = og.cycle_finder(threshold_multiplicity=thr, threads=1)
    ent = res["entries"]
    cycles = [c for i in res["map_order"] for c in ent[i][1]]
    nodes = sorted({x for c in cycles for x in c})
    seqs = [unpack_read(packed, int(offs[i]), int(offs[i + 1])) for i in range(len(offs) - 1)]
    reads = og.get_reads(seqs, len(seqs), nodes)
    keys, mult = og.arrays()
    outs = {}
    for threads in (1, 3, 8):
        valid = og.valid().astype(np.uint8).copy()
        path = tmp_path / f"arrays_{threads}.txt"
        capfd.readouterr()
        n = DS.crispr_arrays(k, keys, mult, valid, cycles, reads, str(path), threads=threads)
        printed = [ln for ln in capfd.readouterr().out.splitlines()
                   if not ln.startswith("TIMING") and "Time elapsed" not in ln]
        outs[threads] = (n, path.read_text(), printed, valid.tobytes())
    assert outs[1] == outs[3] == outs[8]
    assert sum("Subproblem" in ln for ln in outs[1][2]) >= 2, "the fixture must hold several subproblems"
