"""Relevant-read mapping: the GPU get_reads (mcaat_map_reads) against
the oracle's line restatement of reads.cpp:20-130 on the same sequences and graph.

Bar: bit-exact node-id chains, same reads, same order. Inputs are FASTQ files written by the
test (single-end, paired-end with the second file reverse-complemented by the reference,
non-ACGT and lowercase symbols, reads no longer than 2k), so the product's parsing of the
mapping view is covered too. The oracle's reverse_pair_ends_sequence is pinned by the
reference's own test vectors in tests/test_oracle.py.
"""
import os

import numpy as np
import pytest

import mcaat_amd as M
import oracle as O
from tests.helpers import unpack_read

pytestmark = pytest.mark.gpu


def _write_fastq(path, seqs):
    with open(path, "w") as f:
        for i, s in enumerate(seqs):
            f.write(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")


def _cycle_nodes(res):
    return sorted({x for _, cycles in res.entries for c in cycles for x in c})


def _run(ctx, tmp_path, seqs1, seqs2, k, prm, max_batch_ids=0):
    files = [str(tmp_path / "r1.fq")]
    _write_fastq(files[0], seqs1)
    if seqs2 is not None:
        files.append(str(tmp_path / "r2.fq"))
        _write_fastq(files[1], seqs2)
    reads = M.Reads.from_fastx(ctx, files)
    g = M.Graph.build(ctx, reads, k)
    keys, mult, _ = g.download()
    res = g.cycle_finder(prm)
    nodes = _cycle_nodes(res)
    mapped = g.map_reads(reads, np.array(nodes, dtype=np.uint64), max_batch_ids=max_batch_ids)
    og = O.OGraph.from_arrays(keys, mult, k)
    want = og.get_reads(list(seqs1) + list(seqs2 or []), len(seqs1), nodes)
    got = [mapped.read(i) for i in range(len(mapped))]
    return reads, nodes, got, want


def _synth_seqs(spec):
    packed, offs = M.synth_host(spec)
    return [unpack_read(packed, int(offs[i]), int(offs[i + 1])) for i in range(len(offs) - 1)]


def test_map_reads_single_end(gpu_ctx, tmp_path):
    seqs = _synth_seqs(M.SynthSpec())
    reads, nodes, got, want = _run(gpu_ctx, tmp_path, seqs, None, 23, M.CfParams())
    assert reads.records_info() == (len(seqs), False)  # one ACGT-only file: the counting view
    assert len(nodes) > 0 and len(want) > 0
    assert got == want


def test_map_reads_paired_end_with_ambiguous_symbols(gpu_ctx, tmp_path):
    spec = M.SynthSpec(seed=5, n_reads=12_000)
    seqs = _synth_seqs(spec)
    rng = np.random.default_rng(3)
    s1, s2 = [], []
    for i, s in enumerate(seqs):
        s = list(s)
        if i % 37 == 0:
            s[int(rng.integers(len(s)))] = "N"
        if i % 53 == 0:
            j = int(rng.integers(len(s)))
            s[j] = s[j].lower()
        s = "".join(s)
        if i % 101 == 0:
            s = s[:40]  # <= 2k: never relevant
        # half of the pairs: the second file holds the reverse complement (as sequencers write R2)
        if i % 2:
            s2.append(s[::-1].translate(str.maketrans("ACGTacgt", "TGCAtgca")))
        else:
            s1.append(s)
    reads, nodes, got, want = _run(gpu_ctx, tmp_path, s1, s2, 23, M.CfParams())
    n_rec, separate = reads.records_info()
    assert separate and n_rec == len(s1) + len(s2)
    assert len(want) > 0
    assert got == want


def test_map_reads_small_batches(gpu_ctx, tmp_path):
    seqs = _synth_seqs(M.SynthSpec(seed=9))
    _, _, got, want = _run(gpu_ctx, tmp_path, seqs, None, 27, M.CfParams(), max_batch_ids=300)
    assert len(want) > 2
    assert got == want


def test_map_reads_edge_cases(gpu_ctx):
    spec = M.SynthSpec(n_reads=3000)
    reads = M.Reads.synth(gpu_ctx, spec)
    g = M.Graph.build(gpu_ctx, reads, 23)
    # no cycle nodes -> no reads
    assert len(g.map_reads(reads, np.zeros(0, dtype=np.uint64))) == 0
    # every edge a "cycle node": every read longer than 2k is relevant, ids match the oracle
    keys, mult, _ = g.download()
    allnodes = np.arange(keys.size, dtype=np.uint64)
    m = g.map_reads(reads, allnodes, max_batch_ids=1000)
    packed, offs = M.synth_host(spec)
    seqs = [unpack_read(packed, int(offs[i]), int(offs[i + 1])) for i in range(len(offs) - 1)]
    og = O.OGraph.from_arrays(keys, mult, 23)
    want = og.get_reads(seqs, len(seqs), allnodes.tolist())
    assert len(m) == len(want) == len(seqs)
    assert [m.read(i) for i in range(len(m))] == want
    assert np.array_equal(m.records, np.arange(len(seqs), dtype=np.uint64))
