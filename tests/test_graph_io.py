"""Graph checkpoint / resume (mcaat_graph_save / mcaat_graph_load; SURVEY.md §8f rank 4 in the
library's own format — MEGAHIT's graph.sdbg* is unpinned offline). Round trips: a loaded graph
answers every query as the saved one (keys, multiplicities, valid bits, neighbours) and
CycleFinder on it gives the oracle's results; a graph saved after CycleFinder keeps its valid
bits; damaged files fail loudly; the CLI resumes from a kept graph with the same cycles."""
import os
import subprocess

import numpy as np
import pytest

import mcaat_amd as M
import oracle as O
from tests.helpers import unpack_read

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SPEC = M.SynthSpec(seed=7, n_genomes=4, genome_len=20_000, arrays_per_genome=2, spacers_per_array=8,
                   repeat_len_min=32, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36,
                   n_reads=24_000, error_rate=0.002, paired=True)
K = 23
PRM = M.CfParams(threshold_multiplicity=5)


def _same_graph(a, b):
    ka, ma, va = a.download()
    kb, mb, vb = b.download()
    assert a.size == b.size and a.info()[0] == b.info()[0]
    assert np.array_equal(ka, kb) and np.array_equal(ma, mb) and np.array_equal(va, vb)
    ids = np.random.default_rng(1).choice(a.size, size=min(a.size, 4000), replace=False).astype(np.uint64)
    for inc in (False, True):
        oa, ca = a.neighbors(ids, incoming=inc)
        ob, cb = b.neighbors(ids, incoming=inc)
        assert np.array_equal(ca, cb) and np.array_equal(oa, ob)


def test_round_trip_then_cycle_finder(gpu_ctx, tmp_path):
    reads = M.Reads.synth(gpu_ctx, SPEC)
    g = M.Graph.build(gpu_ctx, reads, K)
    path = str(tmp_path / "g.mcaat_sdbg")
    g.save(path)
    h = M.Graph.load(gpu_ctx, path)
    _same_graph(g, h)
    res = h.cycle_finder(PRM)
    packed, offs = M.synth_host(SPEC)
    ores = O.OGraph.build(packed, offs, K, threads=4).cycle_finder(threshold_multiplicity=5)
    assert res.stats[:6] == ores["stats"]
    assert [(s, c) for s, c in res.entries] == [tuple(e) for e in ores["entries"]]
    # saved after CycleFinder: the pruned valid bits come back
    h.save(path)
    _same_graph(h, M.Graph.load(gpu_ctx, path))


def test_empty_graph_round_trip(gpu_ctx, tmp_path):
    from tests.helpers import pack_reads

    packed, offs = pack_reads(["ACGT", "GATTACA"])
    g = M.Graph.build(gpu_ctx, M.Reads.from_host(gpu_ctx, packed, offs), 9)
    path = str(tmp_path / "e.mcaat_sdbg")
    g.save(path)
    assert M.Graph.load(gpu_ctx, path).size == 0


def test_damaged_files_fail_loudly(gpu_ctx, tmp_path):
    reads = M.Reads.synth(gpu_ctx, M.SynthSpec())
    g = M.Graph.build(gpu_ctx, reads, K)
    path = tmp_path / "g.mcaat_sdbg"
    g.save(str(path))
    data = bytearray(path.read_bytes())
    cases = {
        "flip": data[:1000] + bytes([data[1000] ^ 1]) + data[1001:],
        "trunc": data[: len(data) // 2],
        "magic": b"X" + data[1:],
    }
    for name, blob in cases.items():
        p = tmp_path / f"{name}.mcaat_sdbg"
        p.write_bytes(bytes(blob))
        with pytest.raises(M.McaatError):
            M.Graph.load(gpu_ctx, str(p))
    with pytest.raises(M.McaatError):
        M.Graph.load(gpu_ctx, str(tmp_path / "missing"))


def test_cli_keep_and_resume(tmp_path):
    packed, offs = M.synth_host(M.SynthSpec())
    fq = tmp_path / "r.fq"
    with open(fq, "w") as f:
        for r in range(len(offs) - 1):
            s = unpack_read(packed, int(offs[r]), int(offs[r + 1]))
            f.write(f"@r{r}\n{s}\n+\n{'I' * len(s)}\n")
    cli = os.path.join(ROOT, "mcaat_amd", "mcaat")
    a = subprocess.run([cli, "-i", str(fq), "--output-folder", str(tmp_path / "a"), "--keep-graph"],
                       capture_output=True, text=True, timeout=300)
    assert a.returncode == 0, a.stderr
    kept = tmp_path / "a" / "graph" / "graph.mcaat_sdbg"
    assert kept.exists()
    b = subprocess.run([cli, "-i", str(fq), "--output-folder", str(tmp_path / "b"), "--load-graph", str(kept)],
                       capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    assert "Resumed the graph" in b.stdout
    for name in ("cycles/cycles.txt", "CRISPR_Arrays.txt"):
        assert (tmp_path / "a" / name).read_text() == (tmp_path / "b" / name).read_text()
