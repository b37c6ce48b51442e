"""CPU tests of the oracle (test infrastructure) — no GPU.

The oracle is "parity unpinned" (the reference's MEGAHIT-backed path cannot be built
here and ships no golden vectors). These tests pin it instead to:
  * brute-force pure-Python restatements of the SDBG conventions,
  * analytic known answers (a CRISPR array R S1 R ... Sn R yields exactly one cycle per
    spacer whose edges are the (k+1)-mers of the circular string R+Si),
  * a compiled libstdc++ probe of the unordered_set iteration order the GPU emulates,
  * committed regression fixtures (tests/golden/, made by tests/golden/make_golden.py).
"""
import json
import os
import random
import subprocess

import numpy as np
import pytest

import oracle as O
from tests.helpers import boss_key, brute_graph, brute_neighbors, lsb_value, pack_reads, rc

HERE = os.path.dirname(os.path.abspath(__file__))


def rand_seq(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


@pytest.mark.parametrize("k", [5, 6, 7, 11])
def test_count_canonical_matches_bruteforce(k):
    rng = random.Random(k)
    seqs = [rand_seq(rng, rng.randint(1, 60), "ACGT" if i % 3 else "AC") for i in range(80)]
    packed, offs = pack_reads(seqs)
    keys, counts = O.count_canonical(packed, offs, k)
    E = k + 1
    ref = {}
    for s in seqs:
        for i in range(len(s) - E + 1):
            e = s[i:i + E]
            c = min(lsb_value(e), lsb_value(rc(e)))
            ref[c] = ref.get(c, 0) + 1
    assert list(keys) == sorted(ref)
    assert list(counts) == [ref[x] for x in sorted(ref)]


@pytest.mark.parametrize("k", [4, 5, 7])
def test_sdbg_arrays_and_neighbors_match_bruteforce(k):
    rng = random.Random(100 + k)
    seqs = [rand_seq(rng, rng.randint(10, 40), "ACGT" if i % 2 else "ACG") for i in range(60)]
    seqs.append("ACGTACGT" * 3)  # palindromic edges for even k+1
    packed, offs = pack_reads(seqs)
    g = O.OGraph.build(packed, offs, k)
    edges, mult = brute_graph(seqs, k)
    keys, m = g.arrays()
    assert list(keys) == [boss_key(e, k) for e in edges]
    assert list(m) == [mult[e] for e in edges]
    out, inc = brute_neighbors(edges, k)
    for i in range(len(edges)):
        assert g.outgoing(i) == out[i]
        assert g.incoming(i) == inc[i]
        # GetLabel: source-node label, symbols 1..4 (tmp_utils.cpp:83-89)
        assert g.label(i) == ["ACGT".index(c) + 1 for c in edges[i][:k]]
    # IndexBinarySearch: last edge of the node with that label, -1 when absent
    for i, e in enumerate(edges):
        lab = [("ACGT".index(c) + 1) for c in e[:k]]
        j = g.index_binary_search(lab)
        assert edges[j][:k] == e[:k] and (j + 1 == len(edges) or edges[j + 1][:k] != e[:k])
    labels = {e[:k] for e in edges}
    import itertools

    missing = next(("".join(t) for t in itertools.product("ACGT", repeat=k) if "".join(t) not in labels), None)
    if missing is not None:
        assert g.index_binary_search(["ACGT".index(c) + 1 for c in missing]) == -1


def test_valid_only_degrees():
    seqs = ["ACGTTGCAAGGCTT" * 3, "ACGTTGCAAGGCTA" * 3]
    packed, offs = pack_reads(seqs)
    g = O.OGraph.build(packed, offs, 5)
    for e in range(g.size):
        outs = g.outgoing(e)
        if not outs:
            continue
        v = g.valid().copy()
        v[outs[0]] = 0
        g.set_valid(v)
        assert outs[0] not in g.outgoing(e)
        v[outs[0]] = 1
        g.set_valid(v)


def _peel_levels(g, tips):
    """Level-synchronous peel (the GPU's formulation): remove every valid seed tip with no
    valid successor, then every valid parent of a removed node whose valid out-degree is
    now zero, until nothing changes."""
    v = g.valid().copy()
    n = g.size
    # static adjacency (valid-only queries would hide removed nodes' parents)
    g.set_valid(np.ones(n, dtype=np.uint8))
    succ = [g.outgoing(x) for x in range(n)]
    pred = [g.incoming(x) for x in range(n)]
    g.set_valid(v)
    frontier = [t for t in range(n) if tips[t] and v[t] and not any(v[y] for y in succ[t])]
    while frontier:
        for t in frontier:
            v[t] = 0
        nxt = {p for t in frontier for p in pred[t] if v[p] and not any(v[y] for y in succ[p])}
        frontier = sorted(nxt)
    return v


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_recursive_reduction_is_order_independent_fixpoint(seed):
    rng = random.Random(seed)
    base = rand_seq(rng, 300)
    seqs = []
    for _ in range(120):
        a = rng.randint(0, 260)
        s = list(base[a:a + rng.randint(20, 40)])
        for j in range(len(s)):
            if rng.random() < 0.03:
                s[j] = rng.choice("ACGT")
        seqs.append("".join(s))
    packed, offs = pack_reads(seqs)
    g = O.OGraph.build(packed, offs, 7)
    tips = g.collect_tips()
    g.invalidate_mult_one()
    g2 = O.OGraph.build(packed, offs, 7)
    g2.invalidate_mult_one()
    g.recursive_reduction(tips)
    v_level = _peel_levels(g2, tips)
    assert np.array_equal(g.valid(), v_level)


def _array_genome(rng, rep_len, spacers, flank=400):
    R = rand_seq(rng, rep_len)
    S = [rand_seq(rng, rng.randint(30, 34)) for _ in range(spacers)]
    arr = R + "".join(s + R for s in S)
    return rand_seq(rng, flank) + arr + rand_seq(rng, flank), R, S


@pytest.mark.parametrize("k", [21, 23])
def test_known_answer_one_cycle_per_spacer(k):
    rng = random.Random(k * 7)
    genome, R, S = _array_genome(rng, 30, 7)
    # perfect tiling reads, both strands, 60x
    reads = []
    for i in range(0, len(genome) - 100 + 1, 5):
        reads.append(genome[i:i + 100])
        reads.append(rc(genome[i:i + 100]))
    packed, offs = pack_reads(reads)
    g = O.OGraph.build(packed, offs, k)
    keys, _ = g.arrays()
    E = k + 1
    res = g.cycle_finder(threshold_multiplicity=5)
    assert res["stats"][5] == 2 * len(S)  # both strands
    # expected cycle edge sets: (k+1)-mers of the circular strings R+Si and their rc
    expected = set()
    for sp in S:
        circ = R + sp
        ext = circ + circ[:E]
        expected.add(frozenset(boss_key(ext[i:i + E], k) for i in range(len(circ))))
        rcc = rc(circ)
        ext = rcc + rcc[:E]
        expected.add(frozenset(boss_key(ext[i:i + E], k) for i in range(len(rcc))))
    got = set()
    for start, cycles in res["entries"]:
        for c in cycles:
            assert c[0] == start
            assert len(c) == len(set(c))
            got.add(frozenset(int(keys[x]) for x in c))
    assert got == expected


def test_unordered_set_order_model_matches_libstdcxx(tmp_path):
    """The GPU FindCycle emulates libstdc++ unordered_set<uint64_t> iteration order for
    <= 4 elements (13 buckets, identity hash): a new element goes before the first element
    of its bucket, or to the front when the bucket is empty; erase/copy keep the order."""
    src = tmp_path / "probe.cpp"
    src.write_text(r'''
#include <unordered_set>
#include <cstdio>
#include <cstdint>
int main(){ uint64_t v; int n;
  while (scanf("%d", &n) == 1) { std::unordered_set<uint64_t> s;
    for (int i = 0; i < n; ++i) { scanf("%lu", &v); s.insert(v); }
    std::unordered_set<uint64_t> c = s; for (auto x : c) printf("%lu ", x); printf("\n"); } }''')
    exe = tmp_path / "probe"
    subprocess.run(["g++", "-O1", "-std=c++17", str(src), "-o", str(exe)], check=True)
    rng = random.Random(5)
    cases = []
    for t in range(3000):
        n = rng.randint(1, 4)
        cases.append([rng.randrange(60) if t % 2 else rng.randrange(1 << 40) for _ in range(n)])
    inp = "".join(f"{len(c)} " + " ".join(map(str, c)) + "\n" for c in cases)
    out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()

    def model(ins):
        L = []
        for x in ins:
            if x in L:
                continue
            pos = next((i for i, y in enumerate(L) if y % 13 == x % 13), 0)
            L.insert(pos, x)
        return L

    for c, line in zip(cases, out):
        assert [int(x) for x in line.split()] == model(c)


def test_dls_requires_cycle_within_limit():
    # a single cycle of length 40 edges through a branching node
    rng = random.Random(9)
    loop = rand_seq(rng, 40)
    tail = rand_seq(rng, 30)
    genome = tail + loop * 4 + rand_seq(rng, 30)
    reads = [genome[i:i + 60] for i in range(0, len(genome) - 60 + 1, 2)]
    reads += [rc(r) for r in reads]
    packed, offs = pack_reads(reads)
    g = O.OGraph.build(packed, offs, 9)
    keys, mult = g.arrays()
    branching = [e for e in range(g.size) if len(g.incoming(e)) >= 2]
    assert branching
    for e in branching:
        assert g.dls(e, limit=77)          # the 40-edge loop is within the limit
        assert not g.dls(e, limit=30)      # ... but not within 30


GOLDEN = os.path.join(HERE, "golden")


@pytest.mark.parametrize("name", sorted(f[:-5] for f in os.listdir(GOLDEN) if f.endswith(".json")))
def test_golden_regression(name):
    """Committed oracle outputs (regression pins of the restatement, not reference outputs)."""
    import mcaat_amd as M

    with open(os.path.join(GOLDEN, name + ".json")) as f:
        gold = json.load(f)
    spec = M.SynthSpec(**gold["spec"])
    packed, offs = M.synth_host(spec)
    g = O.OGraph.build(packed, offs, gold["k"], threads=2)
    keys, mult = g.arrays()
    assert g.size == gold["D"]
    assert int(np.bitwise_xor.reduce(keys)) == gold["keys_xor"]
    assert int(mult.astype(np.uint64).sum()) == gold["mult_sum"]
    res = g.cycle_finder(**gold["params"])
    assert res["stats"] == gold["stats"]
    assert res["candidates"] == gold["candidates"]
    assert res["buckets"] == gold["buckets"]
    assert [[s, c] for s, c in res["entries"]] == gold["entries"]
    assert res["map_order"] == gold["map_order"]


# reference tests/test_reads.cpp:10-62 (ReadsTest.*): reverse_pair_ends_sequence vectors
@pytest.mark.parametrize("inp,expected", [
    ("ACGT", "ACGT"), ("ACGTT", "AACGT"), ("AAGCT", "AGCTT"), ("AXGT", "ACXT"),
    ("XXXQUIOCPOPYM", "MYPOPGOIUQXXX"),
])
def test_reverse_pair_ends_reference_vectors(inp, expected):
    assert O.reverse_pair_ends(inp) == expected


def test_get_reads_restatement_small():
    """reads.cpp:57-130 on a hand-checked case: ids of every k-mer for reads whose first or
    last k-mer maps to a cycle node; reads of length <= 2k skipped; N maps like T."""
    k = 4
    seqs = ["ACGTACGGTCAG", "TTTTGGGGCCCCAAAA"]
    packed, offs = pack_reads(seqs)
    g = O.OGraph.build(packed, offs, k)
    enc = {"A": 1, "C": 2, "G": 3, "T": 4}
    ibs = lambda s: g.index_binary_search([enc.get(c, 4) for c in s]) % (1 << 64)
    first = ibs(seqs[0][:k])
    got = g.get_reads(seqs + ["ACGTNCGGTCAG", "ACGTACGG"], 4, [first])
    want0 = [ibs(seqs[0][i:i + k]) for i in range(len(seqs[0]) - k + 1)]
    want2 = [ibs("ACGTNCGGTCAG"[i:i + k]) for i in range(12 - k + 1)]
    assert got == [want0, want2]


def test_oracle_c_fastq_reader_matches_fastx_restatement(tmp_path):
    """The C FASTQ reader of the CPU baseline (oracle_read_fastq) gives the counting view of
    the Python restatement (oracle/fastx.py): reads split at non-ACGT, lowercase, CRLF."""
    from oracle import fastx as FX

    rng = np.random.default_rng(9)
    seqs = ["".join(rng.choice(list("ACGTacgtN"), size=int(rng.integers(0, 200)))) for _ in range(300)]
    text = "".join(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n" for i, s in enumerate(seqs))
    for crlf in (False, True):
        f = tmp_path / f"x{int(crlf)}.fq"
        f.write_bytes((text.replace("\n", "\r\n") if crlf else text).encode())
        packed, offs = O.read_fastq(str(f))
        want_p, want_o = FX.pack_bases(FX.counting_view(FX.fastq_sequences(text)))
        assert np.array_equal(offs, want_o)
        nw = (int(want_o[-1]) + 31) // 32
        assert packed.size == nw and np.array_equal(packed, want_p[:nw])
    bad = tmp_path / "bad.fq"
    bad.write_text("@r\nACGT\n+\n")
    with pytest.raises(ValueError):
        O.read_fastq(str(bad))


def test_id_convention_relabelling(tmp_path):
    """edge ids here leave out MEGAHIT's `$` dummy edges, so a real mcaat run
    numbers the same edges id' = f(id) for an increasing f (dummies interleaved). Two outputs
    depend on the id VALUES, not only on their order:
      (1) results' libstdc++ iteration order, i.e. the order cycles_map_to_cycles
          (tmp_utils.cpp:26-38) hands the cycles to steps 7-8;
      (2) FindCycle's <= 4-element neighbour sets (unordered_set, identity hash mod 13,
          cycle_finder.cpp:58-88): the out-sets are invariant (consecutive ids), the in-sets
          used by the lock relaxation are not.
    (1) is checked invariant where it should be: on multi-array fixtures CRISPR_Arrays.txt is
    the same when the cycles come in the relabelled map's order (a compiled libstdc++ probe,
    pinned against the oracle's own map order). (2) out-sets are shown invariant and in-sets NOT:
    the relaxation visits in-edges in another order, which changes nothing in the lock values it
    reaches (a fixpoint) but is where the numbering could show. Everything ordered by
    id (candidate lists, buckets' ascending order, DESCENDING out / ASCENDING in neighbours) is
    invariant under any increasing f."""
    import mcaat_amd as M
    import mcaat_amd.downstream as DS
    from tests.helpers import unpack_read

    src = tmp_path / "mapprobe.cpp"
    src.write_text(r'''
#include <unordered_map>
#include <cstdio>
#include <cstdint>
#include <vector>
int main(){ int n; while (scanf("%d", &n) == 1) { std::unordered_map<uint64_t, int> m; uint64_t v;
  for (int i = 0; i < n; ++i) { scanf("%lu", &v); m[v] = i; }
  for (auto &kv : m) printf("%d ", kv.second); printf("\n"); } }''')
    exe = tmp_path / "mapprobe"
    subprocess.run(["g++", "-O1", "-std=c++17", str(src), "-o", str(exe)], check=True)

    def map_order(keys):
        inp = f"{len(keys)} " + " ".join(map(str, keys)) + "\n"
        out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True).stdout
        return [int(x) for x in out.split()]

    specs = [M.SynthSpec(seed=21, n_genomes=3, genome_len=20_000, arrays_per_genome=1, spacers_per_array=9,
                         repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36, n_reads=15_000,
                         error_rate=0.001),
             M.SynthSpec(seed=5, n_genomes=4, genome_len=30_000, arrays_per_genome=2, spacers_per_array=12,
                         repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36, n_reads=30_000,
                         error_rate=0.002)]
    rng = np.random.default_rng(3)
    changed_order = 0
    for si, spec in enumerate(specs):
        k = 23
        packed, offs = M.synth_host(spec)
        og = O.OGraph.build(packed, offs, k, threads=4)
        res = og.cycle_finder(threshold_multiplicity=5, threads=1)
        ent = res["entries"]
        starts = [int(s) for s, _ in ent]
        assert map_order(starts) == res["map_order"], "the probe must reproduce the oracle's map order"
        # an increasing relabelling: 0..3 dummies before every edge
        f = np.cumsum(rng.integers(0, 4, size=og.size + 1)).astype(np.int64) + np.arange(og.size + 1)
        relab = map_order([int(f[s]) for s in starts])
        changed_order += relab != res["map_order"]
        seqs = [unpack_read(packed, int(offs[i]), int(offs[i + 1])) for i in range(len(offs) - 1)]
        keys, mult = og.arrays()
        texts = []
        for order in (res["map_order"], relab):
            cycles = [c for i in order for c in ent[i][1]]
            nodes = sorted({x for c in cycles for x in c})
            reads = og.get_reads(seqs, len(seqs), nodes)
            valid = og.valid().astype(np.uint8).copy()
            path = tmp_path / f"arrays_{si}_{len(texts)}.txt"
            DS.crispr_arrays(k, keys, mult, valid, cycles, reads, str(path))
            texts.append(path.read_text())
        assert texts[0] == texts[1], f"spec {si}: CRISPR_Arrays.txt depends on results' iteration order"
        assert "Number of Systems: 0" not in texts[0]
    assert changed_order, "the relabelling should move results' iteration order on these fixtures"

    # (2) neighbour-set order is NOT invariant: a shift by dummies reorders some <= 4-element sets
    def set_order(ins):
        L = []
        for x in ins:
            if x not in L:
                L.insert(next((i for i, y in enumerate(L) if y % 13 == x % 13), 0), x)
        return L

    # Out-neighbour sets are a node's out-edges: consecutive ids (siblings differ only in W, so
    # no dummy falls between them), a span below 13, distinct buckets: the order is the reverse
    # insertion order whatever the values, and stays. In-neighbour sets are up to 4 positions of
    # a 16-edge (k-1)-suffix group, which a dummy `$`-edge with that suffix can join: the span
    # and the residues mod 13 change unevenly (a uniform shift would keep every collision).
    f = np.cumsum(rng.integers(0, 2, size=1 << 16)) + np.arange(1 << 16)
    inv = {int(y): x for x, y in enumerate(f)}
    out_moved = in_moved = 0
    for _ in range(2000):
        lo = int(rng.integers(0, (1 << 16) - 20))
        outs = list(range(lo, lo + int(rng.integers(2, 5))))[::-1]  # OutgoingEdges: descending
        out_moved += set_order(outs) != [inv[y] for y in set_order([int(f[x]) for x in outs])]
        ins = sorted(lo + int(x) for x in rng.choice(16, size=int(rng.integers(2, 5)), replace=False))
        in_moved += set_order(ins) != [inv[y] for y in set_order([int(f[x]) for x in ins])]
    assert out_moved == 0 and in_moved > 0
