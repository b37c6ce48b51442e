"""GPU parity: every stage of the HIP path against the CPU oracle on the same seeded inputs.

Bar: bit-exact (integer/index work). Calls go through the C ABI (libmcaat_gpu.so).
Oracle parity status: "parity unpinned"  — the oracle itself is
checked by tests/test_oracle.py against brute-force restatements and analytic answers.
"""
import numpy as np
import pytest

import mcaat_amd as M
import oracle as O
from tests.helpers import pack_reads

pytestmark = pytest.mark.gpu

CONFIGS = {
    # C1 tiny: one 50 kbp genome, one array (repeat 30, spacer 32, 12 copies)
    "c1_k23": (M.SynthSpec(), 23, M.CfParams()),
    "c1_k27": (M.SynthSpec(), 27, M.CfParams()),
    # errors, several genomes/arrays, paired-end, ragged repeat/spacer lengths
    "pe_err": (M.SynthSpec(seed=7, n_genomes=4, genome_len=20_000, arrays_per_genome=2, spacers_per_array=8,
                           repeat_len_min=32, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36,
                           n_reads=24_000, error_rate=0.002, paired=True), 23, M.CfParams(threshold_multiplicity=5)),
    # low-abundance mode: threshold 2 -> many candidates and conflicting speculative starts
    "low_thr": (M.SynthSpec(seed=11, n_genomes=3, genome_len=15_000, arrays_per_genome=2, spacers_per_array=10,
                            repeat_len_min=30, repeat_len_max=34, spacer_len_min=30, spacer_len_max=34,
                            n_reads=12_000, error_rate=0.004), 23,
                M.CfParams(threshold_multiplicity=2, low_abundance=True)),
    "low_abundance_false": (M.SynthSpec(seed=12, n_genomes=2, genome_len=12_000, arrays_per_genome=1,
                                        spacers_per_array=6, n_reads=8_000, error_rate=0.003), 21,
                            M.CfParams(threshold_multiplicity=3, low_abundance=False, cycle_min_length=20,
                                       cycle_max_length=70)),
}


def _oracle_graph(packed, offs, k):
    return O.OGraph.build(packed, offs, k, threads=4)


@pytest.fixture(scope="module", params=sorted(CONFIGS))
def case(request, gpu_ctx):
    spec, k, prm = CONFIGS[request.param]
    packed, offs = M.synth_host(spec)
    reads = M.Reads.synth(gpu_ctx, spec)
    return request.param, spec, k, prm, packed, offs, reads


def test_synth_reads_device_equals_host(case):
    _, spec, _, _, packed, offs, reads = case
    dp, do = reads.download()
    assert np.array_equal(do, offs)
    assert np.array_equal(dp[: packed.size], packed)


def test_node_counter_parity(case, gpu_ctx):
    _, _, k, _, packed, offs, reads = case
    gk, gc = M.count_edges(gpu_ctx, reads, k)
    ok, oc = O.count_canonical(packed, offs, k, threads=4)
    assert gk.size == ok.size
    assert np.array_equal(gk, ok)
    assert np.array_equal(gc, oc)


def test_sdbg_build_parity(case, gpu_ctx):
    _, _, k, _, packed, offs, reads = case
    g = M.Graph.build(gpu_ctx, reads, k)
    og = _oracle_graph(packed, offs, k)
    keys, mult, valid = g.download()
    okeys, omult = og.arrays()
    assert g.size == og.size
    assert np.array_equal(keys, okeys)
    assert np.array_equal(mult, omult)
    assert valid.all()
    # neighbour queries (valid-only, DESCENDING out / ASCENDING in) on a sample of edges
    rng = np.random.default_rng(0)
    ids = rng.choice(g.size, size=min(g.size, 3000), replace=False).astype(np.uint64)
    out, oc = g.neighbors(ids, incoming=False)
    inn, ic = g.neighbors(ids, incoming=True)
    for i, e in enumerate(ids):
        assert list(out[i, : oc[i]]) == og.outgoing(int(e))
        assert list(inn[i, : ic[i]]) == og.incoming(int(e))


def test_cycle_finder_parity(case, gpu_ctx):
    name, _, k, prm, packed, offs, reads = case
    g = M.Graph.build(gpu_ctx, reads, k)
    res = g.cycle_finder(prm)
    og = _oracle_graph(packed, offs, k)
    ores = og.cycle_finder(threshold_multiplicity=prm.threshold_multiplicity, low_abundance=prm.low_abundance,
                           cycle_max_length=prm.cycle_max_length, cycle_min_length=prm.cycle_min_length, threads=1)
    assert res.stats[:6] == ores["stats"], name
    assert res.candidates == ores["candidates"]
    assert res.buckets == ores["buckets"]
    assert len(res.entries) == len(ores["entries"])
    for (s, cyc), (os_, ocyc) in zip(res.entries, ores["entries"]):
        assert s == os_
        assert cyc == ocyc
    # post-prune / post-search valid bits equal
    _, _, valid = g.download()
    assert np.array_equal(valid, og.valid())


def test_fastx_reader_splits_on_n(gpu_ctx, tmp_path):
    seqs = ["ACGTACGTTTGACCA" * 6, "GGGTTTAAACCC" * 5 + "N" + "ACGATCGATCGGATTAC" * 3, "ACGTNNACGT"]
    fq = tmp_path / "r.fq"
    with open(fq, "w") as f:
        for i, s in enumerate(seqs):
            f.write(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")
    reads = M.Reads.from_fastx(gpu_ctx, [str(fq)])
    parts = []
    for s in seqs:
        parts += [p for p in s.split("N") if p]
    packed, offs = pack_reads(parts)
    dp, do = reads.download()
    assert np.array_equal(do, offs)
    assert np.array_equal(dp[: packed.size], packed)
    gk, gc = M.count_edges(gpu_ctx, reads, 11)
    ok, oc = O.count_canonical(packed, offs, 11)
    assert np.array_equal(gk, ok) and np.array_equal(gc, oc)


def test_edge_cases_empty_and_short(gpu_ctx):
    # reads shorter than k+1 contribute nothing; an all-short input gives an empty graph
    packed, offs = pack_reads(["ACGT", "GATTACA", "A"])
    reads = M.Reads.from_host(gpu_ctx, packed, offs)
    g = M.Graph.build(gpu_ctx, reads, 9)
    assert g.size == 0
    res = g.cycle_finder(M.CfParams())
    assert res.entries == [] and res.stats[:6] == [0, 0, 0, 0, 0, 0]


def test_palindromes_and_homopolymers(gpu_ctx):
    # palindromic (k+1)-mers (k+1 even) and a poly-A self-loop edge
    pal = "ACGTACGT"  # rc(ACGTACGT) == ACGTACGT
    seqs = [pal * 20, "A" * 60, "T" * 30 + pal + "GGCC" * 10]
    packed, offs = pack_reads(seqs)
    reads = M.Reads.from_host(gpu_ctx, packed, offs)
    for k in (7, 9):
        g = M.Graph.build(gpu_ctx, reads, k)
        og = O.OGraph.build(packed, offs, k)
        keys, mult, _ = g.download()
        okeys, omult = og.arrays()
        assert np.array_equal(keys, okeys) and np.array_equal(mult, omult)
        res = g.cycle_finder(M.CfParams(threshold_multiplicity=1, cycle_min_length=1, cycle_max_length=20))
        ores = og.cycle_finder(threshold_multiplicity=1, cycle_min_length=1, cycle_max_length=20)
        assert res.entries == [tuple(e) for e in ores["entries"]]
        assert res.stats[:6] == ores["stats"]


def test_cluster_bound_and_step_cap(gpu_ctx):
    # many spacers through one repeat: >= cluster_bound cycles -> empty entry (cycle_finder.cpp:162-165);
    # a tiny step cap truncates the search (cycle_finder.cpp:148-151)
    spec = M.SynthSpec(seed=21, n_genomes=1, genome_len=30_000, arrays_per_genome=1, spacers_per_array=40,
                       repeat_len_min=30, repeat_len_max=30, spacer_len_min=30, spacer_len_max=34, n_reads=30_000)
    packed, offs = M.synth_host(spec)
    reads = M.Reads.synth(gpu_ctx, spec)
    for bound, cap in ((5, 10_000_000), (500, 10_000_000), (500, 200), (3, 5000)):
        g = M.Graph.build(gpu_ctx, reads, 23)
        res = g.cycle_finder(M.CfParams(cluster_bound=bound, step_cap=cap))
        og = O.OGraph.build(packed, offs, 23)
        ores = og.cycle_finder(cluster_bound=bound, step_cap=cap)
        assert res.stats[:6] == ores["stats"], (bound, cap)
        assert [(s, c) for s, c in res.entries] == [tuple(e) for e in ores["entries"]], (bound, cap)


def test_lds_overflow_fallback_low_coverage(gpu_ctx):
    """Low coverage: almost every edge is distinct and every LDS partition overflows. By default
    the partitions are split down to eight classes (round 4); with the split depth of round 3
    (two bits) the global-table fallback counts the classes still over. Both equal the oracle."""
    spec = M.SynthSpec(seed=31, n_genomes=50, genome_len=1_000_000, arrays_per_genome=0, n_reads=60_000,
                       error_rate=0.01)
    packed, offs = M.synth_host(spec)
    reads = M.Reads.synth(gpu_ctx, spec)
    ok, oc = O.count_canonical(packed, offs, 27, threads=4)
    for depth in (3, 2):
        gpu_ctx.reset_timing()
        with gpu_ctx.knobs(nc__split_max=depth):
            gk, gc = M.count_edges(gpu_ctx, reads, 27)
        assert np.array_equal(gk, ok) and np.array_equal(gc, oc), depth
        if depth == 2:
            assert gpu_ctx.kernel_timing("lds_count_overflow_partitions")[1] > 0


@pytest.mark.parametrize("mini_w", ["", "14", "16"])
def test_descriptor_overflow_classes(gpu_ctx, monkeypatch, mini_w):
    """~2x coverage with 1% errors: fine partitions hold more distinct super-k-mers than the
    LDS descriptor table, so pass C counts them as edge-disjoint minimizer-hash classes (and
    sends classes whose edges overflow to the class-filtered global fallback). Also covers the
    minimizer-window knob. Counts must equal the oracle."""
    if mini_w:
        monkeypatch.setenv("MCAAT_MINI_W", mini_w)
    else:
        monkeypatch.delenv("MCAAT_MINI_W", raising=False)
    spec = M.SynthSpec(seed=41, n_genomes=10, genome_len=1_000_000, arrays_per_genome=0, n_reads=150_000,
                       error_rate=0.01)
    packed, offs = M.synth_host(spec)
    reads = M.Reads.synth(gpu_ctx, spec)
    gk, gc = M.count_edges(gpu_ctx, reads, 27)
    ok, oc = O.count_canonical(packed, offs, 27, threads=4)
    assert np.array_equal(gk, ok) and np.array_equal(gc, oc)


@pytest.mark.parametrize("n_reads", [12, 400])
def test_poly_t_runs(gpu_ctx, n_reads):
    """Super-k-mers starting inside a run of >= 32 T have an all-ones first word, the LDS
    descriptor table's empty marker: up to 64 per partition are deferred and expanded with
    weight 1, more send the partition down the raw path. Counts must equal the oracle."""
    rng = np.random.default_rng(n_reads)
    seqs = []
    for i in range(n_reads):
        flank = "".join(rng.choice(list("ACGT"), size=70))
        seqs.append(flank[:30] + "T" * (60 + (i * 7) % 90) + flank[30:])
    packed, offs = pack_reads(seqs)
    reads = M.Reads.from_host(gpu_ctx, packed, offs)
    for k in (23, 27):
        gk, gc = M.count_edges(gpu_ctx, reads, k)
        ok, oc = O.count_canonical(packed, offs, k)
        assert np.array_equal(gk, ok) and np.array_equal(gc, oc), k


def test_mixed_read_lengths(gpu_ctx):
    """Variable-length reads, longer than one 128-position work item (items split reads)."""
    rng = np.random.default_rng(4)
    genome = "".join(rng.choice(list("ACGT"), size=20_000))
    seqs = []
    for i in range(3000):
        L = int(rng.integers(20, 700))
        a = int(rng.integers(0, len(genome) - L))
        seqs.append(genome[a:a + L])
    packed, offs = pack_reads(seqs)
    reads = M.Reads.from_host(gpu_ctx, packed, offs)
    for k in (15, 23, 30):
        gk, gc = M.count_edges(gpu_ctx, reads, k)
        ok, oc = O.count_canonical(packed, offs, k)
        assert np.array_equal(gk, ok) and np.array_equal(gc, oc), k


@pytest.mark.parametrize("glen", [400, 6000])
def test_long_peel_chains(gpu_ctx, glen):
    """Reads tiling a linear genome end to end (both strands, >= 2x at the ends): the seed tips
    survive the multiplicity filter and the reduction peels back along the whole genome; 6000
    bases exceed the frontier level cap and exercise the ruler/list-ranking fallback."""
    rng = np.random.default_rng(glen)
    genome = "".join(rng.choice(list("ACGT"), size=glen))
    from tests.helpers import rc

    seqs = []
    for i in range(0, glen - 100 + 1):
        seqs += [genome[i:i + 100], rc(genome[i:i + 100])]
    packed, offs = pack_reads(seqs)
    reads = M.Reads.from_host(gpu_ctx, packed, offs)
    g = M.Graph.build(gpu_ctx, reads, 23)
    res = g.cycle_finder(M.CfParams(threshold_multiplicity=2))
    og = O.OGraph.build(packed, offs, 23)
    ores = og.cycle_finder(threshold_multiplicity=2)
    assert res.stats[:6] == ores["stats"]
    _, _, valid = g.download()
    assert np.array_equal(valid, og.valid())
    assert ores["stats"][2] < og.size // 2  # most of the genome was peeled


def test_cycle_results_as_arrays(gpu_ctx):
    """The bench's array form of the results holds exactly the list form's cycles."""
    reads = M.Reads.synth(gpu_ctx, M.SynthSpec())
    a = M.Graph.build(gpu_ctx, reads, 23).cycle_finder(M.CfParams())
    b = M.Graph.build(gpu_ctx, reads, 23).cycle_finder(M.CfParams(), as_arrays=True)
    assert len(a.entries) == len(b.entries) and a.stats == b.stats
    for (s1, cyc), (s2, (flat, offs)) in zip(a.entries, b.entries):
        assert s1 == s2
        assert cyc == [flat[offs[j]:offs[j + 1]].tolist() for j in range(len(offs) - 1)]
    assert list(b.candidates) == a.candidates and list(b.buckets) == a.buckets


def test_graph_from_sorted_rejects_bad_keys(gpu_ctx):
    """mcaat_graph_from_sorted takes sorted unique BOSS keys below 4^(k+1). The directory pass
    checks both and a violation is MCAAT_E_INVALID, not a silently wrong directory (the round-3
    clamp in k_dir kept out-of-range prefixes from writing past it, but built a wrong graph)."""
    from tests.helpers import HipBuffer

    spec = M.SynthSpec()
    k = 23
    reads = M.Reads.synth(gpu_ctx, spec)
    keys, mult, _ = M.Graph.build(gpu_ctx, reads, k).download()

    def build(kk):
        tk, tm = HipBuffer(kk), HipBuffer(mult)
        return M.Graph.from_sorted(gpu_ctx, k, tk.addr, tm.addr, int(kk.size))

    g = build(keys)  # the good keys build the same graph
    k2, m2, _ = g.download()
    assert np.array_equal(k2, keys) and np.array_equal(m2, mult)
    bad = keys.copy()
    bad[bad.size // 2] = np.uint64(1) << np.uint64(2 * (k + 1))  # past 4^(k+1) (then also unsorted)
    bad[-1] = np.uint64((1 << (2 * (k + 1))) + 5)
    with pytest.raises(M.McaatError) as ei:
        build(bad)
    assert ei.value.code == -1
    # in range, out of order / repeated: inside a 64-edge row, across rows, across 256-edge chunks
    for a in (100, 63, 255):
        swapped = keys.copy()
        swapped[[a, a + 1]] = swapped[[a + 1, a]]
        with pytest.raises(M.McaatError) as ei:
            build(swapped)
        assert ei.value.code == -1
        dup = keys.copy()
        dup[a + 1] = dup[a]
        with pytest.raises(M.McaatError) as ei:
            build(dup)
        assert ei.value.code == -1


@pytest.mark.parametrize("frac,compact", [(0.02, 0), (0.3, 0), (0.02, 1), (0.3, 1)])
def test_cycle_finder_on_a_graph_with_invalid_edges(gpu_ctx, frac, compact):
    """CycleFinder on a graph whose valid bits were cleared before it runs (the host's
    SetInvalidEdge): the tips pass then reads the unfiltered bitmap (not every edge is valid), and
    the peel's compact slots cover only the edges valid after the filter. Stats, the valid bitmap
    afterwards and the results equal the oracle run on the same bits."""
    spec, k, prm = CONFIGS["pe_err"]
    packed, offs = M.synth_host(spec)
    reads = M.Reads.synth(gpu_ctx, spec)
    g = M.Graph.build(gpu_ctx, reads, k)
    og = _oracle_graph(packed, offs, k)
    rng = np.random.default_rng(int(frac * 100))
    drop = np.sort(rng.choice(g.size, size=int(frac * g.size), replace=False)).astype(np.uint64)
    g.set_valid(drop, False)
    v = og.valid().astype(np.uint8)
    v[drop.astype(np.int64)] = 0
    og.set_valid(v)
    with gpu_ctx.knobs(cf__compact=compact):
        res = g.cycle_finder(prm)
    ores = og.cycle_finder(threshold_multiplicity=prm.threshold_multiplicity, low_abundance=prm.low_abundance,
                           cycle_max_length=prm.cycle_max_length, cycle_min_length=prm.cycle_min_length, threads=1)
    assert res.stats[:6] == ores["stats"]
    assert res.candidates == ores["candidates"] and res.buckets == ores["buckets"]
    _, _, valid = g.download()
    assert np.array_equal(valid, og.valid())
    assert [(s, c) for s, c in res.entries] == [tuple(e) for e in ores["entries"]]


@pytest.mark.parametrize("hops", [0, 1, 5, 40])
def test_keep_region_equals_host_growth(gpu_ctx, hops):
    """mcaat_graph_keep_region (step 7's keep_crispr_regions_extended_by_k on the device) equals the
    host growth: seeds grown `hops` rounds over valid in/out neighbours of valid frontier nodes,
    then valid &= region."""
    spec, k, prm = CONFIGS["pe_err"]
    reads = M.Reads.synth(gpu_ctx, spec)
    g = M.Graph.build(gpu_ctx, reads, k)
    rng = np.random.default_rng(hops)
    # some invalid edges first, and seeds both valid and invalid
    g.set_valid(np.sort(rng.choice(g.size, size=g.size // 10, replace=False)).astype(np.uint64), False)
    _, _, v0 = g.download()
    seeds = rng.choice(g.size, size=200, replace=False).astype(np.uint64)
    region = set(int(x) for x in seeds)
    frontier = list(region)
    for _ in range(hops):
        expand = np.array([e for e in frontier if v0[e]], dtype=np.uint64)
        nxt = []
        if expand.size:
            for inc in (False, True):
                nb, cnt = g.neighbors(expand, incoming=inc)
                for i in range(expand.size):
                    for j in range(cnt[i]):
                        x = int(nb[i, j])
                        if x not in region:
                            region.add(x)
                            nxt.append(x)
        frontier = nxt
    want = v0.copy()
    keep = np.zeros_like(want)
    keep[np.array(sorted(region), dtype=np.int64)] = 1
    want &= keep.astype(want.dtype)
    g.keep_region(seeds, hops)
    _, _, v1 = g.download()
    assert np.array_equal(v1.astype(bool), want.astype(bool))


def test_valid_subgraph_equals_neighbors(gpu_ctx):
    """mcaat_graph_valid_subgraph (step 7's SCC input) lists the valid edges ascending and, for each,
    its valid out-neighbours in OutgoingEdges order as positions in that list — the same sets
    mcaat_graph_neighbors gives edge by edge."""
    spec, k, prm = CONFIGS["pe_err"]
    reads = M.Reads.synth(gpu_ctx, spec)
    g = M.Graph.build(gpu_ctx, reads, k)
    rng = np.random.default_rng(7)
    g.set_valid(np.sort(rng.choice(g.size, size=g.size // 4, replace=False)).astype(np.uint64), False)
    _, _, v = g.download()
    ids, nbr, cnt = g.valid_subgraph()
    assert np.array_equal(ids, np.flatnonzero(v).astype(np.uint64))
    nb, c = g.neighbors(ids)
    assert np.array_equal(cnt.astype(np.int32), c)
    got = np.where(np.arange(4)[None, :] < cnt[:, None], ids[np.minimum(nbr, ids.size - 1)], 0)
    want = np.where(np.arange(4)[None, :] < c[:, None], nb, 0)
    assert np.array_equal(got, want)


def test_sharded_build_blocks_two_owners_equal_one_gpu(gpu_ctx):
    """The C-ABI building blocks a host with its own collectives drives (include/mcaat_gpu.h,
    "multi-GPU build"): two read halves counted apart (mcaat_count_local), owner ranges of the
    BOSS key from the summed histogram, each half's pairs grouped by owner
    (mcaat_counts_partition), the 'exchange' done here through host copies, each owner's pairs
    sorted and summed (mcaat_edges_reduce), and the owners' ranges in owner order built into a
    graph (mcaat_graph_from_sorted): the single-GPU keys and multiplicities."""
    from tests.helpers import HipBuffer

    spec, k, prm = CONFIGS["pe_err"]
    want_k, want_m, _ = M.Graph.build(gpu_ctx, M.Reads.synth(gpu_ctx, spec), k).download()
    half = spec.n_reads // 2
    parts = [M.Reads.synth_range(gpu_ctx, spec, 0, half), M.Reads.synth_range(gpu_ctx, spec, half, spec.n_reads - half)]
    counts = [M.Counts.count(gpu_ctx, r, k) for r in parts]
    bits = 10
    hist = sum(c.histogram(bits).astype(np.int64) for c in counts)
    cut = int(np.searchsorted(np.cumsum(hist), hist.sum() // 2))  # bins below go to owner 0
    assert 0 < cut < (1 << bits)
    splits = np.array([cut << (2 * (k + 1) - bits)], dtype=np.uint64)
    sent = []  # per source rank: its owner-major keys and counts, and the owners' sizes
    for c in counts:
        cap = 2 * c.n + 1
        kd, cd = HipBuffer(np.zeros(cap, np.uint64)), HipBuffer(np.zeros(cap, np.uint32))
        sizes = c.partition(splits, kd.addr, cd.addr, cap).astype(np.int64)
        n = int(sizes.sum())
        sent.append((kd.to_numpy(np.uint64, n), cd.to_numpy(np.uint32, n), sizes))
    got_k, got_m = [], []
    for o in range(2):
        ks = np.concatenate([kk[sz[:o].sum():sz[:o + 1].sum()] for kk, _, sz in sent])
        cs = np.concatenate([cc[sz[:o].sum():sz[:o + 1].sum()] for _, cc, sz in sent])
        kb, cb = HipBuffer(ks), HipBuffer(cs)
        ko, mo = HipBuffer(np.zeros(max(1, ks.size), np.uint64)), HipBuffer(np.zeros(max(1, ks.size), np.uint16))
        n = M.edges_reduce(gpu_ctx, k, kb.addr, cb.addr, ks.size, ko.addr, mo.addr)
        got_k.append(ko.to_numpy(np.uint64, n))
        got_m.append(mo.to_numpy(np.uint16, n))
    keys, mult = np.concatenate(got_k), np.concatenate(got_m)
    assert np.all(got_k[0][-1:] < splits[0]) and np.all(got_k[1][:1] >= splits[0])
    kb, mb = HipBuffer(keys), HipBuffer(mult)
    g = M.Graph.from_sorted(gpu_ctx, k, kb.addr, mb.addr, keys.size)
    gk, gm, _ = g.download()
    assert np.array_equal(gk, want_k) and np.array_equal(gm, want_m)
    for c in counts:
        c.free()


def test_arena_reuse_is_stream_ordered(gpu_ctx):
    """(round 5) A block freed while a slow kernel queued on the main stream
    still writes it is taken for a kernel on the side stream: the side stream waits for the
    free's fence, so the side kernel's writes are the ones left (csrc/alloc.hip). (round 6, ADVICE
    r5) The same with a consumer stream the arena does not watch: the block is taken with no
    allocation stream, so the host waits for the main stream's fence first."""
    same, kept, waits, same_f, kept_f = gpu_ctx.arena_check()
    assert same, "the side allocation did not get the freed block (the check tests nothing)"
    assert waits >= 1
    assert kept, "the side kernel ran before the main stream's queued writes to the same block"
    assert same_f, "the foreign-stream allocation did not get the freed block (the check tests nothing)"
    assert kept_f, "the unwatched stream wrote the block before the main stream's queued writes"
