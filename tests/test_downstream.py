"""Host steps after CycleFinder: spacer ordering, get_systems and
CRISPRAnalyzer -> CRISPR_Arrays.txt (libmcaat_host.so, include/mcaat_host.h).

CPU: the reference's own set-cover tests (tests/test_spacer_ordering.cpp), rapidfuzz's
published example scores plus a brute-force restatement on DNA strings, a hand-checked
CRISPRAnalyzer report, and the whole downstream on the oracle's graph/cycles/reads with a
known answer (every reported spacer is a spacer of the synthetic array; the repeat occurs
spacers+1 times). GPU: the mcaat CLI's CRISPR_Arrays.txt (GPU graph, CycleFinder and read
mapping) equals the one the same host code writes from the oracle's graph, cycles and reads.
Parity for cft (set cover) and rapidfuzz is unpinned: both are absent third-party code.
"""
import os
import random
import subprocess

import numpy as np
import pytest

import mcaat_amd as M
import oracle as O
from mcaat_amd import downstream as DS
from tests.helpers import unpack_read

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "mcaat_amd", "mcaat")


# ---- reference tests/test_spacer_ordering.cpp (SolveMinCoverProblemTest.*) ----------------
def _covers(universe, sets, res):
    got = set()
    for i in res:
        got |= set(sets[i])
    return got == set(universe)


def test_min_cover_reference_cases():
    assert DS.min_cover([], [[0, 1], [2, 3]]) == []                      # EmptyUniverse
    assert DS.min_cover([0, 1, 2, 3], []) == []                          # EmptySets
    assert DS.min_cover([0, 1, 2], [[0, 1], [3, 4]]) == []               # NoSolutionPossible
    assert DS.min_cover([0], [[0]]) == [0]                               # SingleElementSingleSet
    sets = [[0, 1, 2], [3, 4], [1, 3], [2, 4]]                           # SimpleOptimalSolution
    r = DS.min_cover(range(5), sets)
    assert 0 < len(r) <= 2 and _covers(range(5), sets, r)
    assert DS.min_cover(range(4), [[0, 1, 2, 3], [0, 1], [2], [3], [1, 2]]) == [0]  # RedundantSets
    sets = [[0, 1, 2, 3], [0, 2, 4, 5], [0, 3, 5, 6], [0, 1, 4], [0, 6]]  # ComplexOverlappingSets
    r = DS.min_cover(range(7), sets)
    assert r and all(i < len(sets) for i in r) and _covers(range(7), sets, r) and len(r) <= 3


def test_min_cover_is_minimum_on_random_instances():
    rng = random.Random(5)
    for _ in range(60):
        n = rng.randint(1, 12)
        sets = [rng.sample(range(n), rng.randint(1, n)) for _ in range(rng.randint(1, 9))]
        universe = sorted({x for s in sets for x in s})
        remap = {x: i for i, x in enumerate(universe)}
        sets = [[remap[x] for x in s] for s in sets]
        r = DS.min_cover(range(len(universe)), sets)
        assert _covers(range(len(universe)), sets, r)
        best = min(bin(m).count("1") for m in range(1, 1 << len(sets))
                   if _covers(range(len(universe)), sets, [i for i in range(len(sets)) if m >> i & 1]))
        assert len(r) == best


# ---- rapidfuzz fuzz.ratio / fuzz.partial_ratio ----------------------------------------------
def _lcs(a, b):
    row = [0] * (len(b) + 1)
    for x in a:
        diag = 0
        for j, y in enumerate(b):
            up = row[j + 1]
            row[j + 1] = diag + 1 if x == y else max(up, row[j])
            diag = up
    return row[-1]


def _ratio(a, b):
    s = len(a) + len(b)
    return 100.0 if s == 0 else (1.0 - (s - 2 * _lcs(a, b)) / s) * 100.0


def _partial(a, b):
    """every window of the longer string (prefixes, full windows, suffixes), both directions
    for equal lengths — the definition the restatement's skips must not change on DNA"""
    if len(a) > len(b):
        a, b = b, a
    if not a:
        return 100.0 if not b else 0.0
    n1, n2 = len(a), len(b)
    wins = [b[:i] for i in range(1, n1)] + [b[i:i + n1] for i in range(n2 - n1 + 1)] + [b[i:] for i in range(n2 - n1, n2)]
    r = max(_ratio(a, w) for w in wins)
    if n1 == n2 and r != 100.0:
        r = max(r, max(_ratio(b, w) for w in [a[:i] for i in range(1, n1)] + [a[i:] for i in range(n1)]))
    return r


def test_fuzz_published_examples():
    # rapidfuzz documentation examples
    assert DS.fuzz_ratio("this is a test", "this is a test!") == pytest.approx(96.55172413793103)
    assert DS.fuzz_partial_ratio("this is a test", "this is a test!") == 100.0
    assert DS.fuzz_ratio("fuzzy wuzzy was a bear", "wuzzy fuzzy was a bear") == pytest.approx(90.9090909090909)
    assert DS.fuzz_ratio("", "") == 100.0 and DS.fuzz_partial_ratio("", "") == 100.0
    assert DS.fuzz_partial_ratio("", "abc") == 0.0


def test_fuzz_matches_brute_force_on_dna():
    rng = random.Random(11)
    for _ in range(300):
        a = "".join(rng.choice("ACGT") for _ in range(rng.randint(23, 50)))
        b = "".join(rng.choice("ACGT") for _ in range(rng.randint(23, 50)))
        if rng.random() < 0.3:  # near-substrings, as spacer duplicates are
            i = rng.randint(0, len(a) - 10)
            b = a[i:i + rng.randint(10, len(a) - i)] + b[: rng.randint(0, 5)]
        assert DS.fuzz_ratio(a, b) == _ratio(a, b)
        assert DS.fuzz_partial_ratio(a, b) == _partial(a, b)
    # the bit-parallel LCS takes either string of <= 64 symbols as the pattern; both longer: DP
    for la, lb in ((64, 100), (65, 64), (100, 130), (1, 64), (64, 64)):
        a = "".join(rng.choice("ACGT") for _ in range(la))
        b = "".join(rng.choice("ACGT") for _ in range(lb))
        assert DS.fuzz_ratio(a, b) == _ratio(a, b)
        assert DS.fuzz_ratio(b, a) == _ratio(b, a)


# ---- CRISPRAnalyzer ----------------------------------------------------------------------
HEADER = ("CRISPR Analysis Report\nThe tool was run with the following parameters:\nAmount of Spacers: 2\n"
          "[Min:Max] Length of Spacers: [23:50]\n[Min:Max] Length of Repeats: [23:50]\n"
          "Mean Similarity Between Spacers: 90\nConservation Threshold: 80%\n" + "-" * 50 + "\n")


def test_crispr_analyzer_report(tmp_path):
    rng = random.Random(3)
    repeat = "GTTTTAGAGCTATGCTGTTTTGAATGGTCC"  # 30 bp
    firsts = "ACGTACGTAC"
    spacers = [firsts[i] + "".join(rng.choice("ACGT") for _ in range(31)) for i in range(10)]
    spacers[-1] = spacers[-1][:-1] + "A"
    out = tmp_path / "CRISPR_Arrays.txt"
    DS.crispr_analyzer([(repeat, spacers), ("ACGTACGTACGTACGTACGTACGTA", spacers[:1]),
                        ("C" * 60, spacers[:5])], str(out))
    txt = out.read_text()
    assert txt.startswith(HEADER)
    body = txt[len(HEADER):].split("\n")
    assert body[0] == "-" * 50 and body[1] == repeat and body[2] == "-" * 50
    listed = body[3:3 + len(spacers)]
    assert sorted(listed) == sorted(spacers)
    assert body[3 + len(spacers)] == "-" * 50
    assert body[4 + len(spacers)] == f"Number of Spacers: {len(spacers)}"
    # one system reported, the single-spacer one and the 60-bp repeat omitted
    assert txt.endswith(f"Number of Systems: 1\nNumber of Spacers: {len(spacers)}\nOmitted Repeats: 2\n")


# ---- whole downstream on the oracle path -----------------------------------------------------
def _oracle_downstream(spec, k, out_file, prm=None):
    packed, offs = M.synth_host(spec)
    og = O.OGraph.build(packed, offs, k, threads=4)
    res = og.cycle_finder(**(prm or {}))
    ent = res["entries"]
    cycles = [c for i in res["map_order"] for c in ent[i][1]]  # cycles_map_to_cycles order
    nodes = sorted({x for c in cycles for x in c})
    seqs = [unpack_read(packed, int(offs[i]), int(offs[i + 1])) for i in range(len(offs) - 1)]
    reads = og.get_reads(seqs, len(seqs), nodes)
    keys, mult = og.arrays()
    valid = og.valid().astype(np.uint8).copy()
    n = DS.crispr_arrays(k, keys, mult, valid, cycles, reads, str(out_file))
    return n, seqs


def _report_systems(txt):
    lines = txt.split("\n")
    systems, i = [], 0
    rule = "-" * 50
    while i < len(lines):
        if lines[i] == rule and i + 2 < len(lines) and lines[i + 2] == rule and lines[i + 1] and \
                not lines[i + 1].startswith("Number"):
            rep = lines[i + 1]
            j = i + 3
            sp = []
            while lines[j] != rule:
                sp.append(lines[j])
                j += 1
            systems.append((rep, sp))
            i = j + 1
        else:
            i += 1
    return systems


@pytest.mark.parametrize("k", [23, 27])
def test_downstream_known_answer_c1(tmp_path, k):
    spec = M.SynthSpec()  # one array: repeat 30 bp, 12 spacers of 32 bp
    out = tmp_path / "CRISPR_Arrays.txt"
    n, _ = _oracle_downstream(spec, k, out)
    genome = unpack_read(M.synth_genome_host(spec), 0, spec.genome_len)
    rcg = genome[::-1].translate(str.maketrans("ACGT", "TGCA"))
    systems = _report_systems(out.read_text())
    assert n == 2 and len(systems) == 2  # the array and its reverse complement
    for rep, sp in systems:
        assert len(sp) == 12 and all(len(s) == 32 for s in sp)
        assert all(s in genome or s in rcg for s in sp)
        assert genome.count(rep) + rcg.count(rep) == 13
    assert out.read_text().endswith("Number of Systems: 2\nNumber of Spacers: 24\nOmitted Repeats: 0\n")


def test_downstream_several_arrays_with_errors(tmp_path):
    spec = M.SynthSpec(seed=21, n_genomes=3, genome_len=20_000, arrays_per_genome=1, spacers_per_array=9,
                       repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36, n_reads=15_000,
                       error_rate=0.001)
    out = tmp_path / "CRISPR_Arrays.txt"
    _oracle_downstream(spec, 23, out, dict(threshold_multiplicity=5))
    genome = unpack_read(M.synth_genome_host(spec), 0, spec.n_genomes * spec.genome_len)
    rcg = genome[::-1].translate(str.maketrans("ACGT", "TGCA"))
    systems = _report_systems(out.read_text())
    assert len(systems) >= 3
    total = sum(len(sp) for _, sp in systems)
    found = sum(1 for _, sp in systems for s in sp if s in genome or s in rcg)
    assert found >= 0.9 * total


# ---- GPU: the CLI's CRISPR_Arrays.txt equals the oracle-driven one --------------------------
# gpus > 1: the CLI forks one rank per GPU; on the one-GPU box the ranks share it through the
# shared-memory transport (FASTQ parts, sharded build, CycleFinder over ranks, gathered reads)
@pytest.mark.gpu
@pytest.mark.parametrize("paired,gpus,ahead", [(False, 1, "1"), (True, 1, "1"), (False, 3, "1"), (True, 2, "1"),
                                               (True, 1, "0")])
def test_cli_crispr_arrays_match_oracle_path(tmp_path, paired, gpus, ahead):
    """(round 5) the single-GPU CLI counts while it reads (mcaat_count_ahead) unless
    MCAAT_COUNT_AHEAD=0; both give the oracle path's CRISPR_Arrays.txt."""
    spec = M.SynthSpec()
    packed, offs = M.synth_host(spec)
    seqs = [unpack_read(packed, int(offs[i]), int(offs[i + 1])) for i in range(len(offs) - 1)]
    files = []
    if paired:  # second file written reverse-complemented (the reference flips it back)
        halves = [seqs[0::2], [s[::-1].translate(str.maketrans("ACGT", "TGCA")) for s in seqs[1::2]]]
    else:
        halves = [seqs]
    for j, part in enumerate(halves):
        p = tmp_path / f"r{j + 1}.fq"
        with open(p, "w") as f:
            for i, s in enumerate(part):
                f.write(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")
        files.append(str(p))
    multi = ["--gpus", str(gpus), "--comm", "shm"] if gpus > 1 else []
    env = dict(os.environ, MCAAT_COUNT_AHEAD=ahead)
    out = subprocess.run([CLI, "-i", *files, "--output-folder", str(tmp_path / "o"), "--threads", "2", "--ram", "2G",
                          *multi], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr + out.stdout[-2000:]
    got = (tmp_path / "o" / "CRISPR_Arrays.txt").read_text()

    # oracle path over the same sequences in the reference's read order
    og = O.OGraph.build(packed, offs, 23, threads=4)
    res = og.cycle_finder()
    ent = res["entries"]
    cycles = [c for i in res["map_order"] for c in ent[i][1]]
    nodes = sorted({x for c in cycles for x in c})
    order = halves[0] + (halves[1] if paired else [])
    reads = og.get_reads(order, len(halves[0]), nodes)
    keys, mult = og.arrays()
    valid = og.valid().astype(np.uint8).copy()
    ref_file = tmp_path / "oracle_CRISPR_Arrays.txt"
    DS.crispr_arrays(23, keys, mult, valid, cycles, reads, str(ref_file))
    assert got == ref_file.read_text()
    assert "Number of Systems: 2" in got


@pytest.mark.gpu
@pytest.mark.parametrize("comm", ["shm", "rccl"])
def test_cli_rank_dying_before_it_joins_ends_the_run(tmp_path, comm):
    """A forked rank that exits before joining the communicator (device selection, OOM, ...)
    ends the run at once: rank 0 reaps its children from the fork on, so it does not wait in
    the join (ncclCommInitRank has no timeout; the shared-memory join waits 900 s). With one
    GPU on the box, rccl with 2 ranks stops at its own GPU-count check, also promptly."""
    import time

    spec = M.SynthSpec()
    packed, offs = M.synth_host(spec)
    p = tmp_path / "r.fq"
    with open(p, "w") as f:
        for i in range(len(offs) - 1):
            s = unpack_read(packed, int(offs[i]), int(offs[i + 1]))
            f.write(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")
    env = dict(os.environ, MCAAT_TEST_RANK_EXIT="1")
    t0 = time.time()
    out = subprocess.run([CLI, "-i", str(p), "--output-folder", str(tmp_path / "o"), "--threads", "2", "--gpus", "2",
                          "--comm", comm], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode != 0
    assert time.time() - t0 < 120, "the run waited for a rank that had already died"


@pytest.mark.gpu
def test_cli_step7_threads_equal_serial_on_a_device_graph(tmp_path):
    """ The CLI's device-graph path (GPU region growth and valid subgraph, then
    the regions solved on the job's threads) with --threads 1 and --threads 8 on a multi-array
    input: the same CRISPR_Arrays.txt and the same step-7 log, line for line."""
    spec = M.SynthSpec(seed=21, n_genomes=3, genome_len=20_000, arrays_per_genome=2, spacers_per_array=9,
                       repeat_len_min=30, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36, n_reads=24_000,
                       error_rate=0.001)
    packed, offs = M.synth_host(spec)
    p = tmp_path / "r.fq"
    with open(p, "w") as f:
        for i in range(len(offs) - 1):
            s = unpack_read(packed, int(offs[i]), int(offs[i + 1]))
            f.write(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")
    got = {}
    for t in (1, 8):
        o = tmp_path / f"o{t}"
        out = subprocess.run([CLI, "-i", str(p), "--output-folder", str(o), "--threads", str(t), "--ram", "2G"],
                             capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr + out.stdout[-2000:]
        lines = out.stdout.splitlines()
        a = next(i for i, x in enumerate(lines) if "Filtered out" in x)
        b = next(i for i, x in enumerate(lines) if "Completed each subproblem" in x)
        got[t] = ((o / "CRISPR_Arrays.txt").read_text(), lines[a:b + 1])
    assert got[1][0] == got[8][0]
    assert got[1][1] == got[8][1]
    assert "Number of Systems:" in got[1][0] and got[1][1][0].split()[-1] != "0/0"
