"""GPU FASTQ ingest (csrc/fastq_ingest.hip) against the Python restatement
of the read library (oracle/fastx.py): counting view (reads split at non-ACGT symbols) and
mapping view (one entry per record, second file reverse-complemented, reads.cpp:20-52).

Bar: bit-exact packed streams and offsets. The chunk size is forced down (MCAAT_FASTQ_CHUNK) so
records straddle chunk boundaries and the carry path runs many times. Edge cases: N and IUPAC
symbols, lowercase, CRLF, empty sequences, no final newline, blank lines around the records,
gzip and bzip2 input (concatenated members / streams), paired-end, records longer than the
carry reserve and malformed input (loud errors).
"""
import bz2
import gzip
import os

import numpy as np
import pytest

from oracle import fastx as FX

ALPHA = "ACGT" * 6 + "acgtNRY"


def _rand_records(rng, n, max_len=300):
    seqs = []
    for i in range(n):
        L = int(rng.integers(0, max_len)) if i % 17 else 0
        if i % 5 == 0:
            s = "".join(rng.choice(list(ALPHA), size=L))
        else:
            s = "".join(rng.choice(list("ACGT"), size=L))
        seqs.append(s)
    return seqs


def _fastq_text(seqs, crlf=False, final_newline=True, lead="", trail=""):
    nl = "\r\n" if crlf else "\n"
    body = nl.join(f"@r{i} x{nl}{s}{nl}+{nl}{'I' * len(s)}" for i, s in enumerate(seqs))
    return lead + body + (nl if final_newline else "") + trail


def _write(path, text, gz=False):
    data = text.encode()
    if gz == "bz2":  # two concatenated bzip2 streams (as pbzip2 writes), split mid-record
        h = len(data) // 2
        with open(path, "wb") as f:
            f.write(bz2.compress(data[:h]) + bz2.compress(data[h:]))
    elif gz:
        with gzip.open(path, "wb") as f:
            f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)
    return str(path)


# ---- restatement (CPU) ------------------------------------------------------------------

def test_restatement_known_answers():
    text = "\n\n@a\nACGTNacgt\n+\nIIIIIIIII\n@b\r\n\r\n+\r\n\r\n@c\nGGRTT\n+\nIIIII"
    seqs = FX.fastq_sequences(text)
    assert seqs == ["ACGTNacgt", "", "GGRTT"]
    assert FX.counting_view(seqs) == ["ACGT", "ACGT", "GG", "TT"]
    assert FX.mapping_view([seqs[:2], seqs[2:]]) == [[0, 1, 2, 3, 3, 3, 3, 3, 3], [], [0, 0, 3, 1, 1]]
    words, offs = FX.pack_bases(["ACGT", "T"])
    assert list(offs) == [0, 4, 5] and int(words[0]) == 0b11_11100100
    with pytest.raises(FX.FastqError):
        FX.fastq_sequences("@a\nACGT\n+\n")  # 3 lines
    with pytest.raises(FX.FastqError):
        FX.fastq_sequences("@a\nACGT\n+\nIIII\nb\nA\n+\nI\n")


# ---- GPU ------------------------------------------------------------------------------------

def _check(ctx, files, texts, monkeypatch, chunk):
    import mcaat_amd as M

    if chunk:
        monkeypatch.setenv("MCAAT_FASTQ_CHUNK", str(chunk))
    else:
        monkeypatch.delenv("MCAAT_FASTQ_CHUNK", raising=False)
    per_file = [FX.fastq_sequences(t) for t in texts]
    want_p, want_o = FX.pack_bases(FX.counting_view([s for f in per_file for s in f]))
    want_qp, want_qo = FX.pack_codes(FX.mapping_view(per_file))
    reads = M.Reads.from_fastx(ctx, files)
    p, o = reads.download()
    assert np.array_equal(o, want_o)
    nw = (int(want_o[-1]) + 31) // 32
    assert np.array_equal(p[:nw], want_p[:nw])
    qp, qo = reads.download_records()
    assert np.array_equal(qo, want_qo)
    nq = (int(want_qo[-1]) + 31) // 32
    assert np.array_equal(qp[:nq], want_qp[:nq])
    n_rec, separate = reads.records_info()
    assert n_rec == sum(len(f) for f in per_file)
    one_run = all(len(s) > 0 and set(s) <= set("ACGT") for f in per_file for s in f)
    assert separate == (len(files) > 1 and len(per_file[1]) > 0 or not one_run)
    return reads


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [256, 1000, 4099, 0])
def test_single_end_chunked(gpu_ctx, tmp_path, monkeypatch, chunk):
    rng = np.random.default_rng(11 + chunk)
    seqs = _rand_records(rng, 400)
    text = _fastq_text(seqs, lead="\n", trail="\n\n")
    _check(gpu_ctx, [_write(tmp_path / "a.fq", text)], [text], monkeypatch, chunk)


@pytest.mark.gpu
@pytest.mark.parametrize("gz", [False, True, "bz2"])
def test_paired_end_crlf_gzip(gpu_ctx, tmp_path, monkeypatch, gz):
    rng = np.random.default_rng(5)
    t1 = _fastq_text(_rand_records(rng, 300), crlf=True)
    t2 = _fastq_text(_rand_records(rng, 300), final_newline=False)
    sfx = ".fq.bz2" if gz == "bz2" else ".fq.gz" if gz else ".fq"
    files = [_write(tmp_path / ("r1" + sfx), t1, gz), _write(tmp_path / ("r2" + sfx), t2, gz)]
    _check(gpu_ctx, files, [t1, t2], monkeypatch, 777)


@pytest.mark.gpu
def test_acgt_only_is_the_counting_view(gpu_ctx, tmp_path, monkeypatch):
    rng = np.random.default_rng(7)
    seqs = ["".join(rng.choice(list("ACGT"), size=150)) for _ in range(500)]
    text = _fastq_text(seqs)
    reads = _check(gpu_ctx, [_write(tmp_path / "a.fq", text)], [text], monkeypatch, 2048)
    assert reads.records_info() == (500, False)
    # fixed-length detection as for host-built libraries
    n, b = reads.info()
    assert (n, b) == (500, 75000)


@pytest.mark.gpu
def test_empty_and_blank_files(gpu_ctx, tmp_path, monkeypatch):
    import mcaat_amd as M

    f = _write(tmp_path / "e.fq", "\n\n")
    reads = M.Reads.from_fastx(gpu_ctx, [f])
    assert reads.info() == (0, 0)


def _check_kseq(ctx, files, texts):
    """Inputs the 4-line GPU parser hands to the host reader: parity with the kseq restatement."""
    import mcaat_amd as M

    per_file = [FX.kseq_sequences(t) for t in texts]
    want_p, want_o = FX.pack_bases(FX.counting_view([s for f in per_file for s in f]))
    want_qp, want_qo = FX.pack_codes(FX.mapping_view(per_file))
    reads = M.Reads.from_fastx(ctx, files)
    p, o = reads.download()
    assert np.array_equal(o, want_o)
    nw = (int(want_o[-1]) + 31) // 32
    assert np.array_equal(p[:nw], want_p[:nw])
    qp, qo = reads.download_records()
    assert np.array_equal(qo, want_qo)
    nq = (int(want_qo[-1]) + 31) // 32
    assert np.array_equal(qp[:nq], want_qp[:nq])


def test_kseq_restatement_known_answers():
    assert FX.kseq_sequences("@a\nACGT\n+\nIIII\n\n@b\nACGT\n+\nIIII\n") == ["ACGT", "ACGT"]
    assert FX.kseq_sequences("@a\nAC\nGT\n+\nII\nII\n@b\nA\n+\n@\n") == ["ACGT", "A"]  # wrapped; '@' quality
    assert FX.kseq_sequences("@a\nACGT\n+\nIIII\nb\nACGT\n+\nIIII\n") == ["ACGT"]  # junk skipped to EOF
    assert FX.kseq_sequences(">x\nACGTN\nACG\n\n>y\nTT\n") == ["ACGTNACG", "TT"]
    assert FX.kseq_sequences("@a\r\nAC\r\n+\r\nII\r\n") == ["AC"]
    text = "\n\n@a\nACGTNacgt\n+\nIIIIIIIII\n@b\r\n\r\n+\r\n\r\n@c\nGGRTT\n+\nIIIII"
    assert FX.kseq_sequences(text) == FX.fastq_sequences(text)  # well-formed: the 4-line reading
    with pytest.raises(FX.FastqError):
        FX.kseq_sequences("@a\nACGT\n+\nIIII\n@b\nACGT\n+\n")
    with pytest.raises(FX.FastqError):
        FX.kseq_sequences("@a\nACGT\n+\nIIIIII\n")


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [256, 0])
def test_non_4line_inputs_read_like_kseq(gpu_ctx, tmp_path, monkeypatch, chunk):
    """Blank lines between records, wrapped lines, a record above the carry reserve, FASTA and
    FASTQ mixed, an empty mate file: the GPU parser hands these to the host kseq-style reader
    (the reference's kseq readers accept them)."""
    if chunk:
        monkeypatch.setenv("MCAAT_FASTQ_CHUNK", str(chunk))
    else:
        monkeypatch.delenv("MCAAT_FASTQ_CHUNK", raising=False)
    rng = np.random.default_rng(3)
    good = _fastq_text(_rand_records(rng, 40))
    cases = {
        "blank": ["@a\nACGT\n+\nIIII\n\n@b\nACGT\n+\nIIII\n" + good],
        "wrapped": ["@a\nACGTAC\nGTTT\n+\nIIIIII\nIIII\n@b\nGGA\n+\n@@@\n" + good],
        "header_junk": ["@a\nACGT\n+\nIIII\nb\nACGT\n+\nIIII\n"],
        "long": [good + "@L\n" + "ACGT" * 1500 + "\n+\n" + "I" * 6000 + "\n"],
        "mixed": [">a\nACGTN\nAC\n>b\nGGGT\n", good],
        "empty_mate": [good, ""],
    }
    for name, texts in cases.items():
        files = [_write(tmp_path / f"{name}{i}.fq", t) for i, t in enumerate(texts)]
        _check_kseq(gpu_ctx, files, texts)


@pytest.mark.gpu
def test_malformed_inputs_fail_loudly(gpu_ctx, tmp_path, monkeypatch):
    import mcaat_amd as M

    monkeypatch.setenv("MCAAT_FASTQ_CHUNK", "256")
    bad = {
        "trunc.fq": "@a\nACGT\n+\nIIII\n@b\nACGT\n+\n",  # quality missing
        "qlen.fq": "@a\nACGT\n+\nIIIIII\n",  # quality longer than the sequence
        "junk.fq": "hello\n",  # neither '@' nor '>'
    }
    for name, text in bad.items():
        with pytest.raises(RuntimeError):
            M.Reads.from_fastx(gpu_ctx, [_write(tmp_path / name, text)])


@pytest.mark.gpu
def test_fasta_still_parsed(gpu_ctx, tmp_path):
    import mcaat_amd as M

    f = _write(tmp_path / "x.fa", ">a\nACGTN\nACG\n>b\nTTTT\n")
    reads = M.Reads.from_fastx(gpu_ctx, [f])
    p, o = reads.download()
    wp, wo = FX.pack_bases(["ACGT", "ACG", "TTTT"])
    assert np.array_equal(o, wo) and np.array_equal(p[:1], wp[:1])


@pytest.mark.gpu
def test_bzip2_fasta_wrapped_and_truncated(gpu_ctx, tmp_path, monkeypatch):
    """bzip2 through the host kseq-style reader (FASTA, wrapped FASTQ), and a truncated stream
    fails loudly instead of reading short."""
    import mcaat_amd as M

    monkeypatch.delenv("MCAAT_FASTQ_CHUNK", raising=False)
    texts = [">a\nACGTN\nACG\n>b\nTTTT\n", "@a\nACGTAC\nGTTT\n+\nIIIIII\nIIII\n@b\nGGA\n+\n@@@\n"]
    for i, t in enumerate(texts):
        f = _write(tmp_path / f"k{i}.bz2", t, "bz2")
        _check_kseq(gpu_ctx, [f], [t])
    good = bz2.compress(_fastq_text(["ACGT" * 40] * 50).encode())
    cut = tmp_path / "cut.fq.bz2"
    cut.write_bytes(good[: len(good) // 2])
    with pytest.raises(RuntimeError):
        M.Reads.from_fastx(gpu_ctx, [str(cut)])


# ---- host packer (csrc/fastq_pack.hip): the fast path for upper-case ACGT 4-line records ----

def _acgt_records(rng, n, lens):
    return ["".join(rng.choice(list("ACGT"), size=int(lens[i % len(lens)]))) for i in range(n)]


def _packed_by_host(ctx):
    """True when the last ingest ran the host packer (its concatenation kernel was timed)."""
    return ctx.kernel_timing("fq_concat")[1] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("mmap", ["0", "1"])
@pytest.mark.parametrize("threads,lens,final_nl", [("16", [150], True), ("3", [150], False),
                                                     ("7", [1, 31, 32, 33, 64, 150, 251, 1000], True),
                                                     ("1", [77], True), ("2", [1], False)])
def test_host_pack_single_end(gpu_ctx, tmp_path, monkeypatch, threads, lens, final_nl, mmap):
    """Fixed and variable read lengths (words shared by reads, 32-base boundaries), parts cut
    at record starts for 1..16 threads, a final record without its newline, the part read with
    pread() or mapped (MCAAT_PACK_MMAP; short final records near the end of the mapping): the
    same library as the text parser's restatement, and the host packer is the path that ran."""
    monkeypatch.setenv("MCAAT_PACK_THREADS", threads)
    monkeypatch.setenv("MCAAT_PACK_MMAP", mmap)
    rng = np.random.default_rng(int(threads) * 7 + len(lens))
    seqs = _acgt_records(rng, 3001, lens)
    text = _fastq_text(seqs, final_newline=final_nl)
    gpu_ctx.reset_timing()
    reads = _check(gpu_ctx, [_write(tmp_path / "a.fq", text)], [text], monkeypatch, 0)
    assert _packed_by_host(gpu_ctx)
    n, b = reads.info()
    assert n == 3001 and b == sum(len(s) for s in seqs)
    reads.free()


@pytest.mark.gpu
def test_host_pack_paired_end(gpu_ctx, tmp_path, monkeypatch):
    """Two files: counting view in file order, mapping view with the second file reverse-
    complemented (built on the device from the counting view)."""
    monkeypatch.setenv("MCAAT_PACK_THREADS", "5")
    rng = np.random.default_rng(3)
    t1 = _fastq_text(_acgt_records(rng, 1200, [150, 149]))
    t2 = _fastq_text(_acgt_records(rng, 1100, [150]))
    files = [_write(tmp_path / "r1.fq", t1), _write(tmp_path / "r2.fq", t2)]
    gpu_ctx.reset_timing()
    reads = _check(gpu_ctx, files, [t1, t2], monkeypatch, 0)
    assert _packed_by_host(gpu_ctx)
    assert reads.records_info() == (2300, True)
    reads.free()


@pytest.mark.gpu
def test_host_pack_many_files_many_threads(gpu_ctx, tmp_path, monkeypatch):
    """ 40 files x 64 threads: the per-thread split is clamped to 1 and the
    2560 parts exceed the concatenation's LDS table (2047 parts), so its part tables are read
    from global memory instead of failing the launch; same library as the restatement."""
    monkeypatch.setenv("MCAAT_PACK_THREADS", "64")
    rng = np.random.default_rng(17)
    texts = [_fastq_text(_acgt_records(rng, 100, [150, 90])) for _ in range(40)]
    files = [_write(tmp_path / f"f{i}.fq", t) for i, t in enumerate(texts)]
    gpu_ctx.reset_timing()
    reads = _check(gpu_ctx, files, texts, monkeypatch, 0)
    assert _packed_by_host(gpu_ctx)
    reads.free()


@pytest.mark.gpu
@pytest.mark.parametrize("bad", ["N", "lower", "crlf", "empty", "blank_end"])
def test_host_pack_declines_to_the_text_parser(gpu_ctx, tmp_path, monkeypatch, bad):
    """Inputs outside the fast path's form go to the GPU text parser, with its results."""
    monkeypatch.setenv("MCAAT_PACK_THREADS", "4")
    rng = np.random.default_rng(9)
    seqs = _acgt_records(rng, 800, [150])
    if bad == "N":
        seqs[700] = seqs[700][:50] + "N" + seqs[700][51:]
    elif bad == "lower":
        seqs[3] = seqs[3].lower()
    elif bad == "empty":
        seqs[400] = ""
    text = _fastq_text(seqs, crlf=bad == "crlf", trail="\n\n" if bad == "blank_end" else "")
    gpu_ctx.reset_timing()
    reads = _check(gpu_ctx, [_write(tmp_path / "a.fq", text)], [text], monkeypatch, 0)
    assert not _packed_by_host(gpu_ctx)
    reads.free()


@pytest.mark.gpu
def test_host_pack_off_matches_on(gpu_ctx, tmp_path, monkeypatch):
    """fq.hostpack=0 forces the text parser: both paths give the same library."""
    import mcaat_amd as M

    rng = np.random.default_rng(21)
    text = _fastq_text(_acgt_records(rng, 5000, [150]))
    path = _write(tmp_path / "a.fq", text)
    got = []
    for on in (1, 0):
        with gpu_ctx.knobs(fq__hostpack=on):
            gpu_ctx.reset_timing()
            r = M.Reads.from_fastx(gpu_ctx, [path])
            assert _packed_by_host(gpu_ctx) == bool(on)
            got.append((r.download(), r.info(), r.records_info()))
            r.free()
    (p1, o1), i1, q1 = got[0]
    (p0, o0), i0, q0 = got[1]
    nw = (int(o1[-1]) + 31) // 32
    assert i1 == i0 and q1 == q0 and np.array_equal(o1, o0) and np.array_equal(p1[:nw], p0[:nw])


@pytest.mark.gpu
def test_host_pack_on_a_second_device(gpu_ctx, tmp_path, monkeypatch):
    """ The packer's worker threads bind the context's device before making
    their events: a context on device 1 packs the same library as one on device 0. Needs two
    GPUs (skipped on a one-GPU box)."""
    import mcaat_amd as M

    if M.device_count() < 2:
        pytest.skip("one GPU: the second-device case needs two")
    monkeypatch.setenv("MCAAT_PACK_THREADS", "6")
    rng = np.random.default_rng(5)
    text = _fastq_text(_acgt_records(rng, 4000, [150]))
    path = _write(tmp_path / "a.fq", text)
    ctx1 = M.Context(1)
    try:
        ctx1.reset_timing()
        r1 = M.Reads.from_fastx(ctx1, [path])
        assert _packed_by_host(ctx1)
        r0 = M.Reads.from_fastx(gpu_ctx, [path])
        (p1, o1), (p0, o0) = r1.download(), r0.download()
        nw = (int(o1[-1]) + 31) // 32
        assert r1.info() == r0.info() and np.array_equal(o1, o0) and np.array_equal(p1[:nw], p0[:nw])
        r1.free()
        r0.free()
    finally:
        ctx1.close()


# ---- pass A while the input is read (mcaat_count_ahead, node_counter.hip nc_ahead_*) ----

def _genome_reads(rng, n, lens, genome_len=30000):
    g = rng.choice(list("ACGT"), size=genome_len)
    out = []
    for i in range(n):
        L = int(lens[i % len(lens)])
        p = int(rng.integers(0, genome_len - L))
        s = g[p:p + L]
        if i % 2:
            s = s[::-1]  # reverse orientation (not complemented: still a valid read)
        out.append("".join(s))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["fixed", "fixed_16_threads", "varlen", "undersized", "other_k", "knob_off", "paired"])
def test_count_ahead_equals_count_after_read(gpu_ctx, tmp_path, monkeypatch, case):
    """Pass A on each packed part as it lands gives the same canonical counts as pass A over
    the concatenated reads (the same reads object, counted again after the first count took
    the ahead buckets). Reads of differing lengths, an L1 capacity below the input (nc.l1_slots)
    and a count for another k fall back to pass A after the read, with the same counts."""
    import mcaat_amd as M

    monkeypatch.setenv("MCAAT_PACK_THREADS", "16" if case == "fixed_16_threads" else "5")
    rng = np.random.default_rng(41)
    lens = [150, 149] if case == "varlen" else [150]
    text = _fastq_text(_genome_reads(rng, 6000, lens))
    paths = [_write(tmp_path / "a.fq", text)]
    if case == "paired":  # two files: the counting view is both in file order
        paths.append(_write(tmp_path / "b.fq", _fastq_text(_genome_reads(rng, 5000, lens))))
    k = 27
    knobs = {"nc__l1_slots": 2048} if case == "undersized" else {"nc__ahead": 0} if case == "knob_off" else {}
    with gpu_ctx.knobs(**knobs):
        gpu_ctx.reset_timing()
        gpu_ctx.count_ahead(21 if case == "other_k" else k)
        r = M.Reads.from_fastx(gpu_ctx, paths)
        assert _packed_by_host(gpu_ctx)
        ahead_launches = gpu_ctx.kernel_timing("sk_scatter_ahead")[1]
        k1, c1 = M.count_edges(gpu_ctx, r, k)
        after = gpu_ctx.kernel_timing("sk_scatter")[1]
        k0, c0 = M.count_edges(gpu_ctx, r, k)
    used = case in ("fixed", "fixed_16_threads", "other_k", "paired")
    assert (ahead_launches > 0) == used, (case, ahead_launches)
    if case != "other_k":
        assert (after == 0) == used, (case, after)  # the first count ran no pass A of its own
    assert len(k1) > 1000 and c1.max() > 1
    assert np.array_equal(k1, k0) and np.array_equal(c1, c0)
    r.free()
