"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of the read library built from FASTQ.

Only tests/ may import this. It states what the GPU FASTQ parser (mcaat_amd/csrc/fastq_ingest.hip)
must produce, record by record:

* counting view (SDBGBuild::BuildLib, sdbg_build.cpp:82-115 → MEGAHIT buildlib, unpinned
  offline; conventions in DESIGN.md §2): every maximal run of A/C/G/T (either case) of a
  record's sequence is one read; other symbols split reads and are dropped.
* mapping view (get_reads, reads.cpp:88-130): one entry per record; records of every file
  after the first are reversed and complemented (reverse_pair_ends_sequence, reads.cpp:20-31,
  only A/C/G/T change), then coded as k_mer_to_node_id does (reads.cpp:44-52: 'A','C','G' →
  0,1,2 and every other character → 3).

FASTQ records are 4 lines; one trailing '\\r' per line is stripped; blank lines may only precede
the first record or follow the last. Headers must start with '@'. Inputs that break this
(blank lines between records, wrapped sequence/quality lines, records longer than the GPU
parser's carry reserve, FASTA and FASTQ mixed) are read as the reference's kseq reader reads
them: kseq_sequences below.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

_COUNT = {"A": 0, "C": 1, "G": 2, "T": 3, "a": 0, "c": 1, "g": 2, "t": 3}
_COMP = str.maketrans("ACGT", "TGCA")


class FastqError(ValueError):
    pass


def fastq_sequences(text: str) -> List[str]:
    """Sequence lines of a 4-line FASTQ text."""
    lines = text.split("\n")
    lines = [ln[:-1] if ln.endswith("\r") else ln for ln in lines]
    while lines and lines[0].strip(" \t\r") == "":
        lines.pop(0)
    while lines and lines[-1].strip(" \t\r") == "":
        lines.pop()
    if len(lines) % 4:
        raise FastqError("truncated record or blank line")
    seqs = []
    for i in range(0, len(lines), 4):
        if not lines[i].startswith("@"):
            raise FastqError("malformed header")
        seqs.append(lines[i + 1])
    return seqs


def kseq_sequences(text: str) -> List[str]:
    """Record sequences as klib kseq_read (MEGAHIT buildlib; kseq++ in reads.cpp) reads them:
    a record starts at the next '>' or '@' (anything before it is skipped); the header line
    is skipped; sequence lines are concatenated (blank lines skipped, one trailing '\\r'
    dropped) until a line starting with '>', '@' or '+'; '>'/'@' ends a FASTA record; after
    '+' the rest of that line is skipped and quality lines are read until at least as many
    quality characters as sequence characters were read (at least one line); a different
    count is an error. Used for the inputs the 4-line GPU parser hands to the host reader."""
    n = len(text)
    i = 0
    out: List[str] = []

    def line_at(i):
        j = text.find("\n", i)
        e = n if j < 0 else j
        ln = text[i:e]
        if ln.endswith("\r"):
            ln = ln[:-1]
        return ln, (n if j < 0 else j + 1)

    have_header = False
    while True:
        if not have_header:
            while i < n and text[i] not in ">@":
                i += 1
            if i >= n:
                return out
            i += 1
        _, i = line_at(i)  # header line
        seq = []
        c = None
        while i < n:
            c = text[i]
            if c in ">@+":
                break
            if c == "\n":
                i += 1
                c = None
                continue
            ln, i = line_at(i)
            seq.append(ln)
            c = None
        s = "".join(seq)
        if c is None:  # end of input
            out.append(s)
            return out
        if c in ">@":
            out.append(s)
            i += 1
            have_header = True
            continue
        _, i = line_at(i)  # the '+' line
        q = 0
        while i < n:
            ln, i = line_at(i)
            q += len(ln)
            if q >= len(s):
                break
        if q != len(s):
            raise FastqError("quality length differs from sequence length")
        out.append(s)
        have_header = False


def counting_view(seqs: Sequence[str]) -> List[str]:
    out = []
    for s in seqs:
        run = []
        for ch in s:
            if ch in _COUNT:
                run.append(ch.upper())
            elif run:
                out.append("".join(run))
                run = []
        if run:
            out.append("".join(run))
    return out


def mapping_view(files_seqs: Sequence[Sequence[str]]) -> List[List[int]]:
    out = []
    for fi, seqs in enumerate(files_seqs):
        for s in seqs:
            if fi > 0:
                s = s[::-1].translate(_COMP)
            out.append([0 if c == "A" else 1 if c == "C" else 2 if c == "G" else 3 for c in s])
    return out


def pack_codes(codes: Sequence[Sequence[int]]) -> Tuple[np.ndarray, np.ndarray]:
    """Packed 2-bit stream (base j at word j>>5, bits 2(j&31)) and offsets[n+1]."""
    offs = np.zeros(len(codes) + 1, dtype=np.uint64)
    flat = []
    for i, c in enumerate(codes):
        flat.extend(c)
        offs[i + 1] = len(flat)
    n = len(flat)
    words = np.zeros((n + 31) // 32 + 1, dtype=np.uint64)
    if n:
        a = np.asarray(flat, dtype=np.uint64)
        idx = np.arange(n, dtype=np.uint64)
        np.bitwise_or.at(words, (idx >> np.uint64(5)).astype(np.int64), a << (np.uint64(2) * (idx & np.uint64(31))))
    return words, offs


def pack_bases(reads: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
    return pack_codes([[_COUNT[c] for c in r] for r in reads])
