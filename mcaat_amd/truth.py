"""Scoring a CRISPR_Arrays.txt against the planted arrays of a synthetic community.

The reference's own check is step 8 with a benchmark file (main_run_and_debug.cpp:145-218:
each found system's sequence against its most similar true sequence). For the synthetic
configs the truth is exact (mcaat_synth_arrays_host), so recall is decided per planted array:
an array is recalled when one reported system carries at least half of its spacers, each
compared in either orientation (the graph holds both strands, so a system may come out
reverse-complemented) and allowed to differ by a few bases at either end (CRISPRAnalyzer
trims and extends repeat/spacer boundaries by common prefix/suffix k-mers,
post_processing.h:176-259).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

_RC = str.maketrans("ACGT", "TGCA")


def revcomp(s: str) -> str:
    return s.translate(_RC)[::-1]


def parse_crispr_arrays(path: str) -> List[Tuple[str, List[str]]]:
    """(repeat, spacers) per system of a CRISPR_Arrays.txt (crispr_report.cpp format)."""
    rule = "-" * 50
    lines = [ln.rstrip("\n") for ln in open(path)]
    out = []
    i = 0
    while i < len(lines):
        # a system: rule, repeat, rule, spacers..., rule, "Number of Spacers: n", rule
        if lines[i] == rule and i + 2 < len(lines) and lines[i + 2] == rule and lines[i + 1] and \
                set(lines[i + 1]) <= set("ACGTN"):
            repeat = lines[i + 1]
            j = i + 3
            spacers = []
            while j < len(lines) and lines[j] != rule:
                spacers.append(lines[j])
                j += 1
            if j + 1 < len(lines) and lines[j + 1].startswith("Number of Spacers:"):
                out.append((repeat, spacers))
                i = j + 2
                continue
        i += 1
    return out


def _close(a: str, b: str, slack: int) -> bool:
    if a == b:
        return True
    if abs(len(a) - len(b)) > 2 * slack:
        return False
    short, long_ = (a, b) if len(a) <= len(b) else (b, a)
    if len(short) < 16:
        return False
    # one contains the other up to `slack` bases trimmed from each end of the shorter
    for lo in range(0, slack + 1):
        for hi in range(0, slack + 1):
            core = short[lo:len(short) - hi]
            if len(core) >= 16 and core in long_:
                return True
    return False


def planted_recall(systems: Sequence[Tuple[str, List[str]]], planted: Sequence[Tuple[int, int, str, List[str]]],
                   slack: int = 3, need: float = 0.5) -> Dict:
    """Which planted arrays some reported system recalls (see the module docstring)."""
    K = 12
    index: Dict[str, set] = {}  # 12-mer of a reported spacer (either orientation) -> (system, spacer)
    for si, (_rep, sps) in enumerate(systems):
        for sp in sps:
            for o in (sp, revcomp(sp)):
                for i in range(0, len(o) - K + 1):
                    index.setdefault(o[i:i + K], set()).add((si, o))
    recalled = []
    missed = []
    for g, a, _rep, sps in planted:
        hits: Dict[int, int] = {}
        for p in sps:
            cands = set()
            for i in range(slack, len(p) - K - slack + 1, 4):
                cands |= index.get(p[i:i + K], set())
            seen = {si for si, o in cands if _close(o, p, slack)}
            for si in seen:
                hits[si] = hits.get(si, 0) + 1
        best = max(hits.values()) if hits else 0
        if sps and best >= need * len(sps):
            recalled.append((g, a))
        else:
            missed.append({"genome": g, "array": a, "best_spacers": best, "spacers": len(sps)})
    return {
        "planted": len(planted),
        "recalled": len(recalled),
        "recall": len(recalled) / max(1, len(planted)),
        "systems": len(systems),
        "missed": missed[:20],
    }
