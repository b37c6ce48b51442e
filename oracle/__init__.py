"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU restatement (oracle/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
Parity status: "parity unpinned" (see oracle/oracle.h and DESIGN.md §Oracle).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)
_u16p = C.POINTER(C.c_uint16)
_u8p = C.POINTER(C.c_uint8)
_i32p = C.POINTER(C.c_int32)


class _Params(C.Structure):
    _fields_ = [("threshold_multiplicity", C.c_uint64), ("low_abundance", C.c_int), ("cycle_max_length", C.c_int),
                ("cycle_min_length", C.c_int), ("threads", C.c_int),
                ("cluster_bound", C.c_int), ("step_cap", C.c_longlong)]


_SIG = {
    "oracle_count_canonical": (C.c_uint64, [_u64p, _u64p, C.c_uint64, C.c_int, C.c_int, C.POINTER(_u64p), C.POINTER(_u32p)]),
    "oracle_build": (C.c_void_p, [_u64p, _u64p, C.c_uint64, C.c_int, C.c_int]),
    "oracle_graph_from_arrays": (C.c_void_p, [_u64p, _u16p, C.c_uint64, C.c_int]),
    "oracle_graph_free": (None, [C.c_void_p]),
    "oracle_graph_size": (C.c_uint64, [C.c_void_p]),
    "oracle_graph_k": (C.c_int, [C.c_void_p]),
    "oracle_graph_arrays": (None, [C.c_void_p, _u64p, _u16p]),
    "oracle_graph_valid": (None, [C.c_void_p, _u8p]),
    "oracle_graph_set_valid": (None, [C.c_void_p, _u8p]),
    "oracle_outgoing": (C.c_int, [C.c_void_p, C.c_uint64, _u64p]),
    "oracle_incoming": (C.c_int, [C.c_void_p, C.c_uint64, _u64p]),
    "oracle_get_label": (C.c_int, [C.c_void_p, C.c_uint64, _u8p]),
    "oracle_index_binary_search": (C.c_int64, [C.c_void_p, _u8p]),
    "oracle_reverse_pair_ends": (None, [C.c_char_p]),
    "oracle_get_reads": (C.c_uint64, [C.c_void_p, C.POINTER(C.c_char_p), C.c_uint64, C.c_uint64, _u64p, C.c_uint64,
                                      C.POINTER(_u64p), C.POINTER(_u64p)]),
    "oracle_cycle_finder": (C.c_void_p, [C.c_void_p, C.POINTER(_Params)]),
    "oracle_collect_tips": (C.c_uint64, [C.c_void_p, _u8p]),
    "oracle_invalidate_mult_one": (C.c_uint64, [C.c_void_p]),
    "oracle_recursive_reduction": (None, [C.c_void_p, _u8p]),
    "oracle_depth_level_search": (C.c_int, [C.c_void_p, C.c_uint64, C.c_int]),
    "oracle_cf_n_entries": (C.c_uint64, [C.c_void_p]),
    "oracle_cf_entries": (None, [C.c_void_p, _u64p, _u64p]),
    "oracle_cf_n_cycles": (C.c_uint64, [C.c_void_p]),
    "oracle_cf_n_nodes": (C.c_uint64, [C.c_void_p]),
    "oracle_cf_cycles": (None, [C.c_void_p, _u64p, _u64p]),
    "oracle_cf_map_order": (None, [C.c_void_p, _u64p]),
    "oracle_cf_stats": (None, [C.c_void_p, _u64p]),
    "oracle_cf_n_candidates": (C.c_uint64, [C.c_void_p]),
    "oracle_cf_candidates": (None, [C.c_void_p, _u64p, _i32p]),
    "oracle_cf_free": (None, [C.c_void_p]),
    "oracle_free": (None, [C.c_void_p]),
    "oracle_read_fastq": (C.c_uint64, [C.c_char_p, C.POINTER(_u64p), _u64p, C.POINTER(_u64p)]),
}
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        for n, (r, a) in _SIG.items():
            f = getattr(L, n)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def count_canonical(packed: np.ndarray, offsets: np.ndarray, k: int, threads: int = 1) -> Tuple[np.ndarray, np.ndarray]:
    packed = np.ascontiguousarray(packed, dtype=np.uint64)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    kp, cp = _u64p(), _u32p()
    n = lib().oracle_count_canonical(_p(packed, _u64p), _p(offsets, _u64p), offsets.size - 1, k, threads,
                                     C.byref(kp), C.byref(cp))
    keys = np.ctypeslib.as_array(kp, shape=(max(n, 1),))[:n].copy()
    counts = np.ctypeslib.as_array(cp, shape=(max(n, 1),))[:n].copy()
    lib().oracle_free(C.cast(kp, C.c_void_p))
    lib().oracle_free(C.cast(cp, C.c_void_p))
    return keys, counts


def read_fastq(path: str) -> Tuple[np.ndarray, np.ndarray]:
    """4-line FASTQ -> (packed, offsets), reads split at non-ACGT (C parser, test/baseline only)."""
    pp, op = _u64p(), _u64p()
    nw = C.c_uint64(0)
    n = lib().oracle_read_fastq(path.encode(), C.byref(pp), C.byref(nw), C.byref(op))
    if n == (1 << 64) - 1:
        raise ValueError(f"oracle_read_fastq failed on {path}")
    packed = np.ctypeslib.as_array(pp, shape=(max(nw.value, 1),))[: nw.value].copy()
    offs = np.ctypeslib.as_array(op, shape=(n + 1,)).copy()
    lib().oracle_free(C.cast(pp, C.c_void_p))
    lib().oracle_free(C.cast(op, C.c_void_p))
    return packed, offs


def reverse_pair_ends(s: str) -> str:
    """reads.cpp:20-31 (test oracle)."""
    b = C.create_string_buffer(s.encode())
    lib().oracle_reverse_pair_ends(b)
    return b.value.decode()


class OGraph:
    def __init__(self, h):
        self.h = h

    @classmethod
    def build(cls, packed, offsets, k, threads=1):
        packed = np.ascontiguousarray(packed, dtype=np.uint64)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        return cls(lib().oracle_build(_p(packed, _u64p), _p(offsets, _u64p), offsets.size - 1, k, threads))

    @classmethod
    def from_arrays(cls, keys, mult, k):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        mult = np.ascontiguousarray(mult, dtype=np.uint16)
        return cls(lib().oracle_graph_from_arrays(_p(keys, _u64p), _p(mult, _u16p), keys.size, k))

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_graph_free(self.h)
            self.h = None

    @property
    def size(self) -> int:
        return lib().oracle_graph_size(self.h)

    @property
    def k(self) -> int:
        return lib().oracle_graph_k(self.h)

    def arrays(self):
        n = self.size
        keys = np.zeros(max(n, 1), dtype=np.uint64)
        mult = np.zeros(max(n, 1), dtype=np.uint16)
        lib().oracle_graph_arrays(self.h, _p(keys, _u64p), _p(mult, _u16p))
        return keys[:n], mult[:n]

    def valid(self) -> np.ndarray:
        v = np.zeros(max(self.size, 1), dtype=np.uint8)
        lib().oracle_graph_valid(self.h, _p(v, _u8p))
        return v[: self.size]

    def set_valid(self, v: np.ndarray) -> None:
        v = np.ascontiguousarray(v, dtype=np.uint8)
        lib().oracle_graph_set_valid(self.h, _p(v, _u8p))

    def outgoing(self, e: int) -> List[int]:
        o = np.zeros(4, dtype=np.uint64)
        n = lib().oracle_outgoing(self.h, e, _p(o, _u64p))
        return [int(x) for x in o[:n]]

    def incoming(self, e: int) -> List[int]:
        o = np.zeros(4, dtype=np.uint64)
        n = lib().oracle_incoming(self.h, e, _p(o, _u64p))
        return [int(x) for x in o[:n]]

    def label(self, e: int) -> List[int]:
        s = np.zeros(max(self.k, 1), dtype=np.uint8)
        lib().oracle_get_label(self.h, e, _p(s, _u8p))
        return [int(x) for x in s]

    def index_binary_search(self, seq) -> int:
        s = np.ascontiguousarray(seq, dtype=np.uint8)
        return lib().oracle_index_binary_search(self.h, _p(s, _u8p))

    def get_reads(self, seqs: Sequence[str], n_file1: int, cycle_nodes) -> List[List[int]]:
        """reads.cpp:88-130 (test oracle): relevant reads as node-id chains."""
        arr = (C.c_char_p * max(len(seqs), 1))(*[x.encode() for x in seqs])
        nodes = np.ascontiguousarray(np.asarray(list(cycle_nodes), dtype=np.uint64))
        fp, op = _u64p(), _u64p()
        n = lib().oracle_get_reads(self.h, arr, len(seqs), n_file1, _p(nodes, _u64p), nodes.size, C.byref(fp),
                                   C.byref(op))
        offs = np.ctypeslib.as_array(op, shape=(n + 1,)).copy()
        flat = np.ctypeslib.as_array(fp, shape=(max(int(offs[-1]), 1),))[: int(offs[-1])].copy()
        lib().oracle_free(C.cast(fp, C.c_void_p))
        lib().oracle_free(C.cast(op, C.c_void_p))
        return [flat[offs[i]:offs[i + 1]].tolist() for i in range(n)]

    def collect_tips(self) -> np.ndarray:
        t = np.zeros(max(self.size, 1), dtype=np.uint8)
        lib().oracle_collect_tips(self.h, _p(t, _u8p))
        return t[: self.size]

    def invalidate_mult_one(self) -> int:
        return lib().oracle_invalidate_mult_one(self.h)

    def recursive_reduction(self, tips: np.ndarray) -> None:
        t = np.ascontiguousarray(tips, dtype=np.uint8)
        lib().oracle_recursive_reduction(self.h, _p(t, _u8p))

    def dls(self, start: int, limit: int = 77) -> bool:
        return bool(lib().oracle_depth_level_search(self.h, start, limit))

    def cycle_finder(self, threshold_multiplicity=20, low_abundance=True, cycle_max_length=77,
                     cycle_min_length=27, threads=1, cluster_bound=500, step_cap=10_000_000) -> dict:
        p = _Params(threshold_multiplicity, int(low_abundance), cycle_max_length, cycle_min_length, threads,
                    cluster_bound, step_cap)
        L = lib()
        r = L.oracle_cycle_finder(self.h, C.byref(p))
        try:
            ne = L.oracle_cf_n_entries(r)
            starts = np.zeros(max(ne, 1), dtype=np.uint64)
            cb = np.zeros(ne + 1, dtype=np.uint64)
            L.oracle_cf_entries(r, _p(starts, _u64p), _p(cb, _u64p))
            nc = L.oracle_cf_n_cycles(r)
            nn = L.oracle_cf_n_nodes(r)
            nb = np.zeros(nc + 1, dtype=np.uint64)
            nodes = np.zeros(max(nn, 1), dtype=np.uint64)
            L.oracle_cf_cycles(r, _p(nb, _u64p), _p(nodes, _u64p))
            order = np.zeros(max(ne, 1), dtype=np.uint64)
            L.oracle_cf_map_order(r, _p(order, _u64p))
            st = np.zeros(6, dtype=np.uint64)
            L.oracle_cf_stats(r, _p(st, _u64p))
            ncand = L.oracle_cf_n_candidates(r)
            cid = np.zeros(max(ncand, 1), dtype=np.uint64)
            cbk = np.zeros(max(ncand, 1), dtype=np.int32)
            L.oracle_cf_candidates(r, _p(cid, _u64p), _p(cbk, _i32p))
            entries = []
            for i in range(ne):
                cycles = []
                for c in range(int(cb[i]), int(cb[i + 1])):
                    cycles.append([int(x) for x in nodes[int(nb[c]):int(nb[c + 1])]])
                entries.append((int(starts[i]), cycles))
            return {
                "entries": entries,
                "map_order": [int(x) for x in order[:ne]],
                "stats": [int(x) for x in st],
                "candidates": [int(x) for x in cid[:ncand]],
                "buckets": [int(x) for x in cbk[:ncand]],
            }
        finally:
            L.oracle_cf_free(r)
