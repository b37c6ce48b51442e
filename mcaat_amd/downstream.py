"""ctypes binding of libmcaat_host.so (include/mcaat_host.h): the reference's host steps after
CycleFinder — spacer ordering, get_systems and CRISPRAnalyzer (CRISPR_Arrays.txt) — restated
in C++ (mcaat_amd/host/). The mcaat CLI runs the same code; this binding serves tests and tools.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence

import numpy as np

from .lib import McaatError, load_library

HOST_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmcaat_host.so")

_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)
_u16p = C.POINTER(C.c_uint16)
_u8p = C.POINTER(C.c_uint8)

HOST_SIGNATURES = {
    "mcaat_host_last_error": (C.c_char_p, []),
    "mcaat_host_fuzz_ratio": (C.c_double, [C.c_char_p, C.c_char_p]),
    "mcaat_host_fuzz_partial_ratio": (C.c_double, [C.c_char_p, C.c_char_p]),
    "mcaat_host_min_cover": (C.c_int, [_u32p, C.c_size_t, _u32p, _u64p, C.c_size_t, _u64p, C.POINTER(C.c_size_t)]),
    "mcaat_host_crispr_arrays": (C.c_int, [C.c_int, _u64p, _u16p, _u8p, C.c_uint64, _u64p, _u64p, C.c_size_t, _u64p,
                                           _u64p, C.c_size_t, C.c_char_p, C.POINTER(C.c_size_t), C.c_int]),
    "mcaat_host_crispr_analyzer": (C.c_int, [C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_size_t, C.c_char_p]),
}

_hlib: Optional[C.CDLL] = None


def load_host_library(path: str = HOST_LIB_PATH) -> C.CDLL:
    global _hlib
    if _hlib is not None:
        return _hlib
    load_library()  # libmcaat_gpu.so first (dependency)
    if not os.path.exists(path):
        raise McaatError(-1, f"{path} not built; run `make -C mcaat_amd/host` (or __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, (res, args) in HOST_SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _hlib = lib
    return lib


def _check(rc: int) -> None:
    if rc != 0:
        msg = load_host_library().mcaat_host_last_error()
        raise McaatError(rc, msg.decode() if msg else "")


def _flat(seqs: Sequence[Sequence[int]], dtype=np.uint64):
    offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
    for i, s in enumerate(seqs):
        offs[i + 1] = offs[i] + len(s)
    flat = np.zeros(max(int(offs[-1]), 1), dtype=dtype)
    for i, s in enumerate(seqs):
        flat[int(offs[i]):int(offs[i + 1])] = s
    return flat, offs


def fuzz_ratio(a: str, b: str) -> float:
    return load_host_library().mcaat_host_fuzz_ratio(a.encode(), b.encode())


def fuzz_partial_ratio(a: str, b: str) -> float:
    return load_host_library().mcaat_host_fuzz_partial_ratio(a.encode(), b.encode())


def min_cover(universe: Sequence[int], sets: Sequence[Sequence[int]]) -> List[int]:
    """solve_min_cover_problem (spacer_ordering.cpp:265-313)."""
    u = np.ascontiguousarray(np.asarray(list(universe), dtype=np.uint32).reshape(-1))
    flat, offs = _flat(sets, np.uint32)
    out = np.zeros(max(len(sets), 1), dtype=np.uint64)
    n = C.c_size_t(0)
    _check(load_host_library().mcaat_host_min_cover(u.ctypes.data_as(_u32p), u.size, flat.ctypes.data_as(_u32p),
                                                     offs.ctypes.data_as(_u64p), len(sets), out.ctypes.data_as(_u64p),
                                                     C.byref(n)))
    return [int(x) for x in out[: n.value]]


def crispr_arrays(k: int, keys: np.ndarray, mult: np.ndarray, valid: np.ndarray, cycles: Sequence[Sequence[int]],
                  reads: Sequence[Sequence[int]], output_file: str, threads: int = 1) -> int:
    """Steps 7-8 + CRISPRAnalyzer on a host copy of the graph; writes output_file. `valid`
    (uint8, one per edge) is updated in place as the reference mutates the SDBG. threads > 1 solves
    the subproblems on that many host threads (the output is the serial loop's)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    mult = np.ascontiguousarray(mult, dtype=np.uint16)
    assert valid.dtype == np.uint8 and valid.flags["C_CONTIGUOUS"] and valid.size == keys.size
    cf, co = _flat(cycles)
    rf, ro = _flat(reads)
    n = C.c_size_t(0)
    _check(load_host_library().mcaat_host_crispr_arrays(
        k, keys.ctypes.data_as(_u64p), mult.ctypes.data_as(_u16p), valid.ctypes.data_as(_u8p), keys.size,
        cf.ctypes.data_as(_u64p), co.ctypes.data_as(_u64p), len(cycles), rf.ctypes.data_as(_u64p),
        ro.ctypes.data_as(_u64p), len(reads), output_file.encode(), C.byref(n), threads))
    return n.value


def crispr_analyzer(systems: Sequence[tuple], output_file: str) -> None:
    """CRISPRAnalyzer(systems).run_analysis() for [(repeat, [spacers...]), ...] (insertion order)."""
    reps = (C.c_char_p * max(len(systems), 1))(*[r.encode() for r, _ in systems])
    sps = (C.c_char_p * max(len(systems), 1))(*[",".join(s).encode() for _, s in systems])
    _check(load_host_library().mcaat_host_crispr_analyzer(reps, sps, len(systems), output_file.encode()))
