"""ctypes binding of libmcaat_gpu.so (include/mcaat_gpu.h)."""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

# MCAAT_LIB: load another build of the same library (A/B experiments)
LIB_PATH = os.environ.get("MCAAT_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmcaat_gpu.so")

_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)
_u16p = C.POINTER(C.c_uint16)
_u8p = C.POINTER(C.c_uint8)
_i32p = C.POINTER(C.c_int32)


class McaatError(RuntimeError):
    """Raised for a negative mcaat_status (message from mcaat_last_error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"mcaat error {code}: {msg}")
        self.code = code


class _SynthSpec(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("n_genomes", C.c_uint32),
        ("genome_len", C.c_uint64),
        ("arrays_per_genome", C.c_uint32),
        ("spacers_per_array", C.c_uint32),
        ("repeat_len_min", C.c_uint32),
        ("repeat_len_max", C.c_uint32),
        ("spacer_len_min", C.c_uint32),
        ("spacer_len_max", C.c_uint32),
        ("read_len", C.c_uint32),
        ("n_reads", C.c_uint64),
        ("error_rate", C.c_double),
        ("paired", C.c_int32),
    ]


class _CfParams(C.Structure):
    _fields_ = [
        ("threshold_multiplicity", C.c_uint64),
        ("low_abundance", C.c_int32),
        ("cycle_max_length", C.c_int32),
        ("cycle_min_length", C.c_int32),
        ("cluster_bound", C.c_int32),
        ("step_cap", C.c_int64),
    ]


# every exported symbol and its ctypes signature (restype, argtypes)
SIGNATURES = {
    "mcaat_init": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "mcaat_finalize": (None, [C.c_void_p]),
    "mcaat_last_error": (C.c_char_p, []),
    "mcaat_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "mcaat_preload": (C.c_int, [C.c_int]),
    "mcaat_reads_from_host": (C.c_int, [C.c_void_p, _u64p, C.c_uint64, _u64p, C.c_uint64, C.POINTER(C.c_void_p)]),
    "mcaat_reads_from_fastx": (C.c_int, [C.c_void_p, C.POINTER(C.c_char_p), C.c_int, C.POINTER(C.c_void_p)]),
    "mcaat_count_ahead": (C.c_int, [C.c_void_p, C.c_int]),
    "mcaat_reads_info": (C.c_int, [C.c_void_p, _u64p, _u64p]),
    "mcaat_reads_download": (C.c_int, [C.c_void_p, _u64p, _u64p]),
    "mcaat_reads_records_download": (C.c_int, [C.c_void_p, _u64p, _u64p]),
    "mcaat_reads_free": (None, [C.c_void_p]),
    "mcaat_reads_synth": (C.c_int, [C.c_void_p, C.POINTER(_SynthSpec), C.POINTER(C.c_void_p)]),
    "mcaat_synth_host": (C.c_int, [C.POINTER(_SynthSpec), _u64p, _u64p]),
    "mcaat_synth_genome_host": (C.c_int, [C.POINTER(_SynthSpec), _u64p]),
    "mcaat_synth_arrays_host": (C.c_int, [C.POINTER(_SynthSpec), C.c_char_p, C.c_uint64, _u64p]),
    "mcaat_trim": (None, [C.c_void_p]),
    "mcaat_count_edges": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, _u64p, C.POINTER(_u64p), C.POINTER(_u32p)]),
    "mcaat_free": (None, [C.c_void_p]),
    "mcaat_build_graph": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    "mcaat_graph_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), _u64p]),
    "mcaat_graph_download": (C.c_int, [C.c_void_p, _u64p, _u16p, _u8p]),
    "mcaat_graph_set_valid": (C.c_int, [C.c_void_p, _u64p, C.c_size_t, C.c_int]),
    "mcaat_graph_neighbors": (C.c_int, [C.c_void_p, _u64p, C.c_size_t, C.c_int, _u64p, _i32p]),
    "mcaat_graph_free": (None, [C.c_void_p]),
    "mcaat_cf_default_params": (None, [C.POINTER(_CfParams)]),
    "mcaat_cycle_finder": (C.c_int, [C.c_void_p, C.POINTER(_CfParams), C.POINTER(C.c_void_p)]),
    "mcaat_cycles_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_size_t)]),
    "mcaat_cycles_get": (
        C.c_int,
        [C.c_void_p, C.c_size_t, _u64p, C.POINTER(_u64p), C.POINTER(_u64p), C.POINTER(C.c_size_t)],
    ),
    "mcaat_cycles_stats": (C.c_int, [C.c_void_p, _u64p]),
    "mcaat_cycles_export": (C.c_int, [C.c_void_p, _u64p, _u64p, _u64p, _u64p, _u64p]),
    "mcaat_cycles_candidates": (C.c_int, [C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(_u64p), C.POINTER(_i32p)]),
    "mcaat_cycles_free": (None, [C.c_void_p]),
    "mcaat_stage_times": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    "mcaat_kernel_timing": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_double), _u64p, C.POINTER(C.c_double)]),
    "mcaat_reset_timing": (None, [C.c_void_p]),
    "mcaat_reads_synth_range": (C.c_int, [C.c_void_p, C.POINTER(_SynthSpec), C.c_uint64, C.c_uint64,
                                          C.POINTER(C.c_void_p)]),
    "mcaat_count_local": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    "mcaat_counts_info": (C.c_int, [C.c_void_p, _u64p]),
    "mcaat_counts_histogram": (C.c_int, [C.c_void_p, C.c_int, _u64p]),
    "mcaat_counts_partition": (C.c_int, [C.c_void_p, C.c_int, _u64p, _u64p, C.c_void_p, C.c_void_p, C.c_uint64]),
    "mcaat_counts_free": (None, [C.c_void_p]),
    "mcaat_edges_reduce": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                     _u64p]),
    "mcaat_graph_from_sorted": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64,
                                          C.POINTER(C.c_void_p)]),
    "mcaat_reads_records_info": (C.c_int, [C.c_void_p, _u64p, C.POINTER(C.c_int)]),
    "mcaat_graph_keep_only": (C.c_int, [C.c_void_p, _u64p, C.c_size_t]),
    "mcaat_graph_gather": (C.c_int, [C.c_void_p, _u64p, C.c_size_t, _u64p, _u16p]),
    "mcaat_map_reads": (C.c_int, [C.c_void_p, C.c_void_p, _u64p, C.c_size_t, C.c_uint64, C.POINTER(C.c_void_p)]),
    "mcaat_mapped_get": (C.c_int, [C.c_void_p, _u64p, C.POINTER(_u64p), C.POINTER(_u64p), C.POINTER(_u64p)]),
    "mcaat_mapped_free": (None, [C.c_void_p]),
    "mcaat_set_knob": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int64]),
    "mcaat_reads_write_fastq": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int]),
    "mcaat_graph_save": (C.c_int, [C.c_void_p, C.c_char_p]),
    "mcaat_graph_load": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_void_p)]),
    "mcaat_graph_download_range": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, _u64p, _u16p, _u8p]),
    "mcaat_graph_valid_words": (C.c_int, [C.c_void_p, _u64p]),
    "mcaat_graph_keep_region": (C.c_int, [C.c_void_p, _u64p, C.c_size_t, C.c_uint64]),
    "mcaat_graph_succinct_check": (C.c_int, [C.c_void_p, C.c_int, _u64p, C.POINTER(C.c_double)]),
    "mcaat_graph_valid_subgraph": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), _u64p, C.POINTER(C.c_uint32),
                                             _u8p]),
    "mcaat_comm_unique_id": (C.c_int, [_u8p]),
    "mcaat_comm_schedule_check": (C.c_int, [C.c_int, C.c_uint64, C.c_uint64, _u64p]),
    "mcaat_comm_init_rccl": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _u8p, C.POINTER(C.c_void_p)]),
    "mcaat_comm_init_shm": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_char_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    "mcaat_comm_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "mcaat_comm_barrier": (C.c_int, [C.c_void_p]),
    "mcaat_comm_allgather_sizes": (C.c_int, [C.c_void_p, C.c_uint64, _u64p]),
    "mcaat_comm_allgatherv": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, _u64p]),
    "mcaat_comm_free": (None, [C.c_void_p]),
    "mcaat_reads_from_fastx_part": (C.c_int, [C.c_void_p, C.POINTER(C.c_char_p), C.c_int, C.c_int, C.c_int,
                                              C.POINTER(C.c_void_p)]),
    "mcaat_reads_file_records": (C.c_int, [C.c_void_p, C.c_int, _u64p]),
    "mcaat_build_graph_sharded": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    "mcaat_cycle_finder_comm": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(_CfParams), C.POINTER(C.c_void_p)]),
    "mcaat_arena_check": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "mcaat_arena_usage": (C.c_int, [C.c_void_p, C.c_int, _u64p, _u64p, _u64p]),
    "mcaat_graph_shard_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), _u64p, _u64p]),
    "mcaat_graph_unshard": (C.c_int, [C.c_void_p, C.c_void_p]),
}

_lib: Optional[C.CDLL] = None


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load libmcaat_gpu.so (fails loudly: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise McaatError(-1, f"{path} not built; run `make -C mcaat_amd` (or __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc: int) -> None:
    if rc != 0:
        msg = load_library().mcaat_last_error()
        raise McaatError(rc, msg.decode() if msg else "")


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(t)


def device_count() -> int:
    n = C.c_int(0)
    _check(load_library().mcaat_device_count(C.byref(n)))
    return n.value


def preload(device: int = 0) -> None:
    """Load every module's kernel code objects on `device` now (mcaat_preload), so that the
    first launch of a stage does not pay HIP's deferred code-object load inside a timed region."""
    _check(load_library().mcaat_preload(device))


@dataclass
class SynthSpec:
    """Synthetic metagenome. Defaults: the C1 tiny config."""

    seed: int = 1
    n_genomes: int = 1
    genome_len: int = 50_000
    arrays_per_genome: int = 1
    spacers_per_array: int = 12
    repeat_len_min: int = 30
    repeat_len_max: int = 30
    spacer_len_min: int = 32
    spacer_len_max: int = 32
    read_len: int = 150
    n_reads: int = 10_000
    error_rate: float = 0.0
    paired: bool = False

    def to_c(self) -> _SynthSpec:
        return _SynthSpec(
            self.seed, self.n_genomes, self.genome_len, self.arrays_per_genome, self.spacers_per_array,
            self.repeat_len_min, self.repeat_len_max, self.spacer_len_min, self.spacer_len_max,
            self.read_len, self.n_reads, float(self.error_rate), int(self.paired),
        )


def synth_host(spec: SynthSpec) -> Tuple[np.ndarray, np.ndarray]:
    """Host copy of the reads mcaat_reads_synth generates in HBM (packed words, offsets)."""
    nb = spec.n_reads * spec.read_len
    packed = np.zeros((nb + 31) // 32 + 1, dtype=np.uint64)
    offsets = np.zeros(spec.n_reads + 1, dtype=np.uint64)
    s = spec.to_c()
    _check(load_library().mcaat_synth_host(C.byref(s), _ptr(packed, _u64p), _ptr(offsets, _u64p)))
    return packed[: (nb + 31) // 32], offsets


def synth_genome_host(spec: SynthSpec) -> np.ndarray:
    total = spec.n_genomes * spec.genome_len
    packed = np.zeros((total + 31) // 32 + 1, dtype=np.uint64)
    s = spec.to_c()
    _check(load_library().mcaat_synth_genome_host(C.byref(s), _ptr(packed, _u64p)))
    return packed


def synth_arrays(spec: SynthSpec) -> List[Tuple[int, int, str, List[str]]]:
    """The planted CRISPR arrays of the synthetic community: (genome, index, repeat, spacers),
    genome strand (mcaat_synth_arrays_host)."""
    lib = load_library()
    s = spec.to_c()
    n = C.c_uint64(0)
    _check(lib.mcaat_synth_arrays_host(C.byref(s), None, 0, C.byref(n)))
    buf = C.create_string_buffer(n.value + 1)
    _check(lib.mcaat_synth_arrays_host(C.byref(s), buf, n.value + 1, C.byref(n)))
    out = []
    for line in buf.value.decode().splitlines():
        g, a, rep, sp = line.split("\t")
        out.append((int(g), int(a), rep, sp.split(",") if sp else []))
    return out


class Context:
    """One GPU, one HIP stream (mcaat_ctx)."""

    def __init__(self, device: int = 0):
        self._lib = load_library()
        h = C.c_void_p()
        _check(self._lib.mcaat_init(device, C.byref(h)))
        self.h = h
        self.device = device

    def close(self) -> None:
        if self.h:
            self._lib.mcaat_finalize(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def stage_times(self) -> dict:
        names = (C.c_char_p * 32)()
        ms = (C.c_double * 32)()
        n = C.c_int(0)
        _check(self._lib.mcaat_stage_times(self.h, 32, names, ms, C.byref(n)))
        return {names[i].decode(): ms[i] for i in range(min(n.value, 32))}

    def kernel_timing(self, name: str) -> Tuple[float, int, float]:
        avg = C.c_double(0)
        n = C.c_uint64(0)
        b = C.c_double(0)
        _check(self._lib.mcaat_kernel_timing(self.h, name.encode(), C.byref(avg), C.byref(n), C.byref(b)))
        return avg.value, n.value, b.value

    def reset_timing(self) -> None:
        self._lib.mcaat_reset_timing(self.h)

    def trim(self) -> None:
        """Release device memory the arena keeps but nothing uses (mcaat_trim)."""
        self._lib.mcaat_trim(self.h)

    def arena_check(self) -> Tuple[bool, bool, int, bool, bool]:
        """The device arena's stream order (mcaat_arena_check): (same block reused, the side
        stream's writes survived the main stream's queued ones, fence waits, and for a consumer
        stream the arena does not watch: same block reused, its writes survived)."""
        out = (C.c_int64 * 5)()
        _check(self._lib.mcaat_arena_check(self.h, out))
        return bool(out[0]), bool(out[1]), int(out[2]), bool(out[3]), bool(out[4])

    def arena_usage(self, reset_peak: bool = False) -> Tuple[int, int, int]:
        """(bytes in use, peak since the last reset, bytes the arena holds) on this GPU."""
        a, b, c = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        _check(self._lib.mcaat_arena_usage(self.h, int(reset_peak), C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def count_ahead(self, k: int) -> None:
        """The next Reads.from_fastx on this context runs node_counter's pass A for k while
        the input is read (include/mcaat_gpu.h, mcaat_count_ahead); k = 0 cancels."""
        _check(self._lib.mcaat_count_ahead(self.h, int(k)))

    def set_knob(self, name: str, value: int) -> None:
        """Size limit that picks a code path (include/mcaat_gpu.h, mcaat_set_knob); value < 0
        restores the default."""
        _check(self._lib.mcaat_set_knob(self.h, name.encode(), int(value)))

    def knobs(self, **values):
        """Context manager: knobs set for the block (keyword names use '__' for '.'),
        restored to their defaults afterwards."""
        import contextlib

        @contextlib.contextmanager
        def _cm():
            names = [k.replace("__", ".") for k in values]
            try:
                for n, v in zip(names, values.values()):
                    self.set_knob(n, v)
                yield self
            finally:
                for n in names:
                    self.set_knob(n, -1)

        return _cm()


class Comm:
    """The ranks of one multi-GPU run (mcaat_comm): RCCL between GPUs, or a POSIX
    shared-memory segment that stages device data through the host (ranks sharing a GPU,
    rehearsals; ctx None: host collectives only, no GPU needed)."""

    ID_BYTES = 128

    def __init__(self, h):
        self._lib = load_library()
        self.h = h
        w, r = C.c_int(0), C.c_int(0)
        _check(self._lib.mcaat_comm_info(h, C.byref(w), C.byref(r)))
        self.world, self.rank = w.value, r.value

    @staticmethod
    def unique_id() -> bytes:
        buf = np.zeros(Comm.ID_BYTES, dtype=np.uint8)
        _check(load_library().mcaat_comm_unique_id(_ptr(buf, _u8p)))
        return buf.tobytes()

    @staticmethod
    def schedule_check(world: int, seed: int, piece_bytes: int) -> int:
        """Host self-check of the RCCL segment all-to-all's schedule (mcaat_comm_schedule_check):
        raises on a pairing or tiling error, returns the most rounds of any rank."""
        n = C.c_uint64(0)
        _check(load_library().mcaat_comm_schedule_check(int(world), int(seed), int(piece_bytes), C.byref(n)))
        return n.value

    @classmethod
    def rccl(cls, ctx: "Context", world: int, rank: int, uid: bytes) -> "Comm":
        buf = np.frombuffer(uid, dtype=np.uint8).copy()
        h = C.c_void_p()
        _check(load_library().mcaat_comm_init_rccl(ctx.h, world, rank, _ptr(buf, _u8p), C.byref(h)))
        return cls(h)

    @classmethod
    def shm(cls, ctx: Optional["Context"], world: int, rank: int, name: str, slot_bytes: int = 0) -> "Comm":
        h = C.c_void_p()
        _check(load_library().mcaat_comm_init_shm(ctx.h if ctx else None, world, rank, name.encode(), slot_bytes,
                                                  C.byref(h)))
        return cls(h)

    def barrier(self) -> None:
        _check(self._lib.mcaat_comm_barrier(self.h))

    def allgather_bytes(self, data: bytes) -> List[bytes]:
        """Every rank's bytes, in rank order."""
        sizes = np.zeros(self.world, dtype=np.uint64)
        _check(self._lib.mcaat_comm_allgather_sizes(self.h, len(data), _ptr(sizes, _u64p)))
        out = np.zeros(max(int(sizes.sum()), 1), dtype=np.uint8)
        src = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(1, np.uint8)
        _check(self._lib.mcaat_comm_allgatherv(self.h, src.ctypes.data_as(C.c_void_p), len(data),
                                               out.ctypes.data_as(C.c_void_p), _ptr(sizes, _u64p)))
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        return [out[offs[r]:offs[r + 1]].tobytes() for r in range(self.world)]

    def close(self) -> None:
        if self.h:
            self._lib.mcaat_comm_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Reads:
    """Packed 2-bit reads resident in HBM (mcaat_reads)."""

    def __init__(self, ctx: Context, h):
        self.ctx = ctx
        self.h = h

    @classmethod
    def from_host(cls, ctx: Context, packed: np.ndarray, offsets: np.ndarray) -> "Reads":
        packed = np.ascontiguousarray(packed, dtype=np.uint64)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        h = C.c_void_p()
        _check(ctx._lib.mcaat_reads_from_host(ctx.h, _ptr(packed, _u64p), packed.size, _ptr(offsets, _u64p),
                                              offsets.size - 1, C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def synth(cls, ctx: Context, spec: SynthSpec) -> "Reads":
        h = C.c_void_p()
        s = spec.to_c()
        _check(ctx._lib.mcaat_reads_synth(ctx.h, C.byref(s), C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def synth_range(cls, ctx: Context, spec: SynthSpec, first: int, count: int) -> "Reads":
        """Reads [first, first+count) of the stream `synth` generates (a rank's slice)."""
        h = C.c_void_p()
        s = spec.to_c()
        _check(ctx._lib.mcaat_reads_synth_range(ctx.h, C.byref(s), first, count, C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_fastx(cls, ctx: Context, files: Sequence[str]) -> "Reads":
        arr = (C.c_char_p * len(files))(*[f.encode() for f in files])
        h = C.c_void_p()
        _check(ctx._lib.mcaat_reads_from_fastx(ctx.h, arr, len(files), C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_fastx_part(cls, ctx: Context, files: Sequence[str], part: int, n_parts: int) -> "Reads":
        """Part `part` of n_parts of the FASTQ inputs (cut at record starts; .gz whole on part 0)."""
        arr = (C.c_char_p * len(files))(*[f.encode() for f in files])
        h = C.c_void_p()
        _check(ctx._lib.mcaat_reads_from_fastx_part(ctx.h, arr, len(files), part, n_parts, C.byref(h)))
        return cls(ctx, h)

    def file_records(self, file: int) -> int:
        n = C.c_uint64(0)
        _check(self.ctx._lib.mcaat_reads_file_records(self.h, file, C.byref(n)))
        return n.value

    def info(self) -> Tuple[int, int]:
        n = C.c_uint64(0)
        b = C.c_uint64(0)
        _check(self.ctx._lib.mcaat_reads_info(self.h, C.byref(n), C.byref(b)))
        return n.value, b.value

    def records_info(self) -> Tuple[int, bool]:
        n = C.c_uint64(0)
        sep = C.c_int(0)
        _check(self.ctx._lib.mcaat_reads_records_info(self.h, C.byref(n), C.byref(sep)))
        return n.value, bool(sep.value)

    def download(self) -> Tuple[np.ndarray, np.ndarray]:
        n, b = self.info()
        packed = np.zeros((b + 31) // 32, dtype=np.uint64)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        _check(self.ctx._lib.mcaat_reads_download(self.h, _ptr(packed, _u64p), _ptr(offsets, _u64p)))
        return packed, offsets

    def download_records(self) -> Tuple[np.ndarray, np.ndarray]:
        """Mapping view (one entry per input record; reads.cpp:20-52 coding)."""
        n, _ = self.records_info()
        offsets = np.zeros(n + 1, dtype=np.uint64)
        _check(self.ctx._lib.mcaat_reads_records_download(self.h, None, _ptr(offsets, _u64p)))
        packed = np.zeros((int(offsets[-1]) + 31) // 32 + 1, dtype=np.uint64)
        _check(self.ctx._lib.mcaat_reads_records_download(self.h, _ptr(packed, _u64p), _ptr(offsets, _u64p)))
        return packed, offsets

    def write_fastq(self, path: str, threads: int = 8) -> None:
        """The counting view as 4-line FASTQ (mcaat_reads_write_fastq)."""
        _check(self.ctx._lib.mcaat_reads_write_fastq(self.h, path.encode(), threads))

    def free(self) -> None:
        if self.h:
            self.ctx._lib.mcaat_reads_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def count_edges(ctx: Context, reads: Reads, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """node_counter: sorted canonical (k+1)-mers (LSB-first) and their counts."""
    n = C.c_uint64(0)
    kp = _u64p()
    cp = _u32p()
    _check(ctx._lib.mcaat_count_edges(ctx.h, reads.h, k, C.byref(n), C.byref(kp), C.byref(cp)))
    try:
        keys = np.ctypeslib.as_array(kp, shape=(max(n.value, 1),))[: n.value].copy()
        counts = np.ctypeslib.as_array(cp, shape=(max(n.value, 1),))[: n.value].copy()
    finally:
        ctx._lib.mcaat_free(C.cast(kp, C.c_void_p))
        ctx._lib.mcaat_free(C.cast(cp, C.c_void_p))
    return keys, counts


class Counts:
    """Device-resident canonical counts of one rank (mcaat_counts; multi-GPU build)."""

    def __init__(self, ctx: Context, h, k: int):
        self.ctx = ctx
        self.h = h
        self.k = k

    @classmethod
    def count(cls, ctx: Context, reads: Reads, k: int) -> "Counts":
        h = C.c_void_p()
        _check(ctx._lib.mcaat_count_local(ctx.h, reads.h, k, C.byref(h)))
        return cls(ctx, h, k)

    @property
    def n(self) -> int:
        n = C.c_uint64(0)
        _check(self.ctx._lib.mcaat_counts_info(self.h, C.byref(n)))
        return n.value

    def histogram(self, bits: int) -> np.ndarray:
        h = np.zeros(1 << bits, dtype=np.uint64)
        _check(self.ctx._lib.mcaat_counts_histogram(self.h, bits, _ptr(h, _u64p)))
        return h

    def partition(self, splits: np.ndarray, keys_dev: int, counts_dev: int, cap: int) -> np.ndarray:
        """Owner-major oriented (BOSS key, count) pairs into device memory; returns sizes."""
        splits = np.ascontiguousarray(splits, dtype=np.uint64)
        sizes = np.zeros(len(splits) + 1, dtype=np.uint64)
        sp = _ptr(splits, _u64p) if len(splits) else None
        _check(self.ctx._lib.mcaat_counts_partition(self.h, len(splits) + 1, sp, _ptr(sizes, _u64p),
                                                    C.c_void_p(keys_dev), C.c_void_p(counts_dev), cap))
        return sizes

    def free(self) -> None:
        if self.h:
            self.ctx._lib.mcaat_counts_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def edges_reduce(ctx: Context, k: int, keys_dev: int, counts_dev: int, n: int, keys_out_dev: int,
                 mult_out_dev: int) -> int:
    """Sort received (BOSS key, count) pairs and sum equal keys (device memory); returns #unique."""
    out = C.c_uint64(0)
    _check(ctx._lib.mcaat_edges_reduce(ctx.h, k, C.c_void_p(keys_dev), C.c_void_p(counts_dev), n,
                                       C.c_void_p(keys_out_dev), C.c_void_p(mult_out_dev), C.byref(out)))
    return out.value


@dataclass
class CfParams:
    threshold_multiplicity: int = 20
    low_abundance: bool = True
    cycle_max_length: int = 77
    cycle_min_length: int = 27
    cluster_bound: int = 500
    step_cap: int = 10_000_000

    def to_c(self) -> _CfParams:
        return _CfParams(self.threshold_multiplicity, int(self.low_abundance), self.cycle_max_length,
                         self.cycle_min_length, self.cluster_bound, self.step_cap)


@dataclass
class CycleResult:
    """CycleFinder::results in commit order: [(start, [cycle, ...]), ...]."""

    entries: List[Tuple[int, List[List[int]]]] = field(default_factory=list)
    stats: List[int] = field(default_factory=list)
    candidates: List[int] = field(default_factory=list)
    buckets: List[int] = field(default_factory=list)


@dataclass
class MappedReads:
    """Relevant reads (reads.cpp:88-130): read i = ids[offsets[i]:offsets[i+1]]."""

    ids: np.ndarray
    offsets: np.ndarray
    records: np.ndarray

    def __len__(self) -> int:
        return len(self.offsets) - 1

    def read(self, i: int) -> List[int]:
        return self.ids[self.offsets[i]:self.offsets[i + 1]].tolist()


class Graph:
    """Device-resident SDBG (mcaat_graph)."""

    def __init__(self, ctx: Context, h):
        self.ctx = ctx
        self.h = h

    @classmethod
    def build(cls, ctx: Context, reads: Reads, k: int) -> "Graph":
        h = C.c_void_p()
        _check(ctx._lib.mcaat_build_graph(ctx.h, reads.h, k, C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def build_sharded(cls, ctx: Context, comm: Comm, reads: Reads, k: int) -> "Graph":
        """The graph of every rank's reads (mcaat_build_graph_sharded); each rank passes its own."""
        h = C.c_void_p()
        _check(ctx._lib.mcaat_build_graph_sharded(ctx.h, comm.h, reads.h, k, C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_sorted(cls, ctx: Context, k: int, keys_dev: int, mult_dev: int, D: int) -> "Graph":
        """Graph from ascending unique BOSS keys and multiplicities in device memory."""
        h = C.c_void_p()
        _check(ctx._lib.mcaat_graph_from_sorted(ctx.h, k, C.c_void_p(keys_dev), C.c_void_p(mult_dev), D, C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def load(cls, ctx: Context, path: str) -> "Graph":
        """Graph saved by Graph.save (mcaat_graph_load)."""
        h = C.c_void_p()
        _check(ctx._lib.mcaat_graph_load(ctx.h, path.encode(), C.byref(h)))
        return cls(ctx, h)

    def save(self, path: str) -> None:
        _check(self.ctx._lib.mcaat_graph_save(self.h, path.encode()))

    def info(self) -> Tuple[int, int]:
        k = C.c_int(0)
        d = C.c_uint64(0)
        _check(self.ctx._lib.mcaat_graph_info(self.h, C.byref(k), C.byref(d)))
        return k.value, d.value

    @property
    def size(self) -> int:
        return self.info()[1]

    def shard_info(self) -> Tuple[bool, int, int]:
        """(sharded, first id, edges held here) — mcaat_graph_shard_info."""
        sh = C.c_int(0)
        a, n = C.c_uint64(0), C.c_uint64(0)
        _check(self.ctx._lib.mcaat_graph_shard_info(self.h, C.byref(sh), C.byref(a), C.byref(n)))
        return bool(sh.value), a.value, n.value

    def unshard(self, comm: "Comm") -> None:
        """Gather a sharded graph on every rank (collective; mcaat_graph_unshard)."""
        _check(self.ctx._lib.mcaat_graph_unshard(self.h, comm.h))

    def download(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        _, d = self.info()
        keys = np.zeros(max(d, 1), dtype=np.uint64)
        mult = np.zeros(max(d, 1), dtype=np.uint16)
        valid = np.zeros(max(d, 1), dtype=np.uint8)
        _check(self.ctx._lib.mcaat_graph_download(self.h, _ptr(keys, _u64p), _ptr(mult, _u16p), _ptr(valid, _u8p)))
        return keys[:d], mult[:d], valid[:d]

    def download_range(self, first: int, count: int, keys=True, mult=True, valid=False):
        """(keys, mult, valid) of edges [first, first+count); None for the parts not asked for."""
        kk = np.zeros(max(count, 1), dtype=np.uint64) if keys else None
        mm = np.zeros(max(count, 1), dtype=np.uint16) if mult else None
        vv = np.zeros(max(count, 1), dtype=np.uint8) if valid else None
        _check(self.ctx._lib.mcaat_graph_download_range(
            self.h, first, count, _ptr(kk, _u64p) if keys else None, _ptr(mm, _u16p) if mult else None,
            _ptr(vv, _u8p) if valid else None))
        return (kk[:count] if keys else None, mm[:count] if mult else None, vv[:count] if valid else None)

    def neighbors(self, ids: np.ndarray, incoming: bool = False) -> Tuple[np.ndarray, np.ndarray]:
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        out = np.zeros(4 * max(ids.size, 1), dtype=np.uint64)
        cnt = np.zeros(max(ids.size, 1), dtype=np.int32)
        _check(self.ctx._lib.mcaat_graph_neighbors(self.h, _ptr(ids, _u64p), ids.size, int(incoming),
                                                   _ptr(out, _u64p), _ptr(cnt, _i32p)))
        return out[: 4 * ids.size].reshape(-1, 4), cnt[: ids.size]

    def gather(self, ids: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """(keys, mult) of the given edge ids (mcaat_graph_gather)."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        kk = np.zeros(max(ids.size, 1), dtype=np.uint64)
        mm = np.zeros(max(ids.size, 1), dtype=np.uint16)
        _check(self.ctx._lib.mcaat_graph_gather(self.h, _ptr(ids, _u64p), ids.size, _ptr(kk, _u64p), _ptr(mm, _u16p)))
        return kk[: ids.size], mm[: ids.size]

    def succinct_check(self, check: bool = True) -> dict:
        """The succinct (BOSS) view of this graph, built, checked against the arrays and timed
        beside them (mcaat_graph_succinct_check)."""
        out = np.zeros(8, dtype=np.uint64)
        ms = (C.c_double * 6)()
        _check(self.ctx._lib.mcaat_graph_succinct_check(self.h, int(check), _ptr(out, _u64p), ms))
        o = [int(x) for x in out]
        return {"view_bytes": o[0], "array_bytes": o[1], "out_mismatch": o[2], "in_mismatch": o[3], "nodes": o[4],
                "sinks": o[5], "outdeg_sum": o[6], "indeg_sum": o[7], "build_ms": ms[0], "outdeg_info_ms": ms[1],
                "outdeg_sv_ms": ms[2], "indeg_info_ms": ms[3], "indeg_sv_ms": ms[4], "outdeg_sv_stream_ms": ms[5]}

    def keep_region(self, seeds: np.ndarray, hops: int) -> None:
        """valid &= seeds grown by `hops` rounds over valid neighbours (mcaat_graph_keep_region)."""
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        _check(self.ctx._lib.mcaat_graph_keep_region(self.h, _ptr(seeds, _u64p), seeds.size, hops))

    def valid_subgraph(self):
        """(ids, nbr[n, 4], counts): valid edges ascending, out-neighbours as positions in ids."""
        n = C.c_uint64(0)
        _check(self.ctx._lib.mcaat_graph_valid_subgraph(self.h, C.byref(n), None, None, None))
        ids = np.zeros(max(n.value, 1), dtype=np.uint64)
        nbr = np.zeros(4 * max(n.value, 1), dtype=np.uint32)
        cnt = np.zeros(max(n.value, 1), dtype=np.uint8)
        if n.value:
            _check(self.ctx._lib.mcaat_graph_valid_subgraph(self.h, C.byref(n), _ptr(ids, _u64p),
                                                            nbr.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                            _ptr(cnt, _u8p)))
        return ids[: n.value], nbr.reshape(-1, 4)[: n.value], cnt[: n.value]

    def keep_only(self, ids: np.ndarray) -> None:
        """valid &= {ids} (keep_crispr_regions_extended_by_k, spacer_ordering.cpp:129-137)."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        _check(self.ctx._lib.mcaat_graph_keep_only(self.h, _ptr(ids, _u64p), ids.size))

    def map_reads(self, reads: "Reads", cycle_nodes: np.ndarray, max_batch_ids: int = 0) -> "MappedReads":
        """get_reads (reads.cpp:88-130) on the GPU: relevant reads as node-id chains."""
        nodes = np.ascontiguousarray(cycle_nodes, dtype=np.uint64)
        h = C.c_void_p()
        lib = self.ctx._lib
        _check(lib.mcaat_map_reads(self.h, reads.h, _ptr(nodes, _u64p), nodes.size, max_batch_ids, C.byref(h)))
        try:
            n = C.c_uint64(0)
            ip, op, rp = _u64p(), _u64p(), _u64p()
            _check(lib.mcaat_mapped_get(h, C.byref(n), C.byref(ip), C.byref(op), C.byref(rp)))
            offs = np.ctypeslib.as_array(op, shape=(n.value + 1,)).copy()
            ids = np.ctypeslib.as_array(ip, shape=(int(offs[-1]),)).copy() if offs[-1] else np.zeros(0, np.uint64)
            recs = np.ctypeslib.as_array(rp, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint64)
            return MappedReads(ids=ids, offsets=offs, records=recs)
        finally:
            lib.mcaat_mapped_free(h)

    def set_valid(self, ids: np.ndarray, valid: bool) -> None:
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        _check(self.ctx._lib.mcaat_graph_set_valid(self.h, _ptr(ids, _u64p), ids.size, int(valid)))

    def cycle_finder(self, params: Optional[CfParams] = None, as_arrays: bool = False,
                     comm: Optional[Comm] = None) -> CycleResult:
        """CycleFinder results in the reference's commit order. as_arrays: each entry is
        (start, (flat node ids, cycle offsets)) as numpy copies instead of Python lists.
        comm: the searches are split over the ranks that each hold this graph (same results)."""
        p = (params or CfParams()).to_c()
        h = C.c_void_p()
        lib = self.ctx._lib
        if comm is not None:
            _check(lib.mcaat_cycle_finder_comm(self.h, comm.h, C.byref(p), C.byref(h)))
        else:
            _check(lib.mcaat_cycle_finder(self.h, C.byref(p), C.byref(h)))
        try:
            res = CycleResult()
            n = C.c_size_t(0)
            _check(lib.mcaat_cycles_count(h, C.byref(n)))
            if as_arrays:  # one bulk copy (mcaat_cycles_export), then per-entry views
                sz = np.zeros(3, dtype=np.uint64)
                _check(lib.mcaat_cycles_export(h, _ptr(sz, _u64p), None, None, None, None))
                ne, nc_all, nn = (int(x) for x in sz)
                starts = np.zeros(max(ne, 1), dtype=np.uint64)
                eoff = np.zeros(ne + 1, dtype=np.uint64)
                coff = np.zeros(nc_all + 1, dtype=np.uint64)
                nodes = np.zeros(max(nn, 1), dtype=np.uint64)
                _check(lib.mcaat_cycles_export(h, _ptr(sz, _u64p), _ptr(starts, _u64p), _ptr(eoff, _u64p),
                                               _ptr(coff, _u64p), _ptr(nodes, _u64p)))
                for i in range(ne):
                    c0, c1 = int(eoff[i]), int(eoff[i + 1])
                    offs_a = coff[c0:c1 + 1] - coff[c0]
                    flat_a = nodes[int(coff[c0]):int(coff[c1])]
                    res.entries.append((int(starts[i]), (flat_a, offs_a)))
            for i in range(0 if as_arrays else n.value):
                s = C.c_uint64(0)
                fl = _u64p()
                of = _u64p()
                nc = C.c_size_t(0)
                _check(lib.mcaat_cycles_get(h, i, C.byref(s), C.byref(fl), C.byref(of), C.byref(nc)))
                offs = np.ctypeslib.as_array(of, shape=(nc.value + 1,)).tolist()
                flat = np.ctypeslib.as_array(fl, shape=(max(offs[-1], 1),))[: offs[-1]].tolist() if offs[-1] else []
                cycles = [flat[offs[j]:offs[j + 1]] for j in range(nc.value)]
                res.entries.append((s.value, cycles))
            st = (C.c_uint64 * 8)()
            _check(lib.mcaat_cycles_stats(h, st))
            res.stats = list(st)
            nca = C.c_size_t(0)
            ip = _u64p()
            bp = _i32p()
            _check(lib.mcaat_cycles_candidates(h, C.byref(nca), C.byref(ip), C.byref(bp)))
            if as_arrays:
                res.candidates = np.ctypeslib.as_array(ip, shape=(nca.value,)).copy() if nca.value else np.zeros(0, np.uint64)
                res.buckets = np.ctypeslib.as_array(bp, shape=(nca.value,)).copy() if nca.value else np.zeros(0, np.int32)
            else:
                res.candidates = [ip[j] for j in range(nca.value)]
                res.buckets = [bp[j] for j in range(nca.value)]
            return res
        finally:
            lib.mcaat_cycles_free(h)

    def free(self) -> None:
        if self.h:
            self.ctx._lib.mcaat_graph_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
