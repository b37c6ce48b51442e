"""Shared helpers for the parity tests (pure Python/numpy; no product code)."""
import numpy as np

CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def pack_reads(seqs):
    """list of ACGT strings -> (packed words LSB-first, offsets) in the library layout."""
    total = sum(len(s) for s in seqs)
    words = np.zeros((total + 31) // 32 + 1, dtype=np.uint64)
    offs = [0]
    j = 0
    for s in seqs:
        for ch in s:
            words[j >> 5] |= np.uint64(CODE[ch]) << np.uint64(2 * (j & 31))
            j += 1
        offs.append(j)
    return words[: (total + 31) // 32], np.array(offs, dtype=np.uint64)


def unpack_read(packed, a, b):
    out = []
    for j in range(a, b):
        out.append("ACGT"[(int(packed[j >> 5]) >> (2 * (j & 31))) & 3])
    return "".join(out)


def rc(s):
    return s[::-1].translate(str.maketrans("ACGT", "TGCA"))


def lsb_value(s):
    return sum(CODE[c] << (2 * i) for i, c in enumerate(s))


def boss_key(s, k):
    """BOSS key of an edge string s (len k+1): colex label then W."""
    lsb = lsb_value(s)
    return ((lsb & ((1 << (2 * k)) - 1)) << 2) | (lsb >> (2 * k))


def brute_graph(seqs, k):
    """Pure-Python restatement of the SDBG conventions for small inputs:
    returns (sorted edge strings, {edge: mult})."""
    occ = {}
    E = k + 1
    for s in seqs:
        for i in range(len(s) - E + 1):
            e = s[i:i + E]
            occ[e] = occ.get(e, 0) + 1
    mult = {}
    for e, c in occ.items():
        for x in (e, rc(e)):
            mult[x] = 0
    for e in list(mult):
        r = rc(e)
        m = occ.get(e, 0) + (occ.get(r, 0) if r != e else occ.get(e, 0))
        mult[e] = min(m, 65535)
    edges = sorted(mult, key=lambda x: boss_key(x, k))
    return edges, mult


def brute_neighbors(edges, k):
    """outgoing (descending id) and incoming (ascending id) edge ids per edge."""
    index = {e: i for i, e in enumerate(edges)}
    by_label = {}
    for i, e in enumerate(edges):
        by_label.setdefault(e[:k], []).append(i)
    out, inc = [], []
    for e in edges:
        tgt = e[1:]
        out.append(sorted(by_label.get(tgt, []), reverse=True))
        preds = [index[x + e[:k]] for x in "ACGT" if (x + e[:k]) in index]
        inc.append(sorted(preds))
    return out, inc


class HipBuffer:
    """A device buffer from the HIP runtime libmcaat_gpu.so itself links (libamdhip64), for tests
    that hand device pointers to the C ABI. (torch ships its own HIP runtime; two runtimes in one
    process do not reliably share the device, so tests do not mix torch in.)"""

    _hip = None

    @classmethod
    def hip(cls):
        if cls._hip is None:
            import ctypes

            import mcaat_amd as M

            M.load_library()  # the runtime it links is then in the process: reuse that very file
            path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
            cls._hip = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        return cls._hip

    def __init__(self, arr: np.ndarray):
        import ctypes

        arr = np.ascontiguousarray(arr)
        h = self.hip()
        self.ptr = ctypes.c_void_p()
        assert h.hipMalloc(ctypes.byref(self.ptr), ctypes.c_size_t(max(arr.nbytes, 8))) == 0
        assert h.hipMemcpy(self.ptr, arr.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(arr.nbytes), 1) == 0
        assert h.hipDeviceSynchronize() == 0

    @property
    def addr(self) -> int:
        return int(self.ptr.value)

    def to_numpy(self, dtype, n: int) -> np.ndarray:
        """The first n elements of the buffer, copied to the host."""
        import ctypes

        out = np.zeros(max(n, 1), dtype=dtype)
        h = self.hip()
        assert h.hipDeviceSynchronize() == 0
        assert h.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), self.ptr, ctypes.c_size_t(out.itemsize * n), 2) == 0
        return out[:n]

    def __del__(self):
        if getattr(self, "ptr", None) is not None and self.ptr.value:
            self.hip().hipFree(self.ptr)
            self.ptr = None
