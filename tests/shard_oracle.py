"""TEST INFRASTRUCTURE — CPU restatement of the per-rank pieces of the sharded build
(mcaat_amd.shard.DeviceOps's interface), on the oracle's counts. Lets the sharded
orchestration (histogram all-reduce, owner ranges, all-to-all, owner reduce, all-gather)
run on gloo without a GPU and be compared with the single-process oracle graph."""
from __future__ import annotations

import numpy as np
import torch

import oracle as O

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mask(n: int) -> np.uint64:
    return M64 if n >= 64 else np.uint64((1 << n) - 1)


def rev2_64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    for s, m in ((2, 0x3333333333333333), (4, 0x0F0F0F0F0F0F0F0F), (8, 0x00FF00FF00FF00FF),
                 (16, 0x0000FFFF0000FFFF)):
        m = np.uint64(m)
        s = np.uint64(s)
        x = ((x >> s) & m) | ((x & m) << s)
    return (x >> np.uint64(32)) | (x << np.uint64(32))


def oriented(keys: np.ndarray, cnt: np.ndarray, k: int):
    """BOSS keys and partial counts of both orientations (palindromes: one, twice the count)."""
    E = k + 1
    a = keys.astype(np.uint64)
    b = (rev2_64(a) >> np.uint64(64 - 2 * E)) ^ _mask(2 * E)

    def boss(x):
        return ((x & _mask(2 * k)) << np.uint64(2)) | (x >> np.uint64(2 * k))

    pal = a == b
    K = np.concatenate([boss(a), boss(b[~pal])])
    c = np.concatenate([np.where(pal, 2 * cnt.astype(np.int64), cnt.astype(np.int64)), cnt[~pal].astype(np.int64)])
    return K, c


class OracleOps:
    device = torch.device("cpu")

    def __init__(self, k: int):
        self.k = k

    def count(self, reads):
        packed, offsets = reads
        return O.count_canonical(packed, offsets, self.k)

    def histogram(self, counts, bits: int) -> np.ndarray:
        K, _ = oriented(counts[0], counts[1], self.k)
        return np.bincount((K >> np.uint64(2 * (self.k + 1) - bits)).astype(np.int64),
                           minlength=1 << bits).astype(np.uint64)

    def partition(self, counts, splits: np.ndarray):
        K, c = oriented(counts[0], counts[1], self.k)
        owner = np.searchsorted(splits, K, side="right")
        order = np.argsort(owner, kind="stable")
        sizes = np.bincount(owner, minlength=len(splits) + 1).astype(np.uint64)
        return (torch.from_numpy(K[order].view(np.int64).copy()), torch.from_numpy(c[order].astype(np.int32)), sizes)

    def release(self, counts) -> None:
        pass

    def reduce(self, keys: torch.Tensor, cnt: torch.Tensor):
        K = keys.numpy().view(np.uint64)
        u, inv = np.unique(K, return_inverse=True)
        s = np.bincount(inv, weights=cnt.numpy().astype(np.float64), minlength=len(u)).astype(np.int64)
        m = np.minimum(s, 65535).astype(np.uint16)
        return torch.from_numpy(u.view(np.int64).copy()), torch.from_numpy(m.view(np.int16).copy())

    def build(self, keys: torch.Tensor, mult: torch.Tensor):
        return keys.numpy().view(np.uint64).copy(), mult.numpy().view(np.uint16).copy()
