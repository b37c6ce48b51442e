"""Hash-range sharded graph build, one process per GPU.

Replaces the single-process counting + BOSS build (MEGAHIT Read2SdbgS2::Run driven from
sdbg_build.cpp:171-187) when the reads of one dataset are split over ranks:

1. every rank counts its reads locally (`mcaat_count_local`; LDS pre-aggregation divides
   the exchanged volume by the local coverage);
2. the ranks sum a histogram of the top bits of the oriented edges' BOSS keys and cut it
   into `world` owner ranges of equal weight (contiguous in BOSS order);
3. each rank groups its oriented (BOSS key, partial count) pairs by owner and the ranks
   exchange them with one all-to-all (RCCL over xGMI with the "nccl" backend);
4. each owner sorts its pairs and sums equal keys (`mcaat_edges_reduce`), which gives
   exactly the single-GPU multiplicities of its range;
5. an all-gather in rank order concatenates the ranges into the single-GPU edge array
   (edge ids bit-identical to one GPU), and every rank builds the adjacency words and runs
   CycleFinder on the replicated graph (≈26 B/edge, a fraction of 288 GB).

The collectives run through torch.distributed on torch-allocated device tensors; with
the "gloo" backend the same tensors are staged through host memory (CPU tests, or
several ranks sharing one GPU). `ops` supplies the per-rank pieces: `DeviceOps` is the
HIP library; tests plug in a CPU restatement with the same interface.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from .lib import Context, Counts, Graph, Reads, edges_reduce

HIST_BITS = 12


def choose_splits(hist: np.ndarray, world: int, key_bits: int) -> np.ndarray:
    """world-1 ascending BOSS-key split points at histogram-bin edges with equal weight.

    Owner o takes keys in [splits[o-1], splits[o]) (splits[-1] = 0, splits[world-1] = inf).
    """
    nb = len(hist)
    bits = nb.bit_length() - 1
    assert 1 << bits == nb, "histogram length must be a power of two"
    shift = key_bits - bits
    cum = np.cumsum(hist.astype(np.float64))
    total = cum[-1] if nb else 0.0
    out: List[int] = []
    prev = 0
    for o in range(1, world):
        b = int(np.searchsorted(cum, total * o / world, side="left")) + 1 if total > 0 else nb
        b = min(max(b, prev), nb)
        out.append(b << shift)
        prev = b
    return np.array(out, dtype=np.uint64)


def _comm_device(group) -> torch.device:
    if dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


class DeviceOps:
    """Per-rank pieces on the GPU (libmcaat_gpu.so), data in torch-allocated device memory.

    Every library call is host-synchronous on the library's stream; torch's stream is
    synchronised before the library reads tensors written by torch/RCCL.
    """

    def __init__(self, ctx: Context, k: int):
        self.ctx = ctx
        self.k = k
        self.device = torch.device("cuda", torch.cuda.current_device())

    def count(self, reads: Reads) -> Counts:
        return Counts.count(self.ctx, reads, self.k)

    def histogram(self, counts: Counts, bits: int) -> np.ndarray:
        return counts.histogram(bits)

    def partition(self, counts: Counts, splits: np.ndarray):
        cap = max(1, 2 * counts.n)
        keys = torch.empty(cap, dtype=torch.int64, device=self.device)
        cnt = torch.empty(cap, dtype=torch.int32, device=self.device)
        torch.cuda.synchronize()
        sizes = counts.partition(splits, keys.data_ptr(), cnt.data_ptr(), cap)
        n = int(sizes.sum())
        return keys[:n], cnt[:n], sizes

    def release(self, counts: Counts) -> None:
        counts.free()

    def reduce(self, keys: torch.Tensor, cnt: torch.Tensor):
        n = keys.numel()
        ko = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        mo = torch.empty(max(n, 1), dtype=torch.int16, device=self.device)
        torch.cuda.synchronize()
        u = edges_reduce(self.ctx, self.k, keys.data_ptr(), cnt.data_ptr(), n, ko.data_ptr(), mo.data_ptr())
        return ko[:u], mo[:u]

    def build(self, keys: torch.Tensor, mult: torch.Tensor) -> Graph:
        torch.cuda.synchronize()
        return Graph.from_sorted(self.ctx, self.k, keys.data_ptr(), mult.data_ptr(), keys.numel())


def sharded_build(ops, reads, group=None, hist_bits: int = HIST_BITS, times: Optional[Dict[str, float]] = None):
    """Build the graph of the reads of all ranks of `group` (each passes its own slice)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cdev = _comm_device(group)
    t = [time.perf_counter()]

    def mark(name):
        if times is not None:
            now = time.perf_counter()
            times[name] = times.get(name, 0.0) + (now - t[0]) * 1e3
            t[0] = now

    counts = ops.count(reads)
    mark("shard_count")
    hist = ops.histogram(counts, hist_bits)
    h = torch.from_numpy(hist.view(np.int64).copy()).to(cdev)
    dist.all_reduce(h, group=group)
    splits = choose_splits(h.cpu().numpy().view(np.uint64), world, 2 * (ops.k + 1))
    keys, cnt, sizes = ops.partition(counts, splits)
    ops.release(counts)
    mark("shard_partition")

    # exchange: sizes, then keys and partial counts (one all-to-all each)
    send = torch.from_numpy(sizes.astype(np.int64)).to(cdev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    in_sizes = [int(x) for x in sizes]
    out_sizes = [int(x) for x in recv.cpu()]
    rk = torch.empty(sum(out_sizes), dtype=torch.int64, device=cdev)
    rc = torch.empty(sum(out_sizes), dtype=torch.int32, device=cdev)
    dist.all_to_all_single(rk, keys.to(cdev), out_sizes, in_sizes, group=group)
    dist.all_to_all_single(rc, cnt.to(cdev), out_sizes, in_sizes, group=group)
    del keys, cnt
    mark("shard_all_to_all")

    uk, um = ops.reduce(rk.to(ops.device), rc.to(ops.device))
    del rk, rc
    mark("shard_reduce")

    # all-gather the owners' ranges in rank order (mult as int32: RCCL has no int16)
    n_loc = torch.tensor([uk.numel()], dtype=torch.int64, device=cdev)
    ns_t = [torch.empty_like(n_loc) for _ in range(world)]
    dist.all_gather(ns_t, n_loc, group=group)
    ns = [int(x.item()) for x in ns_t]
    mx = max(max(ns), 1)
    pk = torch.zeros(mx, dtype=torch.int64, device=cdev)
    pm = torch.zeros(mx, dtype=torch.int32, device=cdev)
    pk[: ns[rank]] = uk.to(cdev)
    pm[: ns[rank]] = um.to(cdev).to(torch.int32)
    gk = [torch.empty(mx, dtype=torch.int64, device=cdev) for _ in range(world)]
    gm = [torch.empty(mx, dtype=torch.int32, device=cdev) for _ in range(world)]
    dist.all_gather(gk, pk, group=group)
    dist.all_gather(gm, pm, group=group)
    full_k = torch.cat([gk[r][: ns[r]] for r in range(world)]).to(ops.device)
    full_m = torch.cat([gm[r][: ns[r]] for r in range(world)]).to(torch.int16).to(ops.device)
    del gk, gm, pk, pm
    mark("shard_all_gather")
    g = ops.build(full_k, full_m)
    mark("shard_build")
    return g
