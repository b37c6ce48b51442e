"""Sharded build check (tests/test_shard.py): run under torch.distributed.run.

CPU (--oracle): every rank counts its slice with the oracle and runs the sharded
orchestration over gloo; rank 0 compares the gathered edge array with the single-process
oracle graph. GPU: every rank counts its slice on the GPU (several ranks may share one
GPU; gloo stages the tensors through host memory, nccl runs over RCCL), and rank 0
compares the sharded graph and its CycleFinder results with the single-process build.
Prints one line "SHARD_OK <D>" on success.
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import mcaat_amd as M  # noqa: E402
from mcaat_amd import shard  # noqa: E402


def spec_of(n_reads: int) -> M.SynthSpec:
    return M.SynthSpec(seed=11, n_genomes=3, genome_len=40_000, arrays_per_genome=1, spacers_per_array=10,
                       repeat_len_min=30, repeat_len_max=34, spacer_len_min=30, spacer_len_max=34, read_len=150,
                       n_reads=n_reads, error_rate=2e-3)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--reads", type=int, default=30_000)
    ap.add_argument("--k", type=int, default=27)
    ap.add_argument("--backend", default="gloo")
    args = ap.parse_args()
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    spec = spec_of(args.reads)
    first = rank * spec.n_reads // world
    count = (rank + 1) * spec.n_reads // world - first
    if args.oracle:
        import oracle as O
        from shard_oracle import OracleOps

        dist.init_process_group("gloo")
        packed, offs = M.synth_host(spec)
        keys, mult = shard.sharded_build(OracleOps(args.k), (packed, offs[first:first + count + 1]))
        if rank == 0:
            ek, em = O.OGraph.build(packed, offs, args.k).arrays()
            assert np.array_equal(keys, ek), "sharded keys differ from the single-process graph"
            assert np.array_equal(mult, em), "sharded multiplicities differ"
            print("SHARD_OK", len(keys), flush=True)
        dist.destroy_process_group()
        return 0

    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group(args.backend)
    ctx = M.Context(dev)
    reads = M.Reads.synth_range(ctx, spec, first, count)
    g = shard.sharded_build(shard.DeviceOps(ctx, args.k), reads)
    keys, mult, _ = g.download()
    res = g.cycle_finder(M.CfParams())
    if rank == 0:
        full = M.Reads.synth(ctx, spec)
        g1 = M.Graph.build(ctx, full, args.k)
        k1, m1, _ = g1.download()
        assert np.array_equal(keys, k1), "sharded keys differ from the single-GPU graph"
        assert np.array_equal(mult, m1), "sharded multiplicities differ"
        r1 = g1.cycle_finder(M.CfParams())
        assert res.entries == r1.entries and res.stats == r1.stats, "CycleFinder results differ"
        print("SHARD_OK", len(keys), len(res.entries), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
