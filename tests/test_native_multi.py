"""Native multi-GPU path (include/mcaat_gpu.h "multi-GPU, native"): communicators, the
sharded build and CycleFinder split over ranks, FASTQ parts.

CPU: the shared-memory communicator's host collectives between processes (no GPU).
GPU: ranks sharing the one GPU of the box over the shared-memory transport, and RCCL with
one rank, against the single-GPU graph and CycleFinder results."""
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mcaat_amd as M  # noqa: E402

_HOST_RANK = r"""
import sys, numpy as np
sys.path.insert(0, {root!r})
import mcaat_amd as M
world, rank, name = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
c = M.Comm.shm(None, world, rank, name, 4096)   # 4 KiB slots: large messages move in rounds
assert (c.world, c.rank) == (world, rank)
for rnd in range(3):
    rng = np.random.default_rng(100 * rnd + rank)
    n = [0, 5000, 13, 20000][(rank + rnd) % 4]
    mine = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
    got = c.allgather_bytes(mine)
    for r in range(world):
        rr = np.random.default_rng(100 * rnd + r)
        nr = [0, 5000, 13, 20000][(r + rnd) % 4]
        assert got[r] == rr.integers(0, 256, size=nr, dtype=np.uint8).tobytes(), (rnd, r)
    c.barrier()
c.close()
print("HOST_OK", rank)
"""


def _spawn(argv_list, timeout=300):
    procs = [subprocess.Popen(a, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for a in argv_list]
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            outs.append((p.returncode, o, e))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return outs


@pytest.mark.parametrize("world", [2, 3])
def test_shm_comm_host_allgather_between_processes(world):
    name = f"/mcaat_t_{uuid.uuid4().hex[:12]}"
    code = _HOST_RANK.format(root=ROOT)
    outs = _spawn([[sys.executable, "-c", code, str(world), str(r), name] for r in range(world)], timeout=120)
    for rc, o, e in outs:
        assert rc == 0, e[-2000:]
        assert "HOST_OK" in o
    assert not os.path.exists("/dev/shm" + name), "the segment name must be removed once all ranks attached"


_DYING_RANK = r"""
import os, sys, time
sys.path.insert(0, {root!r})
import mcaat_amd as M
world, rank, name = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
c = M.Comm.shm(None, world, rank, name, 4096)
if rank == world - 1:
    os._exit(3)  # leaves without a word, as a rank that failed an allocation does
t0 = time.time()
try:
    c.allgather_bytes(b"x" * 100)
except M.McaatError as e:
    print("PEER_GONE", round(time.time() - t0, 1), str(e))
"""


def test_shm_comm_ends_waits_for_a_rank_that_exited():
    """(round 6) A rank that exits (an allocation failure on a shared GPU) ends the other ranks'
    waits with an error within seconds, instead of at the 900-s time limit."""
    name = f"/mcaat_t_{uuid.uuid4().hex[:12]}"
    code = _DYING_RANK.format(root=ROOT)
    outs = _spawn([[sys.executable, "-c", code, "3", str(r), name] for r in range(3)], timeout=120)
    for r, (rc, o, e) in enumerate(outs[:2]):
        assert rc == 0, e[-2000:]
        # rank 2 left; the other survivor may itself be gone by the time a rank looks (it stops
        # as soon as it sees rank 2 missing), so either exit is the reported one
        assert "PEER_GONE" in o and ("rank 2 exited" in o or f"rank {1 - r} exited" in o), (o, e)
        assert float(o.split()[1]) < 30, o
    assert outs[2][0] == 3


def test_shm_comm_rejects_bad_arguments():
    with pytest.raises(M.McaatError):
        M.Comm.shm(None, 2, 2, "/mcaat_bad")
    with pytest.raises(M.McaatError):
        M.Comm.shm(None, 1, 0, "no_slash")


def test_shm_comm_single_rank_is_identity():
    c = M.Comm.shm(None, 1, 0, f"/mcaat_t_{uuid.uuid4().hex[:12]}")
    assert c.allgather_bytes(b"abc") == [b"abc"]
    c.barrier()
    c.close()


def _ranks(world, comm, extra=(), timeout=600):
    name = f"/mcaat_g_{uuid.uuid4().hex[:12]}"
    uid = f"/tmp/mcaat_uid_{uuid.uuid4().hex[:12]}"
    script = os.path.join(ROOT, "tools", "native_multi_check.py")
    argv = [[sys.executable, script, "--world", str(world), "--rank", str(r), "--comm", comm, "--name", name,
             "--uid-file", uid, *extra] for r in range(world)]
    try:
        return _spawn(argv, timeout=timeout)
    finally:
        if os.path.exists(uid):
            os.unlink(uid)


@pytest.mark.gpu
@pytest.mark.parametrize("world,extra", [(1, ()), (2, ()), (3, ("--window", "16", "--slot", "65536")), (4, ()),
                                         (3, ("--knob", "dist.oriented=1")), (3, ("--knob", "dist.desc=0")),
                                         # round 4's replicated CycleFinder (every rank the whole graph)
                                         (2, ("--knob", "dist.shard_cf=0")), (3, ("--knob", "dist.shard_cf=0")),
                                         # per-shard peel with every unary edge a ruler / sparse rulers,
                                         # adjacency and window exchanges in many small chunks
                                         (2, ("--knob", "dist.ruler_mask=0")), (3, ("--knob", "dist.ruler_mask=1023")),
                                         (3, ("--knob", "dist.adj_chunk=1024", "--knob", "dist.adj_ranges=0")),
                                         # adjacency, filter windows and flags by request / response
                                         # messages (round 5's first form) instead of target ranges
                                         (2, ("--knob", "dist.adj_ranges=0", "--knob", "dist.win_ranges=0")),
                                         (3, ("--knob", "dist.win_ranges=0")),
                                         # (round 6) the region BFS and the FindCycle reach hop by
                                         # hop with host waits (round 5's forms)
                                         (2, ("--knob", "dist.bfs_sync=1")), (3, ("--knob", "dist.bfs_sync=1")),
                                         # (round 6) the device-resident region BFS with blocks and
                                         # frontiers too small: every rank reruns it with larger ones
                                         (3, ("--knob", "dist.bfs_block=64")),
                                         (2, ("--knob", "dist.bfs_block=64", "--knob", "dist.bfs_frontier=1")),
                                         (1, ("--knob", "dist.bfs_frontier=1")),
                                         # (round 6) branch resolution: routed rounds (round 5's
                                         # form) / fixed blocks checked after every round
                                         (3, ("--knob", "dist.res_fixed=0")), (2, ("--knob", "dist.res_batch=1")),
                                         # (round 6) the walk: every round routed / the fixed-block
                                         # tail from the first round on, checked every round
                                         (3, ("--knob", "dist.walk_block=0")),
                                         (3, ("--knob", "dist.walk_block=4194304", "--knob", "dist.walk_batch=1")),
                                         (4, ("--knob", "dist.walk_block=4194304"))])
def test_sharded_build_and_cycle_finder_ranks_share_one_gpu(world, extra):
    """(round 5: per-shard CycleFinder by default) the sharded build + CycleFinder over 1-4 ranks
    sharing the GPU equal the one-GPU path: keys, multiplicities, valid bits after CycleFinder,
    entries, candidates, buckets, stats."""
    outs = _ranks(world, "shm", extra)
    for rc, o, e in outs:
        assert rc == 0, (o[-2000:], e[-3000:])
        assert "NATIVE_MULTI_OK" in o, o


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["pe_err", "low_thr", "c3_sample", "c5_sample"])
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_per_shard_cycle_finder_parity_cases(case, world):
    """ The per-shard CycleFinder on the parity cases (paired-end
    with errors, threshold 2, the C3 and C5 coverage-matched samples) through 1, 2, 4 and 8
    shared-memory ranks (8: C4's partition, denser rulers above two ranks, eight target ranges)
    equals the one-GPU path: valid bitmap, candidates, buckets, entries, stats."""
    outs = _ranks(world, "shm", ("--case", case, "--slot", "0"))
    for rc, o, e in outs:
        assert rc == 0, (o[-2000:], e[-3000:])
        assert "NATIVE_MULTI_OK" in o and "sharded=True" in o, o


_SINGLE_DIGEST = {}


@pytest.mark.gpu
@pytest.mark.timeout(1500)
@pytest.mark.parametrize("config,world", [("c3", 2), ("c3", 8), ("c5", 2)])
def test_full_dataset_shm_ranks_equal_one_gpu(gpu_ctx, tmp_path, config, world):
    """The C4 / C5 data paths at full size: a whole bench dataset through
    mcaat_build_graph_sharded + mcaat_cycle_finder_comm with `world` shared-memory ranks sharing
    the GPU; keys, multiplicities, post-CycleFinder valid bits (order-sensitive checksums) and the
    full CycleFinder results (entries, candidates, buckets, stats) equal the one-GPU path's.
    (c3, 8): C4's 8-way partition at C3 scale (round 6: fits one GPU with 256-slot pass-A
    reservations, ~30 GB per rank); (c5, 2): D = 3.9e9, so one rank holds only ids above 2^31."""
    import json

    gpu_ctx.trim()  # the ranks need the memory this process's arena keeps from earlier tests
    script = os.path.join(ROOT, "tools", "native_multi_check.py")
    if config not in _SINGLE_DIGEST:
        single = str(tmp_path / "single.json")
        (rc, o, e), = _spawn([[sys.executable, script, "--world", "1", "--rank", "0", "--single", "--config", config,
                               "--digest", single]], timeout=900)
        assert rc == 0, (o[-2000:], e[-3000:])
        _SINGLE_DIGEST[config] = json.load(open(single))
    want = _SINGLE_DIGEST[config]
    assert want["D"] > 9e8 and want["cycles"] > 0
    dig = str(tmp_path / "rank{rank}.json")
    outs = _ranks(world, "shm", ("--config", config, "--digest", dig, "--slot", "0"), timeout=1200)
    for rc, o, e in outs:
        assert rc == 0, (o[-2000:], e[-3000:])
        assert "NATIVE_MULTI_DIGEST" in o, o
    for r in range(world):
        got = json.load(open(dig.format(rank=r)))
        for key in ("D", "keys", "mult", "valid", "stats", "results", "entries", "cycles"):
            assert got[key] == want[key], (r, key, got[key], want[key])
        # every rank holds about 1/world of the graph through CycleFinder
        assert got["cf_hbm_GB"]["graph_at_start"] < 1.5 * want["cf_hbm_GB"]["graph_at_start"] / world + 1, got


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [(), ("--knob", "dist.segs_at_one=1")])
def test_rccl_single_rank_matches_one_gpu(extra):
    """RCCL at one rank equals one GPU; with dist.segs_at_one the descriptor exchange runs through
    the RCCL segment all-to-all (its self-copy path) instead of keeping the buckets."""
    outs = _ranks(1, "rccl", extra)
    rc, o, e = outs[0]
    assert rc == 0, (o[-2000:], e[-3000:])
    assert "NATIVE_MULTI_OK" in o


@pytest.mark.parametrize("world", [2, 3, 8, 64])
def test_rccl_segment_schedule_pairs_pieces(world):
    """ The RCCL segment all-to-all's op schedule (comm.hip seg_schedule, the code the
    transport runs), built for every rank of `world` on the host from random segment lists: each
    pair's j-th send piece equals the peer's j-th receive piece, and the pieces tile the segments
    and the output. Multi-rank RCCL itself cannot run on this pool's one-GPU boxes."""
    for seed in range(1, 40):
        rounds = M.Comm.schedule_check(world, seed, 4096)
        assert rounds >= 0
    with pytest.raises(M.McaatError):
        M.Comm.schedule_check(0, 1, 4096)


@pytest.mark.gpu
def test_fastq_parts_compressed_inputs_go_whole_to_part_zero(gpu_ctx, tmp_path):
    import bz2
    import gzip

    r = M.Reads.synth(gpu_ctx, M.SynthSpec(seed=9, n_reads=3000))
    plain = str(tmp_path / "r.fq")
    r.write_fastq(plain, threads=2)
    r.free()
    data = open(plain, "rb").read()
    for name, blob in (("r.fq.gz", gzip.compress(data)), ("r.fq.bz2", bz2.compress(data))):
        p = tmp_path / name
        p.write_bytes(blob)
        whole = M.Reads.from_fastx(gpu_ctx, [plain])
        want = whole.info()
        whole.free()
        parts = [M.Reads.from_fastx_part(gpu_ctx, [str(p)], i, 3) for i in range(3)]
        assert parts[0].info() == want and parts[1].info() == (0, 0) and parts[2].info() == (0, 0)
        for q in parts:
            q.free()


@pytest.mark.gpu
@pytest.mark.parametrize("paired", [False, True])
def test_fastq_parts_partition_the_records(gpu_ctx, tmp_path, paired):
    spec = M.SynthSpec(seed=7, n_reads=7001, paired=paired, error_rate=1e-3)
    r = M.Reads.synth(gpu_ctx, spec)
    p1 = str(tmp_path / "r1.fq")
    r.write_fastq(p1, threads=2)
    r.free()
    files = [p1]
    if paired:  # a second file with other records (reverse-complemented in the mapping view)
        r2 = M.Reads.synth(gpu_ctx, M.SynthSpec(seed=8, n_reads=3333))
        p2 = str(tmp_path / "r2.fq")
        r2.write_fastq(p2, threads=2)
        r2.free()
        files.append(p2)
    whole = M.Reads.from_fastx(gpu_ctx, files)
    wp, wo = whole.download()
    wrp, wro = whole.download_records()
    n_file = [whole.file_records(f) for f in range(len(files))]
    whole.free()
    for n_parts in (2, 3, 5):
        per_file = np.zeros(len(files), dtype=np.int64)
        parts = []
        for part in range(n_parts):
            pr = M.Reads.from_fastx_part(gpu_ctx, files, part, n_parts)
            parts.append(pr)
            per_file += [pr.file_records(f) for f in range(len(files))]
        assert per_file.tolist() == n_file
        # mapping views: per file, the parts' records in part order are the whole file's records
        def view(p, o, lo, hi):  # records [lo, hi): their lengths and their bases
            return np.diff(o[lo:hi + 1].astype(np.int64)), _bases(p, int(o[lo]), int(o[hi]))
        wl = 0
        for f in range(len(files)):
            want_len, want_b = view(wrp, wro, wl, wl + n_file[f])
            wl += n_file[f]
            lens, bases = [], []
            for pr in parts:
                rp, ro = pr.download_records()
                nf = [pr.file_records(x) for x in range(len(files))]
                lo = sum(nf[:f])
                ln, bs = view(rp, ro, lo, lo + nf[f])
                lens.append(ln)
                bases.append(bs)
            assert np.array_equal(np.concatenate(lens), want_len), (n_parts, f)
            assert np.array_equal(np.concatenate(bases), want_b), (n_parts, f)
        n_all = sum(pr.info()[1] for pr in parts)
        assert n_all == int(wo[-1])
        for pr in parts:
            pr.free()


def _bases(packed, a, b):
    idx = np.arange(a, b, dtype=np.uint64)
    return ((packed[(idx >> np.uint64(5)).astype(np.int64)] >> (np.uint64(2) * (idx & np.uint64(31)))) & np.uint64(3))
