"""One rank of a native multi-GPU check (tests/test_native_multi.py starts `world` of these).

Each rank joins a communicator (shm: POSIX shared memory, ranks may share one GPU; rccl:
one GPU per rank, or world 1), builds the graph of its slice of one synthetic dataset with
mcaat_build_graph_sharded, runs mcaat_cycle_finder_comm, and compares graph and results
with the single-GPU path over all the reads (computed by every rank on its own context).

usage: native_multi_check.py --world N --rank R --comm shm|rccl --name /x [--reads N]
       [--window W] [--uid-file F]
       native_multi_check.py ... --config c3 --digest FILE   (a bench config at full size: the
           rank writes checksums of its graph and results instead of comparing in-process)
       native_multi_check.py --single --config c3 --digest FILE   (the one-GPU path's checksums)
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mcaat_amd as M  # noqa: E402


def checksums(g, res) -> dict:
    """Order-sensitive checksums of the graph (keys, multiplicities, valid bits after
    CycleFinder) and the full CycleFinder results; two runs agree iff these agree (up to
    64-bit checksum collisions)."""
    import hashlib

    D = g.size
    ks = ms = vs = 0
    chunk = 1 << 27
    mask = (1 << 64) - 1
    with np.errstate(over="ignore"):
        for a in range(0, D, chunk):
            n = min(chunk, D - a)
            kk, mm, vv = g.download_range(a, n, valid=True)
            idx = np.arange(a, a + n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1)
            ks = (ks + int((kk * idx).sum(dtype=np.uint64))) & mask
            ms = (ms + int((mm.astype(np.uint64) * idx).sum(dtype=np.uint64))) & mask
            vs = (vs + int((vv.astype(np.uint64) * idx).sum(dtype=np.uint64))) & mask
    h = hashlib.sha256(repr((res.entries, list(res.candidates), list(res.buckets))).encode()).hexdigest()
    return {"D": D, "keys": ks, "mult": ms, "valid": vs, "stats": list(res.stats[:6]), "results": h,
            "entries": len(res.entries), "cycles": res.stats[5]}


XR_STAGES = ("build", "tips_filter", "peel", "recount", "candidates", "dls", "find_cycle")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--comm", default="shm", choices=["shm", "rccl"])
    ap.add_argument("--name", default="/mcaat_check")
    ap.add_argument("--reads", type=int, default=30000)
    ap.add_argument("--window", type=int, default=0, help="cf.fc_window knob (small: many rounds)")
    ap.add_argument("--uid-file", default="")
    ap.add_argument("--slot", type=int, default=1 << 20, help="shm staging bytes per rank")
    ap.add_argument("--config", default="", help="a bench config (mcaat_amd/configs.py) at full size")
    ap.add_argument("--digest", default="", help="write checksums here (JSON) instead of comparing")
    ap.add_argument("--single", action="store_true", help="the one-GPU path alone (with --digest)")
    ap.add_argument("--knob", action="append", default=[], help="name=value knob on every rank's context")
    ap.add_argument("--repeat", type=int, default=1, help="--config: sharded builds in a row (stages of the last)")
    ap.add_argument("--case", default="default", choices=["default", "pe_err", "low_thr", "c3_sample", "c5_sample"],
                    help="the dataset of the in-process comparison")
    a = ap.parse_args()

    def make_comm(ctx):
        if a.comm == "shm":
            return M.Comm.shm(ctx, a.world, a.rank, a.name, a.slot)
        if a.rank == 0:
            uid = M.Comm.unique_id()
            tmp = a.uid_file + ".tmp"
            with open(tmp, "wb") as f:
                f.write(uid)
            os.replace(tmp, a.uid_file)
        else:
            t0 = time.time()
            while not os.path.exists(a.uid_file):
                if time.time() - t0 > 120:
                    raise SystemExit("no unique id file")
                time.sleep(0.05)
        with open(a.uid_file, "rb") as f:
            uid = f.read()
        return M.Comm.rccl(ctx, a.world, a.rank, uid)

    if a.config:
        import json

        from mcaat_amd.configs import CONFIGS

        cfg = CONFIGS[a.config]
        spec, k, prm = cfg["spec"], cfg["k"], M.CfParams(threshold_multiplicity=cfg["thr"])
        ctx = M.Context(a.rank % max(1, M.device_count()) if a.comm == "rccl" else 0)
        M.preload(ctx.device)  # stage times without code-object loads
        for kv in a.knob:
            kn, kval = kv.split("=")
            ctx.set_knob(kn, int(kval))
        t0 = time.time()
        if a.single:
            reads = M.Reads.synth(ctx, spec)
            g = M.Graph.build(ctx, reads, k)
            reads.free()
            cf_base = ctx.arena_usage(reset_peak=True)[0]
            res = g.cycle_finder(prm, as_arrays=False)
            cf_stages = {kk: round(vv, 2) for kk, vv in ctx.stage_times().items()}
            cf_mem = (cf_base, ctx.arena_usage()[1])
            comm = None
        else:
            comm = make_comm(ctx)
            first = a.rank * spec.n_reads // a.world
            count = (a.rank + 1) * spec.n_reads // a.world - first
            mine = M.Reads.synth_range(ctx, spec, first, count)
            ctx.arena_usage(reset_peak=True)
            for rep in range(a.repeat):  # stage times of the last build (the first pays allocations)
                if rep:
                    g.free()
                ctx.stage_times()
                g = M.Graph.build_sharded(ctx, comm, mine, k)
                build_stages = {kk: round(vv, 2) for kk, vv in ctx.stage_times().items()}
            build_peak = ctx.arena_usage()[1]  # this rank's device memory peak through the build
            mine.free()
            cf_base = ctx.arena_usage(reset_peak=True)[0]
            res = g.cycle_finder(prm, comm=comm)
            cf_stages = {kk: round(vv, 2) for kk, vv in ctx.stage_times().items()}
            cf_mem = (cf_base, ctx.arena_usage()[1])
            # a per-shard graph is gathered for the checksums (no-op otherwise); the arena's cached
            # chunks go back first (eight ranks sharing one GPU each gather the whole graph)
            ctx.trim()
            comm.barrier()
            g.unshard(comm)
        d = checksums(g, res)
        d["seconds"] = round(time.time() - t0, 1)
        d["cf_stages_ms"] = cf_stages
        # device memory of this process: in use as CycleFinder starts (the graph), its peak during it
        d["cf_hbm_GB"] = {"graph_at_start": round(cf_mem[0] / 1e9, 2), "peak": round(cf_mem[1] / 1e9, 2)}
        if not a.single:
            d["build_stages_ms"] = build_stages
            d["build_hbm_peak_GB"] = round(build_peak / 1e9, 2)
            # collectives per stage on this rank (each a bulk-synchronous exchange round)
            d["collectives"] = {st: ctx.kernel_timing("xr_" + st)[1] for st in XR_STAGES}
            # of them the device all-to-alls RCCL leaves queued (the rest wait on the host)
            d["collectives_queued"] = {st: ctx.kernel_timing("xq_" + st)[1] for st in XR_STAGES}
        g.free()
        if comm is not None:
            comm.barrier()
            comm.close()
        ctx.close()
        with open(a.digest.format(rank=a.rank), "w") as f:
            json.dump(d, f)
        print(f"rank {a.rank}: {d}", flush=True)
        print("NATIVE_MULTI_DIGEST", flush=True)
        return 0

    spec = M.SynthSpec(seed=11, n_genomes=3, genome_len=40_000, arrays_per_genome=2, spacers_per_array=10,
                       repeat_len_min=30, repeat_len_max=34, spacer_len_min=30, spacer_len_max=36,
                       n_reads=a.reads, error_rate=2e-3)
    k, thr = 27, 20
    if a.case != "default":  # the parity cases of tests/test_scale_parity.py (CASES, SAMPLES)
        from mcaat_amd.configs import CONFIGS

        spec, k, thr = {
            "pe_err": (M.SynthSpec(seed=7, n_genomes=4, genome_len=20_000, arrays_per_genome=2, spacers_per_array=8,
                                   repeat_len_min=32, repeat_len_max=36, spacer_len_min=30, spacer_len_max=36,
                                   n_reads=24_000, error_rate=0.002, paired=True), 23, 5),
            "low_thr": (M.SynthSpec(seed=11, n_genomes=3, genome_len=15_000, arrays_per_genome=2, spacers_per_array=10,
                                    repeat_len_min=30, repeat_len_max=34, spacer_len_min=30, spacer_len_max=34,
                                    n_reads=12_000, error_rate=0.004), 23, 2),
            "c3_sample": (CONFIGS["c3"]["sample"], 27, 20),
            "c5_sample": (CONFIGS["c5"]["sample"], 27, 2),
        }[a.case]
    dev = a.rank % max(1, M.device_count()) if a.comm == "rccl" else 0
    ctx = M.Context(dev)
    if a.window:
        ctx.set_knob("cf.fc_window", a.window)
    for kv in a.knob:
        kn, kval = kv.split("=")
        ctx.set_knob(kn, int(kval))
    comm = make_comm(ctx)
    assert (comm.world, comm.rank) == (a.world, a.rank)

    first = a.rank * spec.n_reads // a.world
    count = (a.rank + 1) * spec.n_reads // a.world - first
    mine = M.Reads.synth_range(ctx, spec, first, count)
    prm = M.CfParams(threshold_multiplicity=thr)
    g = M.Graph.build_sharded(ctx, comm, mine, k)
    sharded = g.shard_info()[0]
    res = g.cycle_finder(prm, comm=comm)
    g.unshard(comm)
    keys, mult, valid = g.download()
    g.free()
    mine.free()

    whole = M.Reads.synth(ctx, spec)
    g1 = M.Graph.build(ctx, whole, k)
    k1, m1, _ = g1.download()
    r1 = g1.cycle_finder(prm)
    _, _, v1 = g1.download()
    g1.free()
    whole.free()

    ok = np.array_equal(keys, k1) and np.array_equal(mult, m1) and np.array_equal(valid, v1)
    ok = ok and res.entries == r1.entries and res.stats[:6] == r1.stats[:6]
    ok = ok and list(res.candidates) == list(r1.candidates) and list(res.buckets) == list(r1.buckets)
    # every rank holds the same results
    digest = repr((res.entries, res.stats[:6])).encode()
    same = len(set(comm.allgather_bytes(digest))) == 1
    xr = {st: ctx.kernel_timing("xr_" + st)[1] for st in XR_STAGES}
    print(f"rank {a.rank}: collectives {xr}", flush=True)
    print(f"rank {a.rank}: D={len(keys)} (single {len(k1)}) entries={len(res.entries)} cycles={res.stats[5]} "
          f"rounds={res.stats[6]} reruns={res.stats[7]} sharded={sharded} match={ok} ranks_agree={same}", flush=True)
    if not ok:
        print(f"rank {a.rank}: keys {np.array_equal(keys, k1)} mult {np.array_equal(mult, m1)} valid "
              f"{np.array_equal(valid, v1)} ({int((valid != v1).sum())} differ) stats {res.stats[:6]} vs {r1.stats[:6]} "
              f"entries {res.entries == r1.entries} cand {list(res.candidates) == list(r1.candidates)}", flush=True)
    comm.barrier()
    comm.close()
    ctx.close()
    if ok and same:
        print("NATIVE_MULTI_OK", flush=True)
        return 0
    return 1


if __name__ == "__main__":
    sys.exit(main())
