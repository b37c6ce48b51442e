#!/usr/bin/env python3
"""bench.py — k-mers/s through node_counter + sdbg_build + cycle_finder on MI355X.

Metric (BASELINE.json): "k-mers/sec through sdbg_build+cycle_finder, 1B-node graph @ 1/2/4/8 GPUs".
One step = one pass of the hot path over one synthetic metagenome resident in HBM:
reads -> edge counting -> SDBG -> CycleFinder (results ready on the host).
k-mers = N_occ = sum over reads of (L - k) edge occurrences.

Workload (N=1): config C3 — ~300M x 150 bp reads, k=27, threshold_multiplicity=20,
error rate tuned so the SDBG has ~1e9 edges (D).
N>1, default --mode shard (config C4): the SAME C3 dataset is split over
the ranks; each runs pass A of the counter on its slice, the super-k-mer descriptors go to the
owners of their minimizer-hash (L1 bucket) ranges by one all-to-all, owners count them to final
counts, the oriented edges are routed to their BOSS-key-range owners and sorted, an exact-size
all-gather in rank order gives every rank the single-GPU graph, and CycleFinder runs over the
ranks (pruning on every rank, candidate scan by id range, DLS and FindCycle starts dealt
round-robin with one ordered commit). All of it is the library's native path
(mcaat_build_graph_sharded, mcaat_cycle_finder_comm) over an RCCL communicator whose id travels
over torch.distributed (gloo, control plane only); MCAAT_COMM_BACKEND=gloo uses the
shared-memory transport instead (ranks sharing one GPU). Scaling "strong": total work fixed.
--mode replicas: every rank runs its own independent C3-sized sample, no collective on the
data path (scaling "weak").
value = all k-mers processed / max-over-ranks step time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|tiny] [--mode shard|replicas]
       N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import mcaat_amd as M  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
# node_counter kernels timed with HIP events on the library stream (mcaat_kernel_timing)
HOT_KERNELS = ("sk_scatter", "l2_hist", "l2_partition", "lds_count")

from mcaat_amd.configs import CONFIGS  # noqa: E402


def n_occ(spec: M.SynthSpec, k: int) -> int:
    return spec.n_reads * max(0, spec.read_len - k)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads() -> int:
    """Host cores this job may use: OMP_NUM_THREADS (16 on the GPU box), else the affinity set."""
    try:
        return max(1, int(os.environ["OMP_NUM_THREADS"]))
    except (KeyError, ValueError):
        return max(1, len(os.sched_getaffinity(0)))


def _oracle_path(path: str, k: int, thr: int, threads: int) -> tuple:
    """The CPU restatement over the reference's span: FASTQ parse -> count -> SDBG -> CycleFinder."""
    import oracle as O

    t0 = time.perf_counter()
    packed, offs = O.read_fastq(path)
    t1 = time.perf_counter()
    g = O.OGraph.build(packed, offs, k, threads=threads)
    res = g.cycle_finder(threshold_multiplicity=thr, threads=threads)
    t2 = time.perf_counter()
    n_occ_s = int(np.maximum(np.diff(offs.astype(np.int64)) - k, 0).sum())
    return t2 - t0, t1 - t0, n_occ_s, g.size, res["stats"][5]


def cpu_baseline(ctx, cfg: dict, threads: int) -> dict:
    """The oracle (CPU restatement, OpenMP) timed from FASTQ to CycleFinder results, as the
    reference's span (main.cpp:517-536), on a coverage-matched sample of the workload (same
    D/N_occ regime), plus C1 tiny at threads=1 (the reference's deterministic mode)."""
    import tempfile

    out = {"unit": "k-mers/s", "cores": threads, "kind": "port", "cpu": cpu_model()}
    for key, spec, thr_n in (("sample", cfg["sample"], threads), ("c1_threads1", CONFIGS["tiny"]["spec"], 1)):
        r = M.Reads.synth(ctx, spec)
        fd, path = tempfile.mkstemp(suffix=".fq", dir="/tmp")
        os.close(fd)
        try:
            r.write_fastq(path, threads=threads)
            r.free()
            size = os.path.getsize(path)
            dt, parse, kmers, D, cyc = _oracle_path(path, cfg["k"], cfg["thr"], thr_n)
        finally:
            os.unlink(path)
        leg = {"value": kmers / dt, "seconds": round(dt, 3), "fastq_parse_s": round(parse, 3), "kmers": kmers,
               "D": D, "cycles": cyc, "threads": thr_n,
               "sample": f"{spec.n_reads} x {spec.read_len} bp over {spec.n_genomes} x {spec.genome_len} bp "
                         f"(coverage {spec.n_reads * spec.read_len / (spec.n_genomes * spec.genome_len):.0f}x), "
                         f"e={spec.error_rate}, {size / 1e6:.0f} MB FASTQ in /tmp, FASTQ parse -> count -> SDBG -> "
                         f"CycleFinder, D/N_occ={D / max(1, kmers):.4f}"}
        if key == "sample":
            out.update(value=leg["value"], sample=leg["sample"], seconds=leg["seconds"], D=D, kmers=kmers)
            out["fastq_parse_s"] = leg["fastq_parse_s"]
        else:
            out[key] = leg
    return out


def preread(path: str, threads: int) -> None:
    import concurrent.futures as cf

    size = os.path.getsize(path)
    piece = (size + threads - 1) // threads

    def rd(i):
        with open(path, "rb", buffering=0) as f:
            f.seek(i * piece)
            left = max(0, min(piece, size - i * piece))
            while left > 0:
                b = f.read(min(left, 64 << 20))
                if not b:
                    break
                left -= len(b)

    with cf.ThreadPoolExecutor(threads) as ex:
        list(ex.map(rd, range(threads)))


def run_e2e(ctx, reads, cfg: dict, spec, n_kmers: int) -> dict:
    """Writes the resident reads as FASTQ to tmpfs (untimed) and measures the CLI span on it."""
    import shutil

    need = 2 * spec.n_reads * spec.read_len + 7 * spec.n_reads
    if shutil.disk_usage("/dev/shm").free < 1.2 * need:
        return {"error": f"/dev/shm holds less than 1.2 x {need / 1e9:.0f} GB"}
    path = f"/dev/shm/mcaat_bench_{os.getpid()}.fq"
    try:
        t0 = time.perf_counter()
        reads.write_fastq(path, threads=host_threads())
        write_s = time.perf_counter() - t0
        # one untimed sequential read settles the freshly written tmpfs pages: the first read
        # after the write runs at ~14 GB/s, every later one at ~40 GB/s (measured, tools/e2e_probe.py)
        t0 = time.perf_counter()
        preread(path, 8)
        pre_s = time.perf_counter() - t0
        out = measure_e2e(cfg, spec, path, host_threads(), n_kmers)
        out["fastq_write_s"] = round(write_s, 3)
        out["fastq_preread_s"] = round(pre_s, 3)
        return out
    except Exception as e:
        return {"error": str(e)}
    finally:
        if os.path.exists(path):
            os.unlink(path)


def measure_e2e(cfg: dict, spec, fastq: str, threads: int, n_kmers: int) -> dict:
    """The reference's headline T: the mcaat CLI (C++ host over the C ABI) in a fresh process on
    the FASTQ, timed by the CLI itself from SDBGBuild start to CycleFinder end (main.cpp:517-536:
    GPU FASTQ ingest + node_counter + sdbg_build + host SDBG load + CycleFinder)."""
    import re
    import shutil
    import subprocess
    import tempfile

    exe = os.path.join(ROOT, "mcaat_amd", "mcaat")
    work = tempfile.mkdtemp(dir="/tmp")
    try:
        st = os.path.join(work, "settings.txt")
        with open(st, "w") as f:
            f.write(f"kmer_k={cfg['k']}\nthreshold_multiplicity={cfg['thr']}\nthreads={threads}\n")
        t0 = time.perf_counter()
        p = subprocess.run([exe, "--settings", st, "--input-files", fastq, "--output-folder",
                            os.path.join(work, "out")], capture_output=True, text=True, timeout=900)
        wall = time.perf_counter() - t0
        if os.environ.get("MCAAT_E2E_LOG"):  # keep the CLI's own output (per-step timers) for study
            with open(os.environ["MCAAT_E2E_LOG"], "w") as f:
                f.write(p.stdout + "\n---- stderr ----\n" + p.stderr)
        m = re.search(r"TIMING span_s=([0-9.]+) sdbg_build_s=([0-9.]+) build_lib_s=([0-9.]+) cycle_finder_s=([0-9.]+)",
                      p.stdout)
        if p.returncode != 0 or not m:
            return {"error": f"CLI rc={p.returncode}: {(p.stderr or p.stdout)[-400:]}"}
        span, build, lib, cf = (float(x) for x in m.groups())
        # the rest of the wall, from the CLI's own phase timers (main.cpp TIMING_TAIL)
        tail = {}
        mt = re.search(r"TIMING_TAIL (.*)", p.stdout)
        if mt:
            tail = {kv.split("=")[0]: round(float(kv.split("=")[1]), 3) for kv in mt.group(1).split()}
            tail["process_start_and_exit_s"] = round(wall - tail.get("main_s", 0.0), 3)
        for tag in ("TIMING_REGIONS", "TIMING_STEP7", "TIMING_GROW"):  # step 7's own split (array_order.cpp, pipeline_steps.cpp)
            ms = re.search(tag + r" (.*)", p.stdout)
            if ms:
                tail[tag.lower()[7:]] = {kv.split("=")[0]: round(float(kv.split("=")[1]), 3)
                                         for kv in ms.group(1).split() if "=" in kv}
        arrays = os.path.join(work, "out", "CRISPR_Arrays.txt")
        n_arr = None
        recall = None
        if os.path.exists(arrays):
            for line in open(arrays):
                if line.startswith("Number of Systems:"):
                    n_arr = int(line.split(":")[1])
            # every planted array of the synthetic community should be in the report
            from mcaat_amd.truth import parse_crispr_arrays, planted_recall

            rec = planted_recall(parse_crispr_arrays(arrays), M.synth_arrays(spec))
            recall = {kk: rec[kk] for kk in ("planted", "recalled", "recall", "systems")}
        return {
            "value": n_kmers / span, "unit": "k-mers/s", "T_s": round(span, 3),
            "build_lib_s": round(lib, 3), "sdbg_build_s": round(build, 3), "cycle_finder_s": round(cf, 3),
            "fastq_bytes": os.path.getsize(fastq), "fastq_GBps": round(os.path.getsize(fastq) / lib / 1e9, 2),
            "cli_wall_s": round(wall, 3), "cli_phases_s": tail, "crispr_systems": n_arr, "planted_recall": recall,
            "note": "fresh CLI process on a GPU no earlier process of this job used, FASTQ in tmpfs (/dev/shm, "
                    "pages settled by one untimed read); the span excludes process start, HIP runtime init and the "
                    "kernels' code-object load (input check, mcaat_preload) and the downstream steps 6-8 "
                    "(cli_wall_s includes them)",
        }
    finally:
        shutil.rmtree(work, ignore_errors=True)


def _traffic_file(config: str) -> str:
    """The committed PMC summary of this config (tools/traffic_summary.py)."""
    return os.path.join(ROOT, "profiles", f"traffic_{config}.json")


def step_traffic_from_profiles(config: str) -> dict | None:
    """HBM bytes of one profiled step of this config: every kernel's per-launch PMC bytes times
    its launches, the synthetic-read generator excluded; FETCH doubled only for the kernels
    whose reads are wide coalesced streams (corrected), and as counted (raw)."""
    try:
        with open(_traffic_file(config)) as f:
            d = json.load(f)
        # entries without "launches" are the bench's short-name aliases of a k_* entry
        rows = [v for kk, v in d.items() if kk != "k_synth" and "launches" in v]
        return {"corrected": float(sum(v["hbm_bytes_per_launch"] * v["launches"] for v in rows)),
                "raw": float(sum(v.get("hbm_bytes_raw", v["hbm_bytes_per_launch"]) * v["launches"] for v in rows))}
    except Exception:
        return None


def traffic_from_profiles(config: str, kernel: str) -> float | None:
    """HBM bytes per launch of the dominant kernel from this config's PMC summary, if any."""
    try:
        with open(_traffic_file(config)) as f:
            d = json.load(f)
        return float(d[kernel]["hbm_bytes_per_launch"])
    except Exception:
        return None


class _DryContext:
    def kernel_timing(self, name):
        return 0.0, 0, 0.0

    def reset_timing(self):
        pass

    def stage_times(self):
        return {}

    def close(self):
        pass


class _DryReads:
    def free(self):
        pass



def fastq_records(spec, n_reads: int) -> np.ndarray:
    """n_reads of the synthetic spec as 4-line FASTQ records, one uint8 row per record."""
    import dataclasses

    sub = dataclasses.replace(spec, n_reads=n_reads)
    packed, offs = M.synth_host(sub)
    L = sub.read_len
    nb = n_reads * L
    idx = np.arange(nb, dtype=np.uint64)
    codes = ((packed[(idx >> np.uint64(5)).astype(np.int64)] >> (np.uint64(2) * (idx & np.uint64(31)))) & np.uint64(3))
    letters = np.frombuffer(b"ACGT", dtype=np.uint8)[codes.astype(np.int64)].reshape(n_reads, L)
    rec = np.empty((n_reads, 2 * L + 7), dtype=np.uint8)
    rec[:, 0:2] = np.frombuffer(b"@r", dtype=np.uint8)
    rec[:, 2] = 10
    rec[:, 3:3 + L] = letters
    rec[:, 3 + L:6 + L] = np.frombuffer(b"\n+\n", dtype=np.uint8)
    rec[:, 6 + L:6 + 2 * L] = ord("I")
    rec[:, 6 + 2 * L] = 10
    return rec, packed


def measure_ingest(ctx, spec, n_reads: int) -> dict:
    """Untimed: FASTQ text -> 2-bit library in HBM through mcaat_reads_from_fastx (the GPU
    parser, csrc/fastq_ingest.hip). The file (n_reads of the same synthetic spec, 150-bp
    4-line records) is written to local /tmp first, so it is read from the page cache."""
    import tempfile

    rec, want = fastq_records(spec, n_reads)
    nb = n_reads * spec.read_len
    fd, path = tempfile.mkstemp(suffix=".fq", dir="/tmp")
    try:
        with os.fdopen(fd, "wb") as f:
            f.write(rec.tobytes())
        size = os.path.getsize(path)
        del rec
        # the first call also allocates the reader's pinned chunks and device buffers (kept on
        # the context); the second is the steady-state rate
        t0 = time.perf_counter()
        M.Reads.from_fastx(ctx, [path]).free()
        first = time.perf_counter() - t0
        ctx.reset_timing()
        t0 = time.perf_counter()
        r = M.Reads.from_fastx(ctx, [path])
        wall = time.perf_counter() - t0
        n_got, b_got = r.info()
        got, _ = r.download()
        nw = (nb + 31) // 32
        ok = bool(n_got == n_reads and b_got == nb and np.array_equal(got[:nw], want[:nw]))
        # the mapping view (one entry per record; the counting view itself for ACGT-only SE input)
        n_rec, _sep = r.records_info()
        rp, ro = r.download_records()
        ok = ok and bool(n_rec == n_reads and np.array_equal(rp[:nw], want[:nw]) and int(ro[-1]) == nb)
        gpu_ms = 0.0
        kern = {}
        host_pack = ctx.kernel_timing("fq_concat")[1] > 0
        for n in ("fq_parse", "fq_records", "fq_emit", "fq_concat"):
            a, l, by = ctx.kernel_timing(n)
            gpu_ms += a * l
            kern[n] = {"ms": round(a * l, 3), "GBps": round(by / (a * 1e-3) / 1e9, 1) if a > 0 else None}
        r.free()
    finally:
        os.unlink(path)
    return {
        "reads": n_reads, "file_bytes": size, "wall_s": round(wall, 3), "first_call_s": round(first, 3),
        "text_GBps": round(size / first / 1e9, 2), "text_GBps_warm_context": round(size / wall / 1e9, 2),
        "reads_per_s": n_reads / first, "gpu_parse_ms": round(gpu_ms, 3), "kernels": kern, "library_matches": ok,
        "path": "host 2-bit packer (csrc/fastq_pack.hip)" if host_pack else "GPU text parser (csrc/fastq_ingest.hip)",
        "note": "page-cached plain FASTQ; text_GBps = first call on the context (includes allocating the "
                "reader's pinned chunks), warm = second call reusing them; wall includes host read, PCIe upload "
                "and GPU parse",
    }

# per-stage collective counters of the sharded path (kstats "xr_<stage>" / "xq_<stage>")
XR_STAGES = ("build", "tips_filter", "peel", "recount", "candidates", "dls", "find_cycle")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--reads", type=int, default=0, help="override n_reads")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: OMP_NUM_THREADS or the affinity set")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the FASTQ-inclusive span (the workload as FASTQ in /dev/shm through the mcaat CLI)")
    ap.add_argument("--no-post", action="store_true", help="skip the untimed relevant-read mapping measurement")
    ap.add_argument("--ingest-reads", type=int, default=2_000_000,
                    help="untimed FASTQ ingest measurement on a file of this many reads (0: skip)")
    ap.add_argument("--mode", default="shard", choices=["shard", "replicas"],
                    help="N>1: one dataset hash-range sharded over the ranks, or one dataset per rank")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU-only rehearsal of the control flow (ranks, barrier, max-reduce, JSON); no GPU work")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    sharded = world > 1 and args.mode == "shard"
    import torch

    dist = None
    cdev = torch.device("cpu")
    native = sharded
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")  # control plane only (barrier, max of times, the RCCL id)

    cfg = dict(CONFIGS[args.config])
    spec = M.SynthSpec(**cfg["spec"].__dict__)
    if args.reads:
        spec.n_reads = args.reads
    if world > 1 and not sharded:
        spec.seed = spec.seed * 1000 + rank  # independent sample per rank (weak scaling)
    first = rank * spec.n_reads // world if sharded else 0
    count = ((rank + 1) * spec.n_reads // world - first) if sharded else spec.n_reads
    k, thr = cfg["k"], cfg["thr"]

    if args.dry_run:
        ctx = _DryContext()
        reads = _DryReads()
    else:
        if sharded:
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
        ctx = M.Context(local)
        # tuning aid: MCAAT_KNOBS="name=value,..." sets path-selecting knobs (mcaat_set_knob)
        for kv in filter(None, os.environ.get("MCAAT_KNOBS", "").split(",")):
            kn, kval = kv.split("=")
            ctx.set_knob(kn.strip(), int(kval))
        reads = M.Reads.synth_range(ctx, spec, first, count) if sharded else M.Reads.synth(ctx, spec)
    comm = None
    if native and not args.dry_run:
        # the library's communicator: RCCL (its id broadcast over the gloo control plane), or
        # the shared-memory transport for ranks that share one GPU (MCAAT_COMM_BACKEND=gloo)
        if os.environ.get("MCAAT_COMM_BACKEND", "nccl") == "nccl":
            obj = [M.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            comm = M.Comm.rccl(ctx, world, rank, obj[0])
        else:
            obj = [f"/mcaat_bench_{os.getpid()}_{int(time.time() * 1e6) % 10**9}" if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            comm = M.Comm.shm(ctx, world, rank, obj[0])
    prm = M.CfParams(threshold_multiplicity=thr)
    # The FASTQ-inclusive span runs first, on a GPU that no earlier process of this job has
    # used: VRAM released by a process is scrubbed by the driver, and a CLI started right after
    # the bench freed ~200 GB would wait for that inside its span.
    e2e = None
    if rank == 0 and world == 1 and not args.dry_run and not args.no_e2e:
        e2e = run_e2e(ctx, reads, cfg, spec, n_occ(spec, k))

    def step():
        if args.dry_run:
            time.sleep(0.01 * (1 + rank))
            return 0, None, {}
        if native:
            g = M.Graph.build_sharded(ctx, comm, reads, k)
            st_build = ctx.stage_times()
        else:
            g = M.Graph.build(ctx, reads, k)
            st_build = ctx.stage_times()
        d = g.size
        res = g.cycle_finder(prm, as_arrays=True, comm=comm)  # results copied to host arrays
        st_cf = ctx.stage_times()
        g.free()
        return d, res, {**st_build, **st_cf}

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    ctx.reset_timing()
    sync = (lambda: None) if args.dry_run else torch.cuda.synchronize
    barrier()
    sync()
    t0 = time.perf_counter()
    D = 0
    res = None
    stages = {}
    for _ in range(args.steps):
        D, res, st = step()
        for kk, vv in st.items():
            stages[kk] = stages.get(kk, 0.0) + vv / args.steps
    sync()
    barrier()
    dt = (time.perf_counter() - t0) / max(1, args.steps)
    hbm_used = None
    if not args.dry_run:
        free_b, total_b = torch.cuda.mem_get_info(local)
        hbm_used = round((total_b - free_b) / 1e9, 1)  # the arena keeps its chunks: ~ the step's peak
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # dominant kernel = largest HIP-event time per step among the hot-path kernels (a kernel
    # may be launched several times per step, e.g. once per group of L1 buckets)
    def per_step_ms(n):
        a, l, _ = ctx.kernel_timing(n)
        return a * l / max(1, args.steps)
    # pass B of the next group runs on a second stream beside pass C of the current one
    # (knob nc.overlap, on by default), so their HIP-event spans include each other's time
    # and measure neither kernel's own rate: the dominant kernel is taken among the others
    overlap = os.environ.get("MCAAT_KNOBS", "").find("nc.overlap=0") < 0
    alone = [n for n in HOT_KERNELS if not (overlap and n in ("l2_partition", "lds_count"))]
    kern = max(alone, key=per_step_ms)
    avg_ms, launches, bytes_per_launch = ctx.kernel_timing(kern)
    kernels_ms = {n: round(per_step_ms(n), 3) for n in HOT_KERNELS}

    # after the timed region (not part of `value`): the next step of the reference's main,
    # relevant-read mapping (reads.cpp:88-130) on the GPU over the reads still in HBM
    post = None
    if rank == 0 and not args.dry_run and not sharded and not args.no_post:
        g = M.Graph.build(ctx, reads, k)
        r2 = g.cycle_finder(prm)
        nodes = np.array(sorted({x for _, cyc in r2.entries for c in cyc for x in c}), dtype=np.uint64)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        mapped = g.map_reads(reads, nodes)
        wall = (time.perf_counter() - t1) * 1e3
        st = ctx.stage_times()
        n_bases = spec.n_reads * spec.read_len
        ends_bytes = n_bases / 4 + 8 * (spec.n_reads + 1) + 9 * spec.n_reads  # stream + offsets + counts/flags
        post = {
            "relevant_reads": len(mapped),
            "mapped_ids": int(mapped.offsets[-1]),
            "cycle_nodes": int(nodes.size),
            "map_reads_ms": round(wall, 3),
            "stages_ms": {kk: round(vv, 3) for kk, vv in st.items()},
            "map_ends_GBps": round(ends_bytes / (st.get("map_ends", 0) * 1e-3) / 1e9, 1) if st.get("map_ends") else None,
            "reads_per_s": spec.n_reads / (wall * 1e-3),
        }
        g.free()
    ingest = None
    if rank == 0 and world == 1 and not args.dry_run and args.ingest_reads > 0:
        ingest = measure_ingest(ctx, spec, args.ingest_reads)
    kmers_rank = count * max(0, spec.read_len - k)
    kmers_total = n_occ(spec, k) if sharded else kmers_rank * world
    value = kmers_total / dt
    if os.environ.get("MCAAT_COMM_BACKEND", "nccl") == "nccl":
        impl = "native RCCL communicator, CycleFinder over the ranks"
    else:
        impl = "native shared-memory communicator, CycleFinder over the ranks"
    if rank == 0:
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        traffic = traffic_from_profiles(args.config, kern)
        out = {
            "metric": "k-mers/sec through sdbg_build+cycle_finder, 1B-node graph @ 1/2/4/8 GPUs",
            "value": value,
            "unit": "k-mers/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (counter-based RNG genomes with CRISPR arrays, reads generated in HBM)",
            "config": {
                "workload": (cfg["name"] + f", hash-range sharded over {world} GPUs (C4)") if sharded else cfg["name"],
                "reads_per_gpu": count,
                "reads_total": spec.n_reads if sharded else spec.n_reads * world,
                "read_len": spec.read_len,
                "k": k,
                "threshold_multiplicity": thr,
                "error_rate": spec.error_rate,
                "kmers_per_gpu": kmers_rank,
                "kmers_total": kmers_total,
                "sdbg_edges_D": D,
                "parallelism": (f"shard{world} (minimizer-range descriptor all-to-all, BOSS-key-range all-to-all + all-gather; {impl})"
                                if sharded else f"replicas{world}"),
                "cycle_entries": len(res.entries) if res else 0,
                "cycles": res.stats[5] if res else 0,
                "cf_stats": list(res.stats) if res else None,
                "start_candidates": len(res.candidates) if res else 0,
                "hbm_used_GB": hbm_used,
            },
            "roofline": {
                "kernel": kern,
                "kernels_ms_per_step": kernels_ms,
                "overlapped_kernels": [n for n in HOT_KERNELS if n not in alone],
                "lds_overflow_partitions": ctx.kernel_timing("lds_count_overflow_partitions")[1],
                "bound": "hbm",
                "achieved": achieved,
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS,
                "traffic": traffic,
                "avg_launch_ms": avg_ms,
                "launches": launches,
                "algorithmic_bytes_per_launch": bytes_per_launch,
            },
            "stages_ms": {kk: round(vv, 3) for kk, vv in stages.items()},
            "post_path": post,
            # N > 1 (sharded): rank 0's collectives per step and stage, and of them the device
            # all-to-alls RCCL leaves queued on the stream (the rest are host round trips)
            "collectives_per_step": ({st: ctx.kernel_timing("xr_" + st)[1] / max(1, args.steps) for st in XR_STAGES}
                                     if sharded and not args.dry_run else None),
            "collectives_queued_per_step": ({st: ctx.kernel_timing("xq_" + st)[1] / max(1, args.steps) for st in XR_STAGES}
                                            if sharded and not args.dry_run else None),
            "fastq_ingest": ingest,
            "cpu_baseline": None,
        }
        # step-level roofline: B_alg = 0.25 N_bases + 16 N_occ + 8 C + 8 D_c + 41 D with
        # C = 2 D_c (count table model) and D_c ~ D/2 distinct canonical edges
        if D:
            d_c = (D + 1) // 2
            b_alg = 0.25 * spec.n_reads * spec.read_len * (1 if sharded else world) + 16.0 * kmers_total \
                + 8.0 * 2 * d_c + 8.0 * d_c + 41.0 * D
            out["step_roofline"] = {
                "B_alg": b_alg, "achieved_GBps": b_alg / dt / 1e9 / world,
                "frac": b_alg / dt / 1e9 / world / PEAK_HBM_GBS,
                "pmc_bytes_per_step": step_traffic_from_profiles(args.config),
                "note": "SURVEY.md §8d algorithmic bytes over the step time, per GPU; pmc_bytes_per_step = "
                        f"FETCH+WRITE of every kernel of one profiled step of this config "
                        f"(profiles/traffic_{args.config}.json; FETCH doubled only for wide coalesced "
                        "stream reads: corrected, and as counted: raw)",
            }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.dry_run:
        try:
            out["cpu_baseline"] = cpu_baseline(ctx, cfg, args.cpu_threads or host_threads())
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"error": str(e)}
    reads.free()
    if comm is not None:
        comm.close()
    ctx.close()
    if rank == 0:
        out["e2e"] = e2e
        # The reference's own headline span (main.cpp:517-536: SDBGBuild start to
        # CycleFinder end, FASTQ parse included), measured by the CLI in a fresh process, at the
        # top level beside `value` (device-resident throughput, the measurement contract's
        # value): without the HIP runtime init + kernel code-object load before the span, and
        # with them (from the CLI's main() start: TIMING_TAIL span_end_s). README names which
        # is the headline.
        if e2e and "T_s" in e2e:
            n_k = n_occ(spec, k)
            t_init = e2e.get("cli_phases_s", {}).get("span_end_s")
            out["span"] = {
                "T_s": e2e["T_s"], "kmers_per_s": n_k / e2e["T_s"],
                "T_with_init_s": round(t_init, 3) if t_init else None,
                "kmers_per_s_with_init": n_k / t_init if t_init else None,
                "init_s": e2e.get("cli_phases_s", {}).get("init_s"),
                "source": "e2e (mcaat CLI on the same reads as FASTQ in tmpfs)",
            }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
