#!/usr/bin/env python3
"""Probe of the FASTQ-inclusive span: writes a config's reads as FASTQ to /dev/shm once, then
runs the mcaat CLI on it under several environment variants (reader threads, chunk size,
MCAAT_VERBOSE stage marks) and prints each run's TIMING line and verbose marks.

usage: python tools/e2e_probe.py [--config c3] [--reads N] [--variants "A=1,B=2;C=3" ...]
"""
import argparse
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import mcaat_amd as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reads", type=int, default=0)
    ap.add_argument("--variants", default="")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--settle", type=float, default=0.0, help="seconds to wait after writing the FASTQ")
    ap.add_argument("--preread", action="store_true", help="read the file once (8 threads) before the runs")
    ap.add_argument("--gap", type=float, default=0.0, help="seconds between runs (the driver scrubs freed VRAM)")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    spec = M.SynthSpec(**cfg["spec"].__dict__)
    if a.reads:
        spec.n_reads = a.reads
    path = f"/dev/shm/e2e_probe_{os.getpid()}.fq"
    with M.Context(0) as ctx:
        r = M.Reads.synth(ctx, spec)
        t0 = time.perf_counter()
        r.write_fastq(path, threads=bench.host_threads())
        print(f"wrote {os.path.getsize(path) / 1e9:.1f} GB in {time.perf_counter() - t0:.1f} s", flush=True)
        r.free()
    if a.settle:
        time.sleep(a.settle)
        print(f"settled {a.settle} s", flush=True)
    if a.preread:
        import concurrent.futures as cf

        size = os.path.getsize(path)
        piece = (size + 7) // 8

        def rd(i):
            with open(path, "rb", buffering=0) as f:
                f.seek(i * piece)
                left = min(piece, size - i * piece)
                while left > 0:
                    b = f.read(min(left, 64 << 20))
                    if not b:
                        break
                    left -= len(b)

        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(8) as ex:
            list(ex.map(rd, range(8)))
        print(f"pre-read {size / 1e9:.1f} GB in {time.perf_counter() - t0:.2f} s", flush=True)
    work = tempfile.mkdtemp(dir="/tmp")
    try:
        st = os.path.join(work, "s.txt")
        with open(st, "w") as f:
            f.write(f"kmer_k={cfg['k']}\nthreshold_multiplicity={cfg['thr']}\n")
        for vi, var in enumerate(a.variants.split(";") if a.variants else [""]):
            if vi and a.gap:
                time.sleep(a.gap)
            env = dict(os.environ)
            for kv in filter(None, var.split(",")):
                k, v = kv.split("=", 1)
                env[k] = v
            if a.verbose:
                env["MCAAT_VERBOSE"] = "1"
            t0 = time.perf_counter()
            p = subprocess.run([os.path.join(ROOT, "mcaat_amd", "mcaat"), "--settings", st, "-i", path,
                                "--output-folder", os.path.join(work, "o")], env=env, capture_output=True, text=True,
                               timeout=900)
            wall = time.perf_counter() - t0
            shutil.rmtree(os.path.join(work, "o"), ignore_errors=True)
            timing = [ln for ln in p.stdout.splitlines() if ln.startswith("TIMING")]
            print(f"variant [{var}] rc={p.returncode} wall={wall:.2f}s {timing}", flush=True)
            if a.verbose or p.returncode:
                for ln in p.stderr.splitlines()[-60:]:
                    print("   ", ln)
    finally:
        shutil.rmtree(work, ignore_errors=True)
        os.unlink(path)


if __name__ == "__main__":
    main()
