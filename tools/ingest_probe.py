"""Times mcaat_reads_from_fastx on one page-cached synthetic FASTQ several times (GPU box)."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mcaat_amd as M  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30_000_000
spec = M.SynthSpec(**bench.CONFIGS["c3"]["spec"].__dict__)
rec, _ = bench.fastq_records(spec, n)
fd, path = tempfile.mkstemp(suffix=".fq", dir="/tmp")
with os.fdopen(fd, "wb") as f:
    f.write(rec.tobytes())
size = os.path.getsize(path)
del rec
with M.Context(0) as ctx:
    for it in range(4):
        ctx.reset_timing()
        t0 = time.perf_counter()
        r = M.Reads.from_fastx(ctx, [path])
        dt = time.perf_counter() - t0
        k = {nm: round(ctx.kernel_timing(nm)[0] * ctx.kernel_timing(nm)[1], 1) for nm in ("fq_parse", "fq_records", "fq_emit")}
        print(f"{size / dt / 1e9:.2f} GB/s  wall {dt * 1e3:.0f} ms  kernels {k}", flush=True)
        r.free()
os.unlink(path)
