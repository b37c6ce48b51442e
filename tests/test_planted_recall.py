"""Planted-array recall of the whole CLI (SURVEY.md §8f rank 1 on top of the hot path): the
synthetic community's CRISPR arrays (mcaat_synth_arrays_host, the ground truth a reference run
would take as its benchmark file, main.cpp:559-569) must all come out of the `mcaat` CLI's
CRISPR_Arrays.txt. Scoring: mcaat_amd/truth.py (a planted array is recalled when one reported
system carries at least half of its spacers, either orientation, a few bases of slack at the
ends). The sizes: a C3-regime sample (40 arrays) and the full C3 dataset (300M reads, 400
arrays, D ~ 1e9, 92 GB of FASTQ in /dev/shm)."""
import dataclasses
import os
import shutil
import subprocess

import pytest

import mcaat_amd as M
from mcaat_amd.configs import CONFIGS
from mcaat_amd.truth import parse_crispr_arrays, planted_recall

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "mcaat_amd", "mcaat")


def _cli_recall(ctx, spec, k, thr, work):
    fq = os.path.join(work, "reads.fq")
    reads = M.Reads.synth(ctx, spec)
    reads.write_fastq(fq, threads=16)
    reads.free()
    ctx.trim()  # the CLI is another process on this GPU
    st = os.path.join(work, "settings.txt")
    with open(st, "w") as f:
        f.write(f"kmer_k={k}\nthreshold_multiplicity={thr}\nthreads=16\n")
    try:
        out = subprocess.run([CLI, "--settings", st, "--input-files", fq, "--output-folder",
                              os.path.join(work, "out")], capture_output=True, text=True, timeout=900)
    finally:
        os.unlink(fq)
    assert out.returncode == 0, out.stderr[-3000:] + out.stdout[-2000:]
    systems = parse_crispr_arrays(os.path.join(work, "out", "CRISPR_Arrays.txt"))
    return planted_recall(systems, M.synth_arrays(spec))


@pytest.mark.gpu
def test_planted_arrays_recalled_c3_sample(gpu_ctx, tmp_path):
    spec = dataclasses.replace(CONFIGS["c3"]["spec"], n_genomes=20, n_reads=30_000_000)
    rec = _cli_recall(gpu_ctx, spec, 27, 20, str(tmp_path))
    assert rec["planted"] == 40
    assert rec["recall"] == 1.0, rec


@pytest.mark.gpu
@pytest.mark.timeout(1500)
def test_planted_arrays_recalled_c3_full(gpu_ctx):
    cfg = CONFIGS["c3"]
    spec = cfg["spec"]
    need = 2 * spec.n_reads * spec.read_len + 7 * spec.n_reads
    if shutil.disk_usage("/dev/shm").free < 1.1 * need:
        pytest.skip(f"/dev/shm holds less than {need / 1e9:.0f} GB")
    work = f"/dev/shm/mcaat_recall_{os.getpid()}"
    os.makedirs(work, exist_ok=True)
    try:
        rec = _cli_recall(gpu_ctx, spec, cfg["k"], cfg["thr"], work)
    finally:
        shutil.rmtree(work, ignore_errors=True)
    assert rec["planted"] == 400
    assert rec["recall"] == 1.0, rec
