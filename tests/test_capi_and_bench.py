"""CPU tests of the C ABI library (loads, exports every declared symbol, fails cleanly
without a GPU), the host-side synthetic generator, and the bench's multi-rank control flow."""
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import mcaat_amd as M
from mcaat_amd import lib as L
from tests.helpers import unpack_read, rc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    txt = open(os.path.join(ROOT, "include", "mcaat_gpu.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mcaat_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = M.load_library()
    names = declared_functions()
    assert len(names) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        assert hasattr(lib, n)
    # and the Python binding declares a signature for each of them
    assert sorted(L.SIGNATURES) == names


def test_init_without_gpu_fails_cleanly():
    if M.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(M.McaatError) as ei:
        M.Context(0)
    assert ei.value.code == -2  # MCAAT_E_HIP
    assert "device" in str(ei.value)


def test_default_cf_params_match_reference_settings():
    p = L._CfParams()
    M.load_library().mcaat_cf_default_params(p)
    # settings.h:34-37, cycle_finder.cpp:132,149
    assert (p.threshold_multiplicity, p.low_abundance, p.cycle_max_length, p.cycle_min_length) == (20, 1, 77, 27)
    assert (p.cluster_bound, p.step_cap) == (500, 10_000_000)


def test_synth_reads_are_genome_segments():
    spec = M.SynthSpec(seed=5, n_genomes=2, genome_len=5000, arrays_per_genome=1, spacers_per_array=4,
                       n_reads=300, read_len=100)
    packed, offs = M.synth_host(spec)
    gen = M.synth_genome_host(spec)
    genomes = [unpack_read(gen, g * 5000, (g + 1) * 5000) for g in range(2)]
    both = genomes + [rc(x) for x in genomes]
    for r in range(spec.n_reads):
        s = unpack_read(packed, int(offs[r]), int(offs[r + 1]))
        assert any(s in x for x in both)
    # deterministic
    p2, _ = M.synth_host(spec)
    assert np.array_equal(packed, p2)


def test_synth_paired_reads_and_errors():
    spec = M.SynthSpec(seed=9, n_genomes=1, genome_len=4000, arrays_per_genome=0, n_reads=400, read_len=80,
                       paired=True, error_rate=0.0)
    packed, offs = M.synth_host(spec)
    g = unpack_read(M.synth_genome_host(spec), 0, 4000)
    for p in range(0, 400, 2):
        r1 = unpack_read(packed, int(offs[p]), int(offs[p + 1]))
        r2 = unpack_read(packed, int(offs[p + 1]), int(offs[p + 2]))
        # mates face each other on opposite strands within 270..330 bp
        if r1 in g:
            i1, i2 = g.find(r1), g.find(rc(r2))
        else:
            i1, i2 = g.find(rc(r1)), g.find(r2)
        assert i1 >= 0 and i2 >= 0
        assert 270 <= abs(i2 - i1) + 80 <= 330
    spec.error_rate = 0.05
    pe, _ = M.synth_host(spec)
    diff = int(np.count_nonzero(pe != packed))
    assert diff > 0


@pytest.mark.parametrize("mode,port", [("replicas", 29561), ("shard", 29562)])
def test_bench_two_ranks_gloo_dry_run(mode, port):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--config", "tiny", "--dry-run", "--mode", mode]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    # value = all k-mers processed / max-over-ranks step time (rank 1 sleeps longer)
    assert d["ms_per_step"] >= 19.0
    total = d["config"]["kmers_total"]
    assert abs(d["value"] - total / (d["ms_per_step"] / 1e3)) / d["value"] < 1e-6
    if mode == "replicas":
        assert d["scaling"] == "weak" and total == 2 * d["config"]["kmers_per_gpu"]
    else:  # one dataset split over the ranks
        assert d["scaling"] == "strong" and total == 2 * d["config"]["kmers_per_gpu"]
        assert d["config"]["reads_total"] == 10_000


def test_host_library_exports_every_declared_symbol():
    """libmcaat_host.so (include/mcaat_host.h): the downstream steps' C ABI."""
    from mcaat_amd import downstream as DS

    txt = open(os.path.join(ROOT, "include", "mcaat_host.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = sorted(set(re.findall(r"\b(mcaat_host_[a-z_]+)\s*\(", txt)))
    assert len(names) >= 6
    out = subprocess.run(["nm", "-D", "--defined-only", DS.HOST_LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert not [n for n in names if n not in exported]
    assert sorted(DS.HOST_SIGNATURES) == names
    DS.load_host_library()
