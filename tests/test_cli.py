"""The mcaat CLI (C++ host mirror of the reference's Settings / SDBGBuild / SDBG / CycleFinder).

CPU: flag/settings.txt parsing and error behaviour mirror the reference (main.cpp:89-301,
settings.h:127-220). GPU: end-to-end FASTQ -> cycles.txt equals the oracle's cycles."""
import os
import subprocess

import numpy as np
import pytest

import mcaat_amd as M
import oracle as O
from tests.helpers import unpack_read

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "mcaat_amd", "mcaat")


def run(args, **kw):
    return subprocess.run([CLI] + args, capture_output=True, text=True, timeout=600, **kw)


def write_fastq(path, packed, offs):
    with open(path, "w") as f:
        for r in range(len(offs) - 1):
            s = unpack_read(packed, int(offs[r]), int(offs[r + 1]))
            f.write(f"@r{r}\n{s}\n+\n{'I' * len(s)}\n")


def test_cli_help():
    out = run(["--help"])
    assert out.returncode == 0
    assert "--input-files" in out.stdout and "--threshold-multiplicity" in out.stdout


def test_cli_missing_inputs_errors(tmp_path):
    out = run(["--output-folder", str(tmp_path / "o")])
    assert out.returncode == 1
    assert "No input files provided" in out.stderr
    out = run(["-i", str(tmp_path / "nope.fq"), "--output-folder", str(tmp_path / "o")])
    assert out.returncode == 1 and "does not exist" in out.stderr


def test_cli_settings_file_and_overrides(tmp_path):
    fq = tmp_path / "r.fq"
    fq.write_text("@a\nACGT\n+\nIIII\n")
    st = tmp_path / "settings.txt"
    st.write_text(
        "# comment\ninput_files=%s\nthreads=2 // trailing\nram=4G\ncycle_max_length=70\n"
        "threshold_multiplicity=7\nlow_abundance=no\nunknown_key=1\nkmer_k=21\n" % fq)
    out = run(["--settings", str(st), "--cycle-min-length", "25", "--output-folder", str(tmp_path / "o")],
              input="n\n")
    assert "max_length=70 min_length=25 threshold_mult=7 low_abundance=false threads=2" in out.stdout
    assert "[✔] RAM: 4.00 GB" in out.stdout
    assert os.path.isdir(tmp_path / "o" / "graph") and os.path.isdir(tmp_path / "o" / "cycles")
    if M.device_count() == 0:
        assert out.returncode == 1 and "no HIP device" in out.stderr
        # SDBGBuild wrote the reference's data.lib before touching the GPU
        lib = (tmp_path / "o" / "graph" / "data.lib").read_text()
        assert lib == f"#lib file for the SDBG from {fq}\nse {fq}"


@pytest.mark.gpu
def test_cli_end_to_end_cycles_match_oracle(tmp_path):
    spec = M.SynthSpec()  # C1 tiny
    packed, offs = M.synth_host(spec)
    fq = tmp_path / "reads.fq"
    write_fastq(fq, packed, offs)
    out = run(["-i", str(fq), "--output-folder", str(tmp_path / "o"), "--threads", "2", "--ram", "2G"])
    assert out.returncode == 0, out.stderr
    txt = (tmp_path / "o" / "cycles" / "cycles.txt").read_text().split("\n")
    seqs = [l for l in txt if l and not l.startswith(">")]
    og = O.OGraph.build(packed, offs, 23)
    res = og.cycle_finder()
    keys, _ = og.arrays()

    def label(e):
        return "".join("ACGT"[x - 1] for x in og.label(e))

    expected = []
    for _, cycles in res["entries"]:
        for c in cycles:
            expected.append(label(c[0]) + "".join(label(x)[-1] for x in c[1:]))
    assert sorted(seqs) == sorted(expected)
    assert len(seqs) == 24
