"""Sharded (multi-GPU) build: the orchestration over gloo with the CPU restatement of the
per-rank pieces (no GPU), and the real kernels with two ranks sharing one GPU."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mcaat_amd import shard  # noqa: E402


def _run(nproc: int, port: int, extra, timeout=600):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tools", "shard_check.py")] + extra
    return subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout)


def test_choose_splits_balances_and_is_monotone():
    rng = np.random.default_rng(5)
    h = rng.integers(0, 1000, size=4096).astype(np.uint64)
    for world in (1, 2, 3, 8):
        sp = shard.choose_splits(h, world, 56)
        assert len(sp) == world - 1
        assert np.all(np.diff(sp.astype(np.float64)) >= 0)
        bins = np.concatenate([[0], (sp >> np.uint64(56 - 12)).astype(np.int64), [4096]])
        loads = [int(h[bins[i]:bins[i + 1]].sum()) for i in range(world)]
        assert max(loads) - min(loads) <= 2 * int(h.max())
    assert len(shard.choose_splits(np.zeros(16, dtype=np.uint64), 4, 10)) == 3


@pytest.mark.parametrize("nproc,port", [(2, 29571), (3, 29572)])
def test_sharded_build_gloo_matches_single_process(nproc, port):
    out = _run(nproc, port, ["--oracle", "--reads", "12000"])
    assert out.returncode == 0, out.stderr[-3000:]
    assert "SHARD_OK" in out.stdout


@pytest.mark.gpu
def test_sharded_build_two_ranks_on_one_gpu():
    out = _run(2, 29573, ["--reads", "30000"])
    assert out.returncode == 0, out.stderr[-3000:]
    assert "SHARD_OK" in out.stdout
