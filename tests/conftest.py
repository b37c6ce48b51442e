import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmcaat_gpu.so on the device)")


_SESSION_CTX = []


@pytest.fixture(scope="session")
def gpu_ctx():
    import mcaat_amd as M

    if M.device_count() < 1:
        pytest.fail("GPU test requested but no HIP device is visible")
    ctx = M.Context(0)
    _SESSION_CTX.append(ctx)
    yield ctx
    _SESSION_CTX.clear()
    ctx.close()


@pytest.fixture(autouse=True)
def _release_cached_device_memory():
    """The session context's arena keeps freed device blocks for reuse; the full-size tests
    leave up to ~260 GB of them. Released before every test, so tests that start other GPU
    processes (ranks, the CLI) find the memory free."""
    for ctx in _SESSION_CTX:
        ctx.trim()
    yield
