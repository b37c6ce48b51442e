import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmcaat_gpu.so on the device)")


@pytest.fixture(scope="session")
def gpu_ctx():
    import mcaat_amd as M

    if M.device_count() < 1:
        pytest.fail("GPU test requested but no HIP device is visible")
    ctx = M.Context(0)
    yield ctx
    ctx.close()
