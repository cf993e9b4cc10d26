import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")
    # A test that hangs fails after this long with every thread's stack
    # (pytest-timeout's thread method: it can interrupt a test stuck in a GPU
    # call) instead of holding the run; --timeout on the command line wins.
    if hasattr(config.option, "timeout") and not config.option.timeout:
        config.option.timeout = 150
        config.option.timeout_method = "thread"


@pytest.fixture(scope="session")
def gpu_device():
    # torch's HIP state first: some GPU tests hand device buffers to the
    # library, and torch initialised after the library's own HIP calls
    # reported no device when a run started with those tests
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    import sahara_amd as sa
    n = sa.lib().sahara_gpu_device_count()
    if n < 1:
        pytest.fail("no HIP device visible; gpu-marked tests need an MI355X")
    return 0
