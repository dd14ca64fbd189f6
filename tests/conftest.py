import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running (full BASELINE sizes)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected but no GPU is visible (run with -m 'not gpu' on CPU hosts)")
    from denseretrievaltoolkits_amd import _native
    _native.load()  # fail loudly if the extension is missing
    return torch.device("cuda", 0)
