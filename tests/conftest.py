import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu on the MI355X box)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def le():
    import leo_erasure_amd
    return leo_erasure_amd


@pytest.fixture(scope="session")
def gpu(le):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    assert le.gf_init() == "ok", le.gf_init()
    return torch
