import os
import sys

import pytest

# glibc writes its fatal-error reports (heap corruption, failed checks) to
# /dev/tty unless this is set; a GPU box has no tty, so an abort there would
# otherwise leave no message (round 2's unexplained abort).
os.environ.setdefault("LIBC_FATAL_STDERR_", "1")

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


class MeasureEnv:
    """LEOEC_* knobs of the measurement build: set / clear a variable and have
    the library re-read them (the product build never reads the environment)."""

    def __init__(self, mp, lib):
        self.mp, self.lib = mp, lib

    def setenv(self, key, value):
        self.mp.setenv(key, value)
        self.lib.measure_reload()

    def delenv(self, key, raising=False):
        self.mp.delenv(key, raising=False)
        self.lib.measure_reload()


@pytest.fixture
def measure(le, gpu, monkeypatch):
    """Route the package through libleoec_measure.so (A/B kernel forms) for
    one test; skipped when that build is absent (`make -C leo_erasure_amd/csrc
    measure`): the forms it adds are not shipped."""
    from leo_erasure_amd import _lib
    if not os.path.exists(_lib.MEASURE_LIB_PATH):
        pytest.skip("measurement build absent (make -C leo_erasure_amd/csrc measure)")
    prev = _lib.use_library(_lib.MEASURE_LIB_PATH)
    try:
        assert le.gf_init() == "ok"
        _lib.measure_reload()
        yield MeasureEnv(monkeypatch, _lib)
    finally:
        monkeypatch.undo()
        _lib.measure_reload()
        _lib.use_library(prev)
