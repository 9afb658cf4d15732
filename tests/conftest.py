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
    config.addinivalue_line("markers", "measure_gpu: measurement-build form tests (GPU); run in "
                            "their own process with LEOEC_LIBRARY=measure")


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


class MeasureKnobs:
    """LEOEC_* knobs of the measurement build, set through the library's own
    setter (leoec_measure_set_knob): the process environment is never
    written while the library's queue threads and the HIP runtime's threads
    run (round 3's verdict on the round-2 abort)."""

    def __init__(self, lib):
        self.lib = lib

    def setenv(self, key, value):
        self.lib.measure_set_knob(key, value)

    def delenv(self, key, raising=False):
        self.lib.measure_set_knob(key, None)


@pytest.fixture
def measure(le, gpu):
    """The measurement build's A/B kernel forms for one test.  They run only
    in a process that loaded libleoec_measure.so alone (LEOEC_LIBRARY=measure,
    tests/test_measure_forms.py's own process, started by
    test_gpu_parity.py::test_measurement_forms_in_own_process): a product-test
    process never loads a second HIP library."""
    from leo_erasure_amd import _lib
    if not _lib.is_measure_build():
        pytest.skip("measurement-form test: runs in its own process with LEOEC_LIBRARY=measure "
                    "(test_measurement_forms_in_own_process)")
    _lib.measure_reset_knobs()
    try:
        yield MeasureKnobs(_lib)
    finally:
        _lib.measure_reset_knobs()
