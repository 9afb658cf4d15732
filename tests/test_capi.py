"""The C-ABI library without a GPU: it loads, exports every symbol that
include/leoec.h declares, and its host logic (parameter checks, stripe
geometry, coding matrices, error strings) agrees with the oracle."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    with open(os.path.join(ROOT, "include", "leoec.h")) as fh:
        text = fh.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(leoec_\w+)\s*\(", text, re.M)))


def test_exports_every_declared_symbol(le):
    names = header_functions()
    assert len(names) >= 13
    so = os.path.join(ROOT, "leo_erasure_amd", "libleoec.so")
    dyn = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (leoec_\w+)$", dyn, re.M))
    for n in names:
        assert n in exported, n
        assert getattr(le.lib, n) is not None
    assert set(le._lib.EXPORTS) == set(names)


def test_library_is_gfx950_code(le, tmp_path):
    """The device code bundled in libleoec.so targets gfx950 only."""
    so = os.path.join(ROOT, "leo_erasure_amd", "libleoec.so")
    fat = tmp_path / "fatbin.bin"
    subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", so, str(fat)])
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          "--input=" + str(fat)], capture_output=True, text=True, check=True)
    targets = {t for t in out.stdout.split() if t.startswith("hip")}
    assert targets == {"hipv4-amdgcn-amd-amdhsa--gfx950"}, targets


CLASSES = {"cauchyrs": 1, "vandrs": 2, "liberation": 3, "isars": 4}


def test_check_params_matches_oracle(le, oracle):
    for coding in range(0, 6):
        for k in (-1, 0, 1, 4, 10, 250, 300):
            for m in (0, 1, 2, 4, 7):
                for w in (0, 1, 2, 3, 5, 6, 7, 8, 9, 11, 13, 16, 31, 32, 33):
                    assert le.lib.leoec_check_params(coding, k, m, w) == \
                        oracle.lib().orc_check_params(coding, k, m, w), (coding, k, m, w)


def test_layout_matches_oracle(le, oracle):
    bs = ctypes.c_uint64()
    filled = ctypes.c_int()
    rng = np.random.default_rng(0)
    sizes = [0, 1, 15, 16, 1023, 1024, 1048576, 10485761, 64 << 20] + \
        [int(x) for x in rng.integers(1, 1 << 26, 50)]
    for cls, k, m, w in [("vandrs", 10, 4, 8), ("vandrs", 4, 2, 16), ("cauchyrs", 4, 2, 3),
                         ("liberation", 4, 2, 7), ("isars", 10, 4, 8), ("vandrs", 6, 3, 32)]:
        for size in sizes:
            assert le.lib.leoec_layout(CLASSES[cls], k, m, w, size, ctypes.byref(bs),
                                       ctypes.byref(filled)) == 0
            assert bs.value == oracle.block_size(k, w, size)
            assert filled.value == (min(size // bs.value, k) if bs.value else 0)


def _engine_matrix(le, coding, k, m, w):
    n = ctypes.c_int()
    le.lib.leoec_coding_matrix(CLASSES[coding], k, m, w, None, 0, ctypes.byref(n))
    out = np.zeros(n.value, dtype=np.uint32)
    rc = le.lib.leoec_coding_matrix(CLASSES[coding], k, m, w,
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                    n.value, ctypes.byref(n))
    assert rc == 0
    return out


@pytest.mark.parametrize("k,m,w", [(10, 4, 8), (4, 2, 8), (8, 3, 8), (4, 1, 8), (7, 7, 8),
                                   (20, 5, 8), (200, 56, 8), (4, 2, 16), (10, 4, 16),
                                   (4, 2, 32), (10, 4, 32)])
def test_vandrs_matrix_matches_oracle(le, oracle, k, m, w):
    assert np.array_equal(_engine_matrix(le, "vandrs", k, m, w),
                          oracle.vandermonde_coding_matrix(k, m, w).reshape(-1))


@pytest.mark.parametrize("k,m", [(10, 4), (4, 2), (8, 3), (100, 20)])
def test_isars_matrix_matches_oracle(le, oracle, k, m):
    assert np.array_equal(_engine_matrix(le, "isars", k, m, 8),
                          oracle.isal_gen_cauchy1_matrix(k + m, k)[k:].reshape(-1))


@pytest.mark.parametrize("k,m,w", [(10, 4, 8), (4, 2, 3), (6, 3, 4), (10, 4, 10), (10, 2, 8),
                                   (30, 2, 5), (12, 4, 16), (5, 3, 13)])
def test_cauchy_bitmatrix_matches_oracle(le, oracle, k, m, w):
    C = oracle.cauchy_good_general_coding_matrix(k, m, w)
    assert np.array_equal(_engine_matrix(le, "cauchyrs", k, m, w),
                          oracle.matrix_to_bitmatrix(k, m, w, C).reshape(-1))


@pytest.mark.parametrize("k,w", [(4, 7), (5, 5), (10, 11), (13, 13), (2, 3)])
def test_liberation_bitmatrix_matches_oracle(le, oracle, k, w):
    assert np.array_equal(_engine_matrix(le, "liberation", k, 2, w),
                          oracle.liberation_coding_bitmatrix(k, w).reshape(-1))


def test_error_strings(le):
    """Message texts of the reference (c_src/*coding.cpp, leo_erasure_nif.cpp)."""
    want = {
        -1: "Invalid Coding", -2: "Invalid Coding Parameters",
        -3: "Invalid Coding Parameters (w = 8/16/32)",
        -4: "Invalid Coding Parameters (larger w)", -5: "Invalid Coding Parameters (m = 2)",
        -6: "Invalid Coding Parameters (k <= w)", -7: "Invalid Coding Parameters (w is prime)",
        -8: "Invalid Coding Parameters (w = 8)", -9: "Not Enough Blocks",
        -10: "Blocks should be unique", -11: "Non Invertible",
    }
    for code, text in want.items():
        assert le.strerror(code) == text


def test_no_cpu_fallback_without_gpu(le):
    """Without a gfx950 device the data path reports NO_DEVICE — never a CPU result."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    st, why = le.nif_encode("vandrs", (10, 4, 8), b"x" * 5000, 5000)
    assert (st, why) == ("error", "No gfx950 HIP device")
    assert le.gf_init() == ("error", "No gfx950 HIP device")
    assert le._lib.lib.leoec_host_lanes(None, 0) == le._lib.E_NO_DEVICE
    assert le._lib.lib.leoec_device() == le._lib.E_NO_DEVICE


def test_measure_knob_setter_never_writes_the_environment():
    """The measurement build's knobs are set through leoec_measure_set_knob
    (an override table inside the library), not setenv: the environment is
    unchanged, a non-LEOEC name is refused, and a reset drops the overrides.
    Loaded in a child process (one HIP library per process)."""
    import subprocess
    import sys
    from leo_erasure_amd import _lib
    if not os.path.exists(_lib.MEASURE_LIB_PATH):
        pytest.skip("measurement build absent")
    code = r'''
import os, sys
sys.path.insert(0, %r)
os.environ["LEOEC_LIBRARY"] = "measure"
from leo_erasure_amd import _lib
assert _lib.is_measure_build()
before = dict(os.environ)
_lib.measure_set_knob("LEOEC_GFBIT_LW", 4)
_lib.measure_set_knob("LEOEC_GFBIT_LW", None)
_lib.measure_set_knob("LEOEC_HOST_STAGING", "gather")
try:
    _lib.measure_set_knob("PATH", "x")
    raise SystemExit("non-LEOEC name accepted")
except ValueError:
    pass
_lib.measure_reset_knobs()
assert dict(os.environ) == before
print("ok")
''' % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr[-2000:]
