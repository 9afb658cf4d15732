"""The bitsliced GF(2^16)/GF(2^32) core of gfs_apply (leo_erasure_amd/csrc/
gfs_core.hpp), compiled for the CPU and checked against the oracle's field:
transposes are exact inverses and put bit k of every word in plane k, and
the plane-domain multiply-accumulate equals XOR_j c_rj * x_j word by word
for zero, one, sparse, dense and random coefficients."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def core(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("gfs") / "libgfs_core_test.so")
    subprocess.run(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-Werror", "-Wno-unknown-pragmas",
                    os.path.join(HERE, "gfs_core_test.cpp"), "-o", so], check=True)
    L = ctypes.CDLL(so)
    L.gfs_region.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2 + [ctypes.c_size_t,
                                                                           ctypes.c_void_p]
    L.gfs_transpose_roundtrip.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3
    return L


def xtime(x, w):
    poly = {16: 0x1100B, 32: 0x100400007}[w]
    top = (x >> (w - 1)) & 1
    return ((x << 1) ^ (top * (poly))) & ((1 << w) - 1)


def gf_mul_vec(c, x, w):
    """c (int) * x (uint64 array) in GF(2^w), shift-and-add."""
    x = x.astype(np.uint64).copy()
    acc = np.zeros_like(x)
    for t in range(w):
        if (c >> t) & 1:
            acc ^= x
        x = xtime(x, w)
    return acc


@pytest.mark.parametrize("w", [16, 32])
def test_transpose_planes(core, w):
    rng = np.random.default_rng(w)
    n = w
    rows = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    planes = np.zeros(n, dtype=np.uint32)
    back = np.zeros(n, dtype=np.uint32)
    core.gfs_transpose_roundtrip(w, rows.ctypes.data, planes.ctypes.data, back.ctypes.data)
    assert np.array_equal(back, rows)
    # the 32 words of the rows: w = 32 the rows; w = 16 the halves of each row
    if w == 32:
        words = rows.astype(np.uint64)
    else:
        words = np.concatenate([rows & 0xFFFF, rows >> 16]).astype(np.uint64)
    for k in range(w):  # plane k holds bit k of all 32 words, each exactly once
        bits = sorted(int(b) for b in range(32) if (int(planes[k]) >> b) & 1)
        assert len(bits) == int(((words >> k) & 1).sum()), k


@pytest.mark.parametrize("w", [16, 32, -32])
@pytest.mark.parametrize("R,K", [(1, 1), (4, 10), (3, 5), (2, 16)])
def test_region_matches_field(core, oracle, w, R, K):
    """w = 32: the packed 16-words-per-lane form gfs_apply ships; -32: the
    unpacked 32-words-per-lane form (R = 1, 4)."""
    wf = w
    w = abs(w)
    if wf < 0 and R not in (1, 4):
        pytest.skip("unpacked form instantiated for R = 1, 4")
    rng = np.random.default_rng(w * 100 + R * 10 + K)
    nwords = 32 * 24
    dt = np.uint16 if w == 16 else np.uint32
    ins = rng.integers(0, 2**w, (K, nwords), dtype=np.uint64).astype(dt)
    special = [0, 1, 2, (1 << w) - 1, 1 << (w - 1), 0x5555 if w == 16 else 0x80000001]
    coef = rng.integers(0, 2**w, (R, K), dtype=np.uint64)
    for i, v in enumerate(special):
        coef.flat[i % coef.size] = v
    coef32 = coef.astype(np.uint32)
    out = np.zeros((R, nwords), dtype=dt)
    assert core.gfs_region(wf, R, K, coef32.ctypes.data, ins.ctypes.data, ins[0].nbytes,
                           out.ctypes.data) == 0
    for r in range(R):
        ref = np.zeros(nwords, dtype=np.uint64)
        for j in range(K):
            ref ^= gf_mul_vec(int(coef[r, j]), ins[j], w)
        assert np.array_equal(out[r].astype(np.uint64), ref), (r, w)
    # the numpy field is the oracle's field
    for _ in range(50):
        a, b = (int(v) for v in rng.integers(1, 2**w, 2, dtype=np.uint64))
        assert int(gf_mul_vec(a, np.array([b], dtype=np.uint64), w)[0]) == oracle.gf_mul(a, b, w)
