"""Pins for the CPU oracle (oracle/leoec_oracle.c).

The reference holds no golden vectors (every eunit test is a
self-consistency check), and its arithmetic libraries are absent.  The oracle
is therefore pinned by:
  1. known-answer values recalled from public documentation (the Jerasure
     manual's reed_sol_01 7 7 8 example, the cbest_2..5 tables of
     cauchy_best_r6.c) and the SURVEY Appendix A values;
  2. an independent second restatement (tests/restate_np.py: log tables,
     closed-form Vandermonde) that must agree entry by entry;
  3. the reference's own properties: every decode subset round-trips, every
     repair equals the encoded block (test/leo_erasure_tests.erl);
  4. committed fixtures (tests/golden/, restatement-derived) as a regression pin.
"""
import itertools
import json
import os

import numpy as np
import pytest

import restate_np as R

HERE = os.path.dirname(os.path.abspath(__file__))


def test_primitive_polynomials(oracle):
    """gf-complete default polynomials generate GF(2^w)* (x has order 2^w - 1)."""
    for w in range(2, 21):
        poly = oracle.prim_poly(w)
        assert poly >> w == 1
        x, order = 1, 0
        while True:
            x = oracle.gf_mul(x, 2, w)
            order += 1
            if x == 1:
                break
            assert order < (1 << w)
        assert order == (1 << w) - 1, w
    assert oracle.prim_poly(8) == 0x11D
    assert oracle.prim_poly(16) == 0x1100B
    assert oracle.prim_poly(32) == (1 << 32) | 0x400007


def test_field_known_values(oracle):
    assert oracle.gf_mul(0x80, 2, 8) == 0x1D
    assert oracle.gf_inv(2, 8) == 0x8E
    for w in (8, 16, 32):
        rng = np.random.default_rng(w)
        for _ in range(200):
            a, b, c = (int(x) for x in rng.integers(1, (1 << w) - 1, 3))
            assert oracle.gf_mul(a, b, w) == oracle.gf_mul(b, a, w)
            assert oracle.gf_mul(a, b ^ c, w) == oracle.gf_mul(a, b, w) ^ oracle.gf_mul(a, c, w)
            assert oracle.gf_mul(a, oracle.gf_inv(a, w), w) == 1


def test_vandermonde_kat(oracle):
    """SURVEY Appendix A.2 and the Jerasure manual example reed_sol_01 7 7 8."""
    C = oracle.vandermonde_coding_matrix(10, 4, 8)
    assert list(C[0]) == [1] * 10
    assert [hex(x) for x in C[1]] == "0x1 0x93 0x8a 0x49 0x5d 0xa1 0x67 0x3a 0x63 0xb2".split()
    assert [hex(x) for x in C[2]] == "0x1 0x67 0x9c 0x97 0x7b 0xbb 0xa6 0xaf 0xf4 0x53".split()
    assert [hex(x) for x in C[3]] == "0x1 0xdc 0xa6 0x7b 0x52 0x8f 0xf5 0x28 0xa7 0x7a".split()
    assert oracle.vandermonde_coding_matrix(4, 2, 8).tolist() == [[1, 1, 1, 1], [1, 70, 143, 200]]
    C7 = oracle.vandermonde_coding_matrix(7, 7, 8)
    assert C7[1].tolist() == [1, 199, 210, 240, 105, 121, 248]
    assert C7[2].tolist() == [1, 70, 91, 245, 56, 142, 167]


@pytest.mark.parametrize("k,m,w", [(4, 2, 8), (6, 2, 8), (8, 3, 8), (10, 4, 8), (4, 1, 8),
                                   (7, 7, 8), (12, 4, 8), (4, 2, 16), (10, 4, 16)])
def test_vandermonde_closed_form(oracle, k, m, w):
    """Elimination (Jerasure) == closed form normalise(V_bot V_top^-1)."""
    assert np.array_equal(oracle.vandermonde_coding_matrix(k, m, w),
                          R.vandermonde_closed_form(k, m, w))


def test_cbest_tables(oracle):
    """Jerasure cauchy_best_r6.c cbest_2..cbest_5 (recalled) == weight order."""
    recalled = {
        2: [1, 2, 3],
        3: [1, 2, 5, 4, 7, 3, 6],
        4: [1, 2, 9, 4, 8, 13, 3, 6, 12, 5, 11, 15, 10, 14, 7],
        5: [1, 2, 18, 4, 9, 8, 22, 16, 3, 11, 19, 5, 10, 6, 20, 27, 13, 23, 26, 12, 17, 25, 24,
            31, 30, 7, 15, 21, 29, 14, 28],
    }
    for w, row in recalled.items():
        assert oracle.cbest_row(w, len(row)).tolist() == row
    # cauchyrs default {4,2,3}: row 0 ones, row 1 = cbest_3[0..3]
    assert oracle.cauchy_good_general_coding_matrix(4, 2, 3).tolist() == [[1] * 4, [1, 2, 5, 4]]


def test_cauchy_good_kat(oracle):
    """cauchy_good(10,4,8) and its 888 bitmatrix ones."""
    C = oracle.cauchy_good_general_coding_matrix(10, 4, 8)
    assert [hex(x) for x in C[1]] == "0x97 0xac 0x1 0xe1 0xa6 0x9e 0x2c 0xd 0xe2 0x36".split()
    assert [hex(x) for x in C[2]] == "0x52 0x8f 0xc8 0xbe 0x97 0xd5 0xac 0xdc 0x1 0x38".split()
    assert [hex(x) for x in C[3]] == "0x1 0xac 0x7b 0x9e 0xc3 0x1f 0x8f 0xe3 0x52 0x22".split()
    assert oracle.matrix_to_bitmatrix(10, 4, 8, C).sum() == 888
    for k, m, w in [(10, 4, 8), (6, 3, 4), (10, 4, 10), (5, 3, 5)]:
        assert np.array_equal(oracle.cauchy_good_general_coding_matrix(k, m, w),
                              R.cauchy_improved(k, m, w)), (k, m, w)
        Cg = oracle.cauchy_good_general_coding_matrix(k, m, w)
        assert np.array_equal(oracle.matrix_to_bitmatrix(k, m, w, Cg), R.to_bitmatrix(Cg, w))


def test_n_ones(oracle):
    F = R.GF(8)
    for e in range(1, 256):
        assert oracle.cauchy_n_ones(e, 8) == R.bitmatrix_ones(F, e)


def test_liberation(oracle):
    for k, w in [(4, 7), (5, 5), (7, 7), (10, 11), (3, 13)]:
        B = oracle.liberation_coding_bitmatrix(k, w)
        assert np.array_equal(B, R.liberation(k, w))
        # minimum density: Q has k*w + k - 1 ones (Plank, "The RAID-6 Liberation codes")
        assert B[w:].sum() == k * w + k - 1
        # MDS: every pair of lost data blocks is recoverable from P and Q
        for a, b in itertools.combinations(range(k), 2):
            cols = list(range(a * w, (a + 1) * w)) + list(range(b * w, (b + 1) * w))
            assert R.rank_gf2(B[:, cols]) == 2 * w


def test_isal_cauchy1(oracle):
    A = oracle.isal_gen_cauchy1_matrix(14, 10)
    assert np.array_equal(A[:10], np.eye(10, dtype=np.uint8))
    assert np.array_equal(A[10:], R.isal_cauchy1(10, 4))
    inv = oracle.isal_invert_matrix(A[:10])
    assert np.array_equal(inv, np.eye(10, dtype=np.uint8))


@pytest.mark.parametrize("cls,k,m,w", [("vandrs", 10, 4, 8), ("isars", 10, 4, 8),
                                       ("vandrs", 8, 3, 16)])
def test_mds_every_subset(oracle, cls, k, m, w):
    """Every k-subset of [I; C] is invertible (all 1001 for RS(10,4))."""
    if cls == "vandrs":
        C = oracle.vandermonde_coding_matrix(k, m, w)
    else:
        C = oracle.isal_gen_cauchy1_matrix(k + m, k)[k:]
    F = R.GF(w)
    G = np.vstack([np.eye(k, dtype=np.int64), C.astype(np.int64)])
    for rows in itertools.combinations(range(k + m), k):
        F.invert(G[list(rows)])  # raises StopIteration if singular


SMALL = [("vandrs", 4, 2, 8), ("vandrs", 10, 4, 8), ("vandrs", 4, 2, 16), ("vandrs", 4, 2, 32),
         ("isars", 10, 4, 8), ("cauchyrs", 4, 2, 3), ("cauchyrs", 10, 4, 8),
         ("liberation", 4, 2, 7)]


@pytest.mark.parametrize("cfg", SMALL, ids=lambda c: "%s-%d-%d-%d" % c)
def test_oracle_roundtrip(oracle, cfg):
    """The reference's suite_test_/repair_test properties on the oracle."""
    cls, k, m, w = cfg
    data = np.random.default_rng(k * m * w).integers(0, 256, 9999, dtype=np.uint8).tobytes()
    blocks = oracle.encode(cls, k, m, w, data)
    bs = oracle.block_size(k, w, len(data))
    assert all(len(b) == bs for b in blocks) and b"".join(blocks[:k])[:len(data)] == data
    for lost in itertools.combinations(range(k + m), m):
        ids = [i for i in range(k + m) if i not in lost]
        assert oracle.decode(cls, k, m, w, [blocks[i] for i in ids], ids, len(data)) == data
        assert oracle.repair(cls, k, m, w, [blocks[i] for i in ids], ids, list(lost)) == \
            [blocks[i] for i in lost]


def test_geometry(oracle):
    """roundTo geometry (c_src/common.cpp:24-33, rscoding.cpp:44) — SURVEY §8a."""
    assert oracle.block_size(10, 8, 1048576) == 104960
    assert oracle.block_size(4, 8, 1048576) == 262144
    assert oracle.block_size(10, 8, 64 << 20) == 6710912
    assert oracle.block_size(10, 8, 10485760 + 1) == 1048704
    assert oracle.block_size(10, 8, 0) == 0


def test_golden_fixtures(oracle):
    """Restatement-derived fixtures (tests/golden/make_golden.py)."""
    with open(os.path.join(HERE, "golden", "index.json")) as fh:
        index = json.load(fh)
    assert index
    for ent in index:
        z = np.load(os.path.join(HERE, "golden", ent["file"]), allow_pickle=False)
        data = z["data"].tobytes()
        blocks = oracle.encode(ent["class"], ent["k"], ent["m"], ent["w"], data)
        assert b"".join(blocks) == z["blocks"].tobytes(), ent["file"]


def test_cpu_baseline_matches_oracle(oracle):
    """The cpu_baseline kernel (split-table PSHUFB) computes the same parity."""
    k, m, size, n = 10, 4, 100000, 3
    bs = oracle.block_size(k, 8, size)
    objs = np.random.default_rng(1).integers(0, 256, (n, size), dtype=np.uint8)
    levels = [1, 2] + ([3] if oracle.simd_level() >= 3 else [])   # 1 = scalar
    for force_scalar in levels:
        par = np.zeros((n, m * bs), dtype=np.uint8)
        oracle.bench_rs8(0, k, m, objs, size, size, n, par, threads=2, force_scalar=force_scalar)
        for o in range(n):
            ref = oracle.encode("vandrs", k, m, 8, objs[o].tobytes())
            assert par[o].tobytes() == b"".join(ref[k:])
        # in-place decode of data blocks {0,1,2,3} rebuilds the same bytes
        work = objs.copy()
        work[:, :4 * bs] = 0
        oracle.bench_rs8(1, k, m, work, size, size, n, par, erased=[0, 1, 2, 3], threads=2,
                         force_scalar=force_scalar)
        assert np.array_equal(work, objs)
