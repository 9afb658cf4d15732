"""ctypes binding of the CPU oracle (oracle/leoec_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product package (leo_erasure_amd) never
imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")

CAUCHYRS, VANDRS, LIBERATION, ISARS = 1, 2, 3, 4
CLASS_IDS = {"cauchyrs": CAUCHYRS, "vandrs": VANDRS, "liberation": LIBERATION, "isars": ISARS}

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.orc_prim_poly.restype = ctypes.c_uint64
        L.orc_gf_mul.restype = ctypes.c_uint32
        L.orc_gf_mul.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
        L.orc_gf_inv.restype = ctypes.c_uint32
        L.orc_gf_inv.argtypes = [ctypes.c_uint32, ctypes.c_int]
        L.orc_gf_div.restype = ctypes.c_uint32
        L.orc_gf_div.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
        L.orc_block_size.restype = ctypes.c_uint64
        L.orc_block_size.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64]
        L.orc_cauchy_n_ones.argtypes = [ctypes.c_uint32, ctypes.c_int]
        for fn in ("orc_vandermonde_coding_matrix", "orc_cauchy_original_coding_matrix",
                   "orc_cauchy_good_general_coding_matrix"):
            getattr(L, fn).argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u32p]
        L.orc_cbest_row.argtypes = [ctypes.c_int, ctypes.c_int, u32p]
        L.orc_liberation_coding_bitmatrix.argtypes = [ctypes.c_int, ctypes.c_int, u8p]
        L.orc_matrix_to_bitmatrix.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u32p, u8p]
        L.orc_isal_gen_cauchy1_matrix.argtypes = [ctypes.c_int, ctypes.c_int, u8p]
        L.orc_isal_invert_matrix.argtypes = [u8p, u8p, ctypes.c_int]
        L.orc_check_params.argtypes = [ctypes.c_int] * 4
        L.orc_encode.argtypes = [ctypes.c_int] * 4 + [ctypes.c_char_p, ctypes.c_uint64, u8p]
        L.orc_decode.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_char_p),
                                                      ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                                      ctypes.c_uint64, ctypes.c_uint64, u8p]
        L.orc_repair.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_char_p),
                                                      ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                                      ctypes.c_uint64, ctypes.POINTER(ctypes.c_int),
                                                      ctypes.c_int, u8p]
        L.orc_bench_rs8_pinned.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
            ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int,
            ctypes.POINTER(ctypes.c_int), ctypes.c_double, ctypes.c_double, ctypes.c_int,
            ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
            ctypes.POINTER(ctypes.c_double), ctypes.c_double, ctypes.POINTER(ctypes.c_double),
            ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.orc_bench_rs8.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int]
        _lib = L
    return _lib


def _u32(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def _u8(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


class OracleError(Exception):
    def __init__(self, code):
        super().__init__(code)
        self.code = code


def _chk(rc):
    if rc != 0:
        raise OracleError(rc)


def prim_poly(w):
    return lib().orc_prim_poly(w)


def gf_mul(a, b, w):
    return lib().orc_gf_mul(a, b, w)


def gf_inv(a, w):
    return lib().orc_gf_inv(a, w)


def gf_div(a, b, w):
    return lib().orc_gf_div(a, b, w)


def block_size(k, w, size):
    return lib().orc_block_size(k, w, size)


def vandermonde_coding_matrix(k, m, w):
    out = np.zeros(m * k, dtype=np.uint32)
    _chk(lib().orc_vandermonde_coding_matrix(k, m, w, _u32(out)))
    return out.reshape(m, k)


def cauchy_original_coding_matrix(k, m, w):
    out = np.zeros(m * k, dtype=np.uint32)
    _chk(lib().orc_cauchy_original_coding_matrix(k, m, w, _u32(out)))
    return out.reshape(m, k)


def cauchy_good_general_coding_matrix(k, m, w):
    out = np.zeros(m * k, dtype=np.uint32)
    _chk(lib().orc_cauchy_good_general_coding_matrix(k, m, w, _u32(out)))
    return out.reshape(m, k)


def cauchy_n_ones(n, w):
    return lib().orc_cauchy_n_ones(n, w)


def cbest_row(w, k):
    out = np.zeros(k, dtype=np.uint32)
    _chk(lib().orc_cbest_row(w, k, _u32(out)))
    return out


def liberation_coding_bitmatrix(k, w):
    out = np.zeros(2 * w * k * w, dtype=np.uint8)
    _chk(lib().orc_liberation_coding_bitmatrix(k, w, _u8(out)))
    return out.reshape(2 * w, k * w)


def matrix_to_bitmatrix(k, m, w, mat):
    mat = np.ascontiguousarray(mat, dtype=np.uint32).reshape(-1)
    out = np.zeros(m * w * k * w, dtype=np.uint8)
    _chk(lib().orc_matrix_to_bitmatrix(k, m, w, _u32(mat), _u8(out)))
    return out.reshape(m * w, k * w)


def isal_gen_cauchy1_matrix(rows, k):
    out = np.zeros(rows * k, dtype=np.uint8)
    _chk(lib().orc_isal_gen_cauchy1_matrix(rows, k, _u8(out)))
    return out.reshape(rows, k)


def isal_invert_matrix(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    n = a.shape[0]
    out = np.zeros((n, n), dtype=np.uint8)
    _chk(lib().orc_isal_invert_matrix(_u8(a), _u8(out), n))
    return out


def check_params(coding, k, m, w):
    return lib().orc_check_params(CLASS_IDS.get(coding, -1) if isinstance(coding, str) else coding,
                                  k, m, w)


def _cls(coding):
    return CLASS_IDS.get(coding, -1) if isinstance(coding, str) else coding


def encode(coding, k, m, w, data):
    """NIF encode/4 semantics: list of k+m blocks (bytes)."""
    data = bytes(data)
    rc = check_params(coding, k, m, w)
    _chk(rc)
    bs = block_size(k, w, len(data))
    out = np.zeros((k + m) * bs + 1, dtype=np.uint8)
    _chk(lib().orc_encode(_cls(coding), k, m, w, data, len(data), _u8(out)))
    return [out[i * bs:(i + 1) * bs].tobytes() for i in range(k + m)]


def decode(coding, k, m, w, blocks, ids, size):
    n = len(blocks)
    bs = len(blocks[-1]) if blocks else 0
    arr = (ctypes.c_char_p * max(n, 1))(*[bytes(b) for b in blocks])
    idv = (ctypes.c_int * max(n, 1))(*ids)
    out = np.zeros(size + 1, dtype=np.uint8)
    _chk(lib().orc_decode(_cls(coding), k, m, w, arr, idv, n, bs, size, _u8(out)))
    return out[:size].tobytes()


def repair(coding, k, m, w, blocks, ids, rep):
    n = len(blocks)
    bs = len(blocks[-1]) if blocks else 0
    arr = (ctypes.c_char_p * max(n, 1))(*[bytes(b) for b in blocks])
    idv = (ctypes.c_int * max(n, 1))(*ids)
    repv = (ctypes.c_int * max(len(rep), 1))(*rep)
    out = np.zeros(len(rep) * bs + 1, dtype=np.uint8)
    _chk(lib().orc_repair(_cls(coding), k, m, w, arr, idv, n, bs, repv, len(rep), _u8(out)))
    return [out[i * bs:(i + 1) * bs].tobytes() for i in range(len(rep))]


def bench_rs8(op, k, m, objs, obj_stride, size, nobj, parity, erased=(), threads=1,
              force_scalar=False):
    """CPU baseline driver (ISA-L split-table technique).  objs/parity: numpy uint8."""
    er = (ctypes.c_int * max(len(erased), 1))(*erased)
    _chk(lib().orc_bench_rs8(op, k, m, objs.ctypes.data, obj_stride, size, nobj,
                             parity.ctypes.data, er, len(erased), threads, int(force_scalar)))


def bench_rs8_pinned(k, m, objs, size, erased, threads, cpus, pass_s, total_s, min_passes=3,
                     max_passes=256, parity_out=None, structure=0, throttled=None,
                     warm_s=0.0, warmup=None):
    """bench.py's timed CPU baseline: workers pinned to `cpus`, each
    first-touching its own slice of `objs` (n x stride numpy uint8), passes of
    >= pass_s seconds of encode + in-place decode of `erased`; returns the
    per-pass GiB/s (oracle/leoec_oracle.c orc_bench_rs8_pinned).
    structure 0: ISA-L's one pass per object; 1: Jerasure's per-(row, input)
    region passes (rscoding.cpp:71 / :147); 2: the one pass with scalar
    table lookups (SURVEY §8(d)'s scalar reference).  `throttled`, a list, receives the
    cgroup's CFS-throttled seconds per pass (None where unreadable).
    warm_s > 0: untimed warm-up passes first, until two consecutive ones agree
    within 3 % or warm_s has elapsed; `warmup`, a list, receives their rates."""
    L = lib()
    n, stride = objs.shape[0], objs.strides[0]
    rates = (ctypes.c_double * max_passes)()
    thr = (ctypes.c_double * max_passes)()
    er = (ctypes.c_int * max(len(erased), 1))(*erased)
    cp = (ctypes.c_int * max(len(cpus), 1))(*cpus) if cpus else None
    po = parity_out.ctypes.data if parity_out is not None else None
    wr = (ctypes.c_double * 64)()
    nw = ctypes.c_int(0)
    rc = L.orc_bench_rs8_pinned(k, m, objs.ctypes.data, stride, size, n, er, len(erased), threads,
                                cp, float(pass_s), float(total_s), min_passes, rates, max_passes,
                                po, int(structure), thr, float(warm_s), wr, 64, ctypes.byref(nw))
    if rc < 0:
        _chk(rc)
    if warmup is not None:
        warmup[:] = list(wr[:nw.value])
    if throttled is not None:
        throttled[:] = [None if t < 0 else t for t in thr[:rc]]
    return list(rates[:rc])


def simd_level():
    return lib().orc_simd_level()
