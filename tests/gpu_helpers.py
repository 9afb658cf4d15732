"""Shared helpers of the GPU parity tests (test_gpu_parity.py, product
library) and the measurement-form tests (test_measure_forms.py, their own
process with LEOEC_LIBRARY=measure)."""
import ctypes

import numpy as np


def rand_bytes(n, seed):
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, n, dtype=np.uint8).tobytes()


def batch(gpu, n, size, stride, seed):
    """n random rows of `stride` bytes, host copy and device copy."""
    rng = np.random.Generator(np.random.PCG64(seed))
    host = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    return host, gpu.from_numpy(host).cuda()


def capi_case(le, oracle, cls, k, m, w, size, seed):
    """Inputs and oracle answers for one object, as numpy buffers for the C ABI."""
    data = np.frombuffer(rand_bytes(size, seed), dtype=np.uint8).copy()
    ref = oracle.encode(cls, k, m, w, data.tobytes())
    bs, filled = le.layout(cls, (k, m, w), size)
    return {"cls": cls, "cid": le._lib.CODING_IDS[cls], "p": (k, m, w), "size": size, "bs": bs,
            "filled": filled, "data": data, "ref": ref,
            "blocks": [np.frombuffer(b, dtype=np.uint8).copy() for b in ref]}


def capi_ops(le, c, t):
    """encode, decode (m blocks lost) and repair (2 blocks) of one case
    through the C ABI, each independent of the others' outcome (decode and
    repair read the oracle's blocks).  Returns {op: (rc, equal, detail)}."""
    L = le.lib
    k, m, w = c["p"]
    bs, filled, size = c["bs"], c["filled"], c["size"]
    res = {}
    out = np.empty(max((k + m - filled) * bs, 1), dtype=np.uint8)
    rc = L.leoec_encode(c["cid"], k, m, w, c["data"].ctypes.data, size, out.ctypes.data, out.size)
    res["encode"] = (rc, b"".join(c["ref"][filled:]) == out[:(k + m - filled) * bs].tobytes(),
                     f"{c['cls']}{c['p']} size {size}")
    lost = sorted({(t * 7 + j * 3) % (k + m) for j in range(m)})
    ids = [b for b in range(k + m) if b not in lost][::-1]
    ptrs = (ctypes.c_void_p * len(ids))(*[c["blocks"][b].ctypes.data for b in ids])
    idv = (ctypes.c_int * len(ids))(*ids)
    dec = np.empty(max(size, 1), dtype=np.uint8)
    rc = L.leoec_decode(c["cid"], k, m, w, ptrs, idv, len(ids), bs, size, dec.ctypes.data)
    res["decode"] = (rc, bool(np.array_equal(dec[:size], c["data"])),
                     f"{c['cls']}{c['p']} lost {lost}")
    res["decode_lost_data"] = any(b < k for b in lost)
    rep = sorted({t % (k + m), (t + 5) % (k + m)})
    avail = [b for b in range(k + m) if b not in rep]
    ptrs = (ctypes.c_void_p * len(avail))(*[c["blocks"][b].ctypes.data for b in avail])
    idv = (ctypes.c_int * len(avail))(*avail)
    repv = (ctypes.c_int * len(rep))(*rep)
    ro = np.empty(len(rep) * bs, dtype=np.uint8)
    rc = L.leoec_repair(c["cid"], k, m, w, ptrs, idv, len(avail), bs, repv, len(rep),
                        ro.ctypes.data)
    res["repair"] = (rc, ro.tobytes() == b"".join(c["ref"][b] for b in rep),
                     f"{c['cls']}{c['p']} {rep}")
    return res


def capi_roundtrip(le, c, t):
    """capi_ops; returns the first failing op as an error string, or None."""
    res = capi_ops(le, c, t)
    for op in ("encode", "decode", "repair"):
        rc, eq, detail = res[op]
        if rc or not eq:
            return f"{op} {detail} rc {rc}"
    return None


MIXED_SPECS = [("vandrs", 10, 4, 8, 1048576), ("vandrs", 10, 4, 8, 1048576),
               ("vandrs", 10, 4, 8, 300001), ("cauchyrs", 10, 4, 8, 1048576 + 77),
               ("isars", 10, 4, 8, 65536 + 7), ("liberation", 4, 2, 7, 777777),
               ("vandrs", 4, 2, 16, 123457), ("vandrs", 6, 3, 32, 99999),
               ("vandrs", 10, 4, 8, 9 << 20), ("cauchyrs", 4, 2, 3, 5000),
               ("vandrs", 20, 6, 8, 2000003)]


def mixed_callers(le, oracle, fail_bs=None, threads=24, rounds=8):
    """Cross-call batching (hostq.cpp): `threads` threads call the C ABI at
    once with mixed classes, widths, sizes (ragged, and 9 MiB objects above
    the batch cap, which take the per-thread path) and erasure patterns, so
    one batch holds several different maps (several launches) and identical
    maps are merged into one launch.  Every result must equal the oracle's.
    fail_bs (measurement build, LEOEC_HOSTQ_FAIL_BS): the batched launches of
    that block size report a HIP error; exactly those calls must fail with
    LEOEC_E_HIP — the encode, the repair, and the decode when it has a data
    block to rebuild — while every other call in the same batches succeeds.
    Returns the list of errors (empty: pass) and the number of injected
    failures seen."""
    import concurrent.futures as cf
    cases = [capi_case(le, oracle, *sp, seed=100 + i) for i, sp in enumerate(MIXED_SPECS)]
    E_HIP = le._lib.E_HIP

    def worker(t):
        failed = 0
        for r in range(rounds):
            c = cases[(t + r) % len(cases)]
            res = capi_ops(le, c, t + r)
            for op in ("encode", "decode", "repair"):
                rc, eq, detail = res[op]
                inject = fail_bs is not None and c["bs"] == fail_bs and (
                    op != "decode" or res["decode_lost_data"])
                if inject:
                    if rc != E_HIP:
                        return f"thread {t}: {op} {detail}: expected the injected failure, rc {rc}", 0
                    failed += 1
                elif rc or not eq:
                    return f"thread {t}: {op} {detail} rc {rc}", 0
        return None, failed

    with cf.ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(worker, range(threads)))
    return [e for e, _ in res if e], sum(f for _, f in res)
