"""The reference's own encode benchmark, on this engine.

bench_encode_test (test/leo_erasure_tests.erl:207-212, 304-336): one encode
of a 100 MiB all-zero binary per class — vandrs{10,4,8}, cauchyrs{10,4,10},
liberation{10,2,11}, isars{10,4,8} — timed around the call with
os:timestamp, rate = 100 / seconds ("MB/s", i.e. MiB/s).  The reference
prints the number and records none.

Here the same call goes through the C ABI leoec_encode (the NIF's entry
point, host memory in and out) from one caller thread, as the eunit test
calls it: the first call of the class (`cold`: the reference's single
measurement; the first class also pays this thread's staging allocation)
and the median of `--reps` further calls (`warm`).  Every output is checked
(the code is linear: all-zero input, all-zero tail block and parity).
Beside it, what bounds the call: the same object encoded in HBM
(leoec_encode_dev, one launch), and torch's H2D of the 100 MiB object / D2H
of the parity from pageable and from pinned memory.  `--forms` adds the
measurement build's staging forms at 100 MiB (LEOEC_HOST_STAGING).

    python tools/ref_encode_bench.py [--reps 5] [--forms]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CLASSES = [("vandrs", (10, 4, 8)), ("cauchyrs", (10, 4, 10)), ("liberation", (10, 2, 11)),
           ("isars", (10, 4, 8))]
CID = {"cauchyrs": 1, "vandrs": 2, "liberation": 3, "isars": 4}
MiB = 1 << 20
SIZE = 100 * MiB


def host_call(le, cls, params, src, out):
    k, m, w = params
    t0 = time.perf_counter()
    rc = le.lib.leoec_encode(CID[cls], k, m, w, src.ctypes.data, SIZE, out.ctypes.data, out.size)
    dt = time.perf_counter() - t0
    assert rc == 0, (cls, rc)
    return dt


def ref_rate(dt):
    """the eunit test's rate: 100 / seconds (its "MB/s" is MiB/s)."""
    return round(100.0 / dt, 1)


def host_path(le, np, reps, tag):
    res = []
    for cls, params in CLASSES:
        k, m, w = params
        bs, filled = le.layout(cls, params, SIZE)
        # the eunit test's <<0:ChunkSizeBits>> is a fresh, zero-written binary:
        # written here too (np.zeros would leave the pages untouched, and the
        # first copy would pay their faults)
        src = np.full(SIZE, 0, dtype=np.uint8)
        out = np.full((k + m - filled) * bs, 0xA5, dtype=np.uint8)
        cold = host_call(le, cls, params, src, out)
        assert not out.any(), f"{cls}: non-zero output for an all-zero object"
        warm = []
        for _ in range(reps):
            out[:] = 0xA5
            warm.append(host_call(le, cls, params, src, out))
            assert not out.any(), f"{cls}: non-zero output for an all-zero object"
        med = statistics.median(warm)
        rec = {"bench": "reference bench_encode_test, C ABI leoec_encode, 1 caller",
               "form": tag, "class": cls, "params": list(params), "block_size": bs,
               "cold_ms": round(cold * 1e3, 2), "cold_MiBps": ref_rate(cold),
               "warm_ms": round(med * 1e3, 2), "warm_MiBps": ref_rate(med),
               "warm_ms_all": [round(x * 1e3, 2) for x in warm],
               "link_bytes": SIZE + m * bs}
        print(json.dumps(rec), flush=True)
        res.append(rec)
    return res


def device_path(le, torch, reps):
    for cls, params in CLASSES:
        k, m, w = params
        bs, _ = le.layout(cls, params, SIZE)
        obj = torch.zeros((1, k * bs), dtype=torch.uint8, device="cuda")
        par = torch.empty((1, m * bs), dtype=torch.uint8, device="cuda")
        fn = lambda: le.device.encode(cls, params, obj, SIZE, par)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        ts = []
        for _ in range(reps * 4):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            fn()
            b.record(s)
            ts.append((a, b))
        torch.cuda.synchronize()
        ms = statistics.median(a.elapsed_time(b) for a, b in ts)
        assert not par.any()
        print(json.dumps({"bench": "same object resident in HBM, leoec_encode_dev (1 object)",
                          "class": cls, "params": list(params), "ms": round(ms, 4),
                          "MiBps": ref_rate(ms / 1e3),
                          "frac_of_8TBps": round((k + m) * bs / ms / 1e6 / 8000.0, 4)}),
              flush=True)


def copies(le, torch, reps):
    """torch H2D of the 100 MiB object and D2H of RS(10,4,8)'s parity, pageable and pinned."""
    par_bytes = 4 * le.layout("vandrs", (10, 4, 8), SIZE)[0]
    for pinned in (False, True):
        h = torch.zeros(SIZE, dtype=torch.uint8)
        hp = torch.empty(par_bytes, dtype=torch.uint8)
        if pinned:
            h, hp = h.pin_memory(), hp.pin_memory()
        d = torch.empty(SIZE, dtype=torch.uint8, device="cuda")
        dp = torch.zeros(par_bytes, dtype=torch.uint8, device="cuda")
        for name, fn, n in (("H2D 100 MiB", lambda: d.copy_(h), SIZE),
                            ("D2H parity 40 MiB", lambda: hp.copy_(dp), par_bytes)):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            t = statistics.median(ts)
            print(json.dumps({"bench": "torch copy", "what": name,
                              "host": "pinned" if pinned else "pageable",
                              "ms": round(t * 1e3, 2), "GBps": round(n / t / 1e9, 2)}), flush=True)


def registered(torch, np, reps):
    """hipHostRegister of a pageable 100 MiB buffer in place (what a large
    call could do instead of bounce-buffer copies): the register and
    unregister costs, and the H2D rate from the registered pages."""
    rt = torch.cuda.cudart()
    h = np.zeros(SIZE, dtype=np.uint8)
    d = torch.empty(SIZE, dtype=torch.uint8, device="cuda")
    reg, unreg, h2d = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        rc = rt.cudaHostRegister(h.ctypes.data, SIZE, 0)
        t1 = time.perf_counter()
        code = int(getattr(rc, "value", rc))
        if code != 0:
            print(json.dumps({"bench": "hipHostRegister", "error": code}), flush=True)
            return
        ht = torch.from_numpy(h)
        d.copy_(ht, non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rt.cudaHostUnregister(h.ctypes.data)
        t3 = time.perf_counter()
        reg.append(t1 - t0)
        h2d.append(t2 - t1)
        unreg.append(t3 - t2)
    print(json.dumps({"bench": "hipHostRegister of a pageable 100 MiB buffer",
                      "register_ms": round(statistics.median(reg) * 1e3, 2),
                      "h2d_ms": round(statistics.median(h2d) * 1e3, 2),
                      "h2d_GBps": round(SIZE / statistics.median(h2d) / 1e9, 2),
                      "unregister_ms": round(statistics.median(unreg) * 1e3, 2)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--forms", action="store_true")
    ap.add_argument("--cold-only", action="store_true",
                    help="gf_init and the first / warm calls only (a short target for a trace)")
    args = ap.parse_args()
    import numpy as np
    import torch
    if args.forms:
        os.environ.setdefault("LEOEC_LIBRARY", "measure")
    import leo_erasure_amd as le
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    assert le.gf_init() == "ok"
    print(json.dumps({"bench": "gf_init", "ms": round((time.perf_counter() - t0) * 1e3, 2)}),
          flush=True)
    host_path(le, np, args.reps, "default")
    if args.cold_only:
        return
    device_path(le, torch, args.reps)
    copies(le, torch, args.reps)
    registered(torch, np, args.reps)
    if args.forms:
        for tag, env in (("pinned ring 4 MiB", {"LEOEC_HOST_STAGING": "pinned",
                                                "LEOEC_STAGE_CHUNK_KIB": "4096"}),
                         ("pinned ring 8 MiB", {"LEOEC_HOST_STAGING": "pinned",
                                                "LEOEC_STAGE_CHUNK_KIB": "8192"}),
                         ("default again", {})):
            le._lib.measure_reset_knobs()
            for k, v in env.items():
                le._lib.measure_set_knob(k, v)
            host_path(le, np, args.reps, tag)
        le._lib.measure_reset_knobs()


if __name__ == "__main__":
    main()
