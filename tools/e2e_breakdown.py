"""Where the time of one NIF-path encode goes (RS(10,4,8), 1 MiB object):
each piece of leoec_encode's host path timed on its own, wall clock, median
of 200 after warm-up.  Pieces: pageable / pinned H2D of the object, one
encode launch on a single device-resident object (+ sync), pageable / pinned
D2H of the parity, and the whole leoec_encode call.

    python tools/e2e_breakdown.py
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def med_us(fn, n=200, warm=20):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def main():
    import numpy as np
    import torch

    import leo_erasure_amd as le
    torch.cuda.set_device(0)
    assert le.gf_init() == "ok"
    K, M, W, size = 10, 4, 8, 1 << 20
    bs, filled = le.layout("vandrs", (K, M, W), size)
    s = torch.cuda.Stream()
    host = torch.from_numpy(np.random.default_rng(1).integers(0, 256, size, dtype=np.uint8))
    hpin = host.pin_memory()
    dev = torch.empty(size, dtype=torch.uint8, device="cuda")
    dpar = torch.empty((1, M * bs), dtype=torch.uint8, device="cuda")
    hpar = torch.empty(M * bs, dtype=torch.uint8)
    hpar_pin = hpar.pin_memory()
    out = {}

    def h2d(src):
        def f():
            with torch.cuda.stream(s):
                dev.copy_(src, non_blocking=True)
            s.synchronize()
        return f

    def d2h(dst):
        def f():
            with torch.cuda.stream(s):
                dst.copy_(dpar[0], non_blocking=True)
            s.synchronize()
        return f

    def kern():
        le.device.encode("vandrs", (K, M, W), dev.view(1, size), size, dpar, stream=s.cuda_stream)
        s.synchronize()

    out["h2d_pageable_1MiB"] = med_us(h2d(host))
    out["h2d_pinned_1MiB"] = med_us(h2d(hpin))
    out["encode_launch_1obj_sync"] = med_us(kern)
    out["d2h_pageable_420KB"] = med_us(d2h(hpar))
    out["d2h_pinned_420KB"] = med_us(d2h(hpar_pin))
    out["empty_sync"] = med_us(lambda: s.synchronize())
    a = np.empty(size, dtype=np.uint8)
    out["host_memcpy_1MiB"] = med_us(lambda: np.copyto(a, host.numpy()))
    src = host.numpy()
    bsz = (K + M - filled) * bs
    o = np.empty(bsz, dtype=np.uint8)
    out["leoec_encode_call"] = med_us(lambda: le.lib.leoec_encode(
        2, K, M, W, src.ctypes.data, size, o.ctypes.data, bsz))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
