"""Latency of ONE host-memory encode call (the NIF's lone-caller path,
basho_bench ..._rs_10_4_8_1M_w_t1.config) under four stagings, RS(10,4,8)
1 MiB objects, median of N calls on one thread:

  pageable   leoec_encode (the shipped per-thread path: pageable
             hipMemcpyAsync in, kernel, pageable copy out)
  dma-pinned host memcpy into a pinned buffer, H2D, kernel, D2H into a
             pinned buffer, one stream sync, host memcpy out
  zero-copy  host memcpy into a pinned, device-mapped buffer; the kernel
             reads its inputs and writes its parity over PCIe directly
             (no DMA copy), one sync, host memcpy out
  zero-copy-wc  the same with a write-combined input buffer

Measurement only.  python tools/zerocopy_probe.py [calls]
"""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

K, M, W, SIZE = 10, 4, 8, 1 << 20


def main():
    import numpy as np
    import torch

    import leo_erasure_amd as le
    torch.cuda.set_device(0)
    assert le.gf_init() == "ok"
    L = le.lib
    hip = ctypes.CDLL("libamdhip64.so")
    bs, filled = le.layout("vandrs", (K, M, W), SIZE)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, SIZE, dtype=np.uint8)
    out_len = (K + M - filled) * bs
    ref = np.empty(out_len, dtype=np.uint8)
    assert L.leoec_encode(2, K, M, W, src.ctypes.data, SIZE, ref.ctypes.data, out_len) == 0
    par_ref = ref[(K - filled) * bs:]  # the m coding blocks

    def host_alloc(nbytes, flags):
        p = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flags)) == 0
        d = ctypes.c_void_p()
        assert hip.hipHostGetDevicePointer(ctypes.byref(d), p, ctypes.c_uint(0)) == 0
        return p.value, d.value

    stream = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(stream), ctypes.c_uint(1)) == 0
    MAPPED, WC = 0x2, 0x4
    in_h, in_d = host_alloc(SIZE + 4096, MAPPED)
    inwc_h, inwc_d = host_alloc(SIZE + 4096, MAPPED | WC)
    par_h, par_d = host_alloc(M * bs, MAPPED)
    dev_in = torch.empty(SIZE + 4096, dtype=torch.uint8, device="cuda")
    dev_par = torch.empty(M * bs, dtype=torch.uint8, device="cuda")
    out = np.empty(M * bs, dtype=np.uint8)

    def pageable():
        rc = L.leoec_encode(2, K, M, W, src.ctypes.data, SIZE, ref.ctypes.data, out_len)
        assert rc == 0

    def dma_pinned():
        ctypes.memmove(in_h, src.ctypes.data, SIZE)
        assert hip.hipMemcpyAsync(ctypes.c_void_p(dev_in.data_ptr()), ctypes.c_void_p(in_h),
                                  ctypes.c_size_t(SIZE), 1, stream) == 0
        assert L.leoec_encode_dev(2, K, M, W, dev_in.data_ptr(), SIZE + 4096, SIZE, 1,
                                  dev_par.data_ptr(), M * bs, stream) == 0
        assert hip.hipMemcpyAsync(ctypes.c_void_p(par_h), ctypes.c_void_p(dev_par.data_ptr()),
                                  ctypes.c_size_t(M * bs), 2, stream) == 0
        assert hip.hipStreamSynchronize(stream) == 0
        ctypes.memmove(out.ctypes.data, par_h, M * bs)

    def zero_copy(ih, idp):
        def f():
            ctypes.memmove(ih, src.ctypes.data, SIZE)
            assert L.leoec_encode_dev(2, K, M, W, idp, SIZE + 4096, SIZE, 1, par_d, M * bs,
                                      stream) == 0
            assert hip.hipStreamSynchronize(stream) == 0
            ctypes.memmove(out.ctypes.data, par_h, M * bs)
        return f

    def with_env(f, env):  # measurement build: a knob set for this form only
        def g():
            for k, v in env.items():
                le._lib.measure_set_knob(k, v)
            try:
                f()
            finally:
                for k in env:
                    le._lib.measure_set_knob(k, None)
        return g

    forms = [("pageable", pageable), ("dma-pinned", dma_pinned),
             ("zero-copy", zero_copy(in_h, in_d)), ("zero-copy-wc", zero_copy(inwc_h, inwc_d))]
    if le._lib.is_measure_build():
        forms.append(("zero-copy 64-lane tiles",
                      with_env(zero_copy(in_h, in_d), {"LEOEC_GF8_WG": "64"})))
    times = {name: [] for name, _ in forms}
    for name, f in forms:  # warm each form, check its parity
        for _ in range(20):
            f()
        if name != "pageable":
            assert np.array_equal(out, par_ref), name
            out[:] = 0
    for r in range(5):  # interleaved rounds
        for name, f in forms:
            for _ in range(n // 5):
                t0 = time.perf_counter()
                f()
                times[name].append(time.perf_counter() - t0)
    for name, _ in forms:
        t = sorted(times[name])
        med = statistics.median(t)
        print(json.dumps({"form": name, "us_median": round(med * 1e6, 1),
                          "us_p10_p90": [round(t[len(t) // 10] * 1e6, 1),
                                         round(t[9 * len(t) // 10] * 1e6, 1)],
                          "GiBps": round(SIZE / med / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
