"""The bench's PCIe link leg (bench.py GpuBackend.link_rates) in isolation,
against the same copies with the pinned buffers from hipHostMalloc instead
of torch's pinned allocator: does torch's `both` (56.5 GB/s, no duplex)
come from the buffers or from the streams?  Measurement only.

    python tools/link_torch.py [MiB]
"""
import ctypes
import sys

import torch


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = mib << 20
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    hip = ctypes.CDLL("libamdhip64.so")
    hsrc = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    hdst = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    dsrc = torch.empty(n, dtype=torch.uint8, device=dev)
    ddst = torch.empty(n, dtype=torch.uint8, device=dev)
    cur = torch.cuda.current_stream(dev)
    up, down = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)

    def torch_copies(h2d, d2h, reps=5):
        ms = []
        for i in range(reps + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(cur)
            for on, s, dst, src in ((h2d, up, ddst, hsrc), (d2h, down, hdst, dsrc)):
                if on:
                    s.wait_stream(cur)
                    with torch.cuda.stream(s):
                        dst.copy_(src, non_blocking=True)
                    cur.wait_stream(s)
            b.record(cur)
            torch.cuda.synchronize()
            if i:
                ms.append(a.elapsed_time(b))
        return (h2d + d2h) * n / (sorted(ms)[len(ms) // 2] * 1e-3) / 1e9

    # the same copies through hipMemcpyAsync on the torch streams, torch buffers
    H2D, D2H = 1, 2
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]

    def raw_copies(h2d, d2h, hs, hd, reps=5):
        import time
        ms = []
        for i in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if h2d:
                assert hip.hipMemcpyAsync(dsrc.data_ptr(), hs, n, H2D, up.cuda_stream) == 0
            if d2h:
                assert hip.hipMemcpyAsync(hd, ddst.data_ptr(), n, D2H, down.cuda_stream) == 0
            torch.cuda.synchronize()
            if i:
                ms.append((time.perf_counter() - t0) * 1e3)
        return (h2d + d2h) * n / (sorted(ms)[len(ms) // 2] * 1e-3) / 1e9

    # the same again on streams the HIP runtime creates for us (not torch's)
    raw_up, raw_down = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(raw_up), ctypes.c_uint(1)) == 0
    assert hip.hipStreamCreateWithFlags(ctypes.byref(raw_down), ctypes.c_uint(1)) == 0

    def raw_streams(h2d, d2h, reps=5):
        import time
        ms = []
        for i in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if h2d:
                assert hip.hipMemcpyAsync(dsrc.data_ptr(), hsrc.data_ptr(), n, H2D, raw_up) == 0
            if d2h:
                assert hip.hipMemcpyAsync(hdst.data_ptr(), ddst.data_ptr(), n, D2H, raw_down) == 0
            assert hip.hipStreamSynchronize(raw_up) == 0 and hip.hipStreamSynchronize(raw_down) == 0
            if i:
                ms.append((time.perf_counter() - t0) * 1e3)
        return (h2d + d2h) * n / (sorted(ms)[len(ms) // 2] * 1e-3) / 1e9

    print({"case": "hipMemcpyAsync on hipStreamCreateWithFlags streams, torch pinned buffers",
           "h2d_GBps": round(raw_streams(True, False), 1), "d2h_GBps": round(raw_streams(False, True), 1),
           "both_GBps": round(raw_streams(True, True), 1)}, flush=True)
    hm_src, hm_dst = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(hm_src), ctypes.c_size_t(n), ctypes.c_uint(2)) == 0
    assert hip.hipHostMalloc(ctypes.byref(hm_dst), ctypes.c_size_t(n), ctypes.c_uint(2)) == 0
    ctypes.memset(hm_src, 0x5A, n)
    ctypes.memset(hm_dst, 0, n)
    for name, fn in (("torch copy_ (bench.py)", lambda a, b: torch_copies(a, b)),
                     ("hipMemcpyAsync, torch pinned buffers",
                      lambda a, b: raw_copies(a, b, hsrc.data_ptr(), hdst.data_ptr())),
                     ("hipMemcpyAsync, hipHostMalloc buffers",
                      lambda a, b: raw_copies(a, b, hm_src.value, hm_dst.value))):
        print({"case": name, "h2d_GBps": round(fn(True, False), 1),
               "d2h_GBps": round(fn(False, True), 1), "both_GBps": round(fn(True, True), 1)},
              flush=True)


if __name__ == "__main__":
    main()
