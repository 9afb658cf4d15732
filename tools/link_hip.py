"""Two pinned 256 MiB copies (host->device, device->host) alone and at once
on two streams, through whichever HIP runtime the process loads: the system
runtime (/opt/rocm, what an Erlang VM loading the NIF gets) when run without
torch, the torch wheel's bundled runtime with --torch.  Measurement only:
does the bench's torch process lose the link's duplex to its runtime?

    python tools/link_hip.py [--torch] [MiB]
"""
import ctypes
import os
import sys
import time


def main():
    use_torch = "--torch" in sys.argv
    args = [a for a in sys.argv[1:] if a != "--torch"]
    mib = int(args[0]) if args else 256
    if use_torch:
        import torch
        torch.cuda.init()
        hip = ctypes.CDLL("libamdhip64.so")
    else:
        hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    n = mib << 20
    vp = ctypes.c_void_p
    hip.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    hip.hipStreamSynchronize.argtypes = [vp]
    assert hip.hipSetDevice(0) == 0
    hs, hd, ds, dd = vp(), vp(), vp(), vp()
    for p in (hs, hd):
        assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(n), ctypes.c_uint(2)) == 0
    for p in (ds, dd):
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n)) == 0
    ctypes.memset(hs, 0x5A, n)
    ctypes.memset(hd, 0, n)
    up, down = vp(), vp()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(up), ctypes.c_uint(1)) == 0
    assert hip.hipStreamCreateWithFlags(ctypes.byref(down), ctypes.c_uint(1)) == 0

    def timed(h2d, d2h, reps=5):
        ms = []
        for i in range(reps + 1):
            t0 = time.perf_counter()
            if h2d:
                assert hip.hipMemcpyAsync(ds, hs, n, 1, up) == 0
            if d2h:
                assert hip.hipMemcpyAsync(hd, dd, n, 2, down) == 0
            assert hip.hipStreamSynchronize(up) == 0 and hip.hipStreamSynchronize(down) == 0
            if i:
                ms.append((time.perf_counter() - t0) * 1e3)
        return round((h2d + d2h) * n / (sorted(ms)[len(ms) // 2] * 1e-3) / 1e9, 1)

    env = {k: v for k, v in os.environ.items() if k.startswith(("HSA_", "HIP_", "GPU_", "ROC", "AMD_"))}
    print({"runtime": "torch-bundled" if use_torch else "system /opt/rocm",
           "h2d_GBps": timed(True, False), "d2h_GBps": timed(False, True),
           "both_GBps": timed(True, True), "env": env}, flush=True)


if __name__ == "__main__":
    main()
