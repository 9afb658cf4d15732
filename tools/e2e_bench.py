"""End-to-end (host memory) encode rates, RS(10,4,8) 1 MiB objects.

The reference path starts and ends in host memory (Erlang binaries), so the
PCIe-inclusive rate is recorded in DESIGN.md (never as the bench value):

  nif    leoec_encode() per object from pageable memory (the NIF path:
         H2D object, kernel, D2H parity, synchronous), 1 thread;
  pinned batched: pinned host objects -> H2D -> leoec_encode_dev -> D2H
         parity, chunks of `chunk` objects double-buffered on two streams.

    python tools/e2e_bench.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def host_paths(le, K, M, W, size, bs, filled, tag):
    import threading

    import numpy as np
    # --- NIF path, pageable, one object per call
    data = np.random.default_rng(1).integers(0, 256, size, dtype=np.uint8).tobytes()
    for _ in range(3):
        le.nif_encode("vandrs", (K, M, W), data, size)
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        st, _ = le.nif_encode("vandrs", (K, M, W), data, size)
        assert st == "ok"
    t = time.perf_counter() - t0
    print(json.dumps({"path": f"nif leoec_encode, 1 object/call, 1 thread [{tag}]",
                      "GiBps": round(n * size / t / 2**30, 2), "us_per_object": round(t / n * 1e6, 1)}))

    # --- NIF decode, data blocks {0,1,2,3} lost (rebuilt on the GPU), 1 thread
    st, blocks = le.nif_encode("vandrs", (K, M, W), data, size)
    ids = list(range(4, K + M))
    surv = [blocks[i] for i in ids]
    for _ in range(3):
        le.nif_decode("vandrs", (K, M, W), surv, ids, size)
    t0 = time.perf_counter()
    for _ in range(n):
        st, out = le.nif_decode("vandrs", (K, M, W), surv, ids, size)
        assert st == "ok"
    t = time.perf_counter() - t0
    assert out == data
    print(json.dumps({"path": f"nif leoec_decode (lose 0-3), 1 object/call, 1 thread [{tag}]",
                      "GiBps": round(n * size / t / 2**30, 2), "us_per_object": round(t / n * 1e6, 1)}))

    # --- C ABI leoec_encode (host memory), T concurrent callers (dirty schedulers)
    bsz = (K + M - filled) * bs
    for T in (1, 4, 8, 16):
        per = 64
        srcs = [np.random.default_rng(t).integers(0, 256, size, dtype=np.uint8) for t in range(T)]
        outs = [np.empty(bsz, dtype=np.uint8) for _ in range(T)]

        ready = threading.Barrier(T + 1)
        go = threading.Event()

        def work(t):
            # warm this thread's stream / staging buffers outside the timed region
            rc = le.lib.leoec_encode(2, K, M, W, srcs[t].ctypes.data, size, outs[t].ctypes.data, bsz)
            assert rc == 0
            ready.wait()
            go.wait()
            for _ in range(per):
                rc = le.lib.leoec_encode(2, K, M, W, srcs[t].ctypes.data, size, outs[t].ctypes.data, bsz)
                assert rc == 0

        ths = [threading.Thread(target=work, args=(t,)) for t in range(T)]
        for th in ths:
            th.start()
        ready.wait()
        t0 = time.perf_counter()
        go.set()
        for th in ths:
            th.join()
        t = time.perf_counter() - t0
        print(json.dumps({"path": f"C ABI leoec_encode, 1 MiB objects, {T} caller threads [{tag}]",
                          "GiBps": round(T * per * size / t / 2**30, 2),
                          "us_per_object_per_thread": round(t / per * 1e6, 1)}))



def main():
    import numpy as np
    import torch

    import leo_erasure_amd as le
    torch.cuda.set_device(0)
    assert le.gf_init() == "ok"
    K, M, W, size = 10, 4, 8, 1 << 20
    bs, filled = le.layout("vandrs", (K, M, W), size)

    # Host staging forms of the host entry points (engine.cpp): the pinned
    # ring at several chunk sizes, and plain pageable copies.
    forms = [("auto", "256"), ("pageable", "256"), ("gather", "256"), ("pinned", "1024")]
    if len(sys.argv) > 1 and sys.argv[1] == "--quick":
        forms = [("auto", "256"), ("pageable", "256")]
    for staging, ck in forms:
        os.environ["LEOEC_HOST_STAGING"] = staging
        os.environ["LEOEC_STAGE_CHUNK_KIB"] = ck
        host_paths(le, K, M, W, size, bs, filled, f"{staging}/{ck}KiB")

    # --- pinned, batched, two streams
    total, chunk = 1024, 64
    host = torch.randint(0, 256, (total, size), dtype=torch.uint8).pin_memory()
    hpar = torch.empty((total, M * bs), dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dobj = [torch.empty((chunk, size), dtype=torch.uint8, device="cuda") for _ in streams]
    dpar = [torch.empty((chunk, M * bs), dtype=torch.uint8, device="cuda") for _ in streams]

    def run():
        for i, c0 in enumerate(range(0, total, chunk)):
            s = streams[i % 2]
            with torch.cuda.stream(s):
                dobj[i % 2].copy_(host[c0:c0 + chunk], non_blocking=True)
                le.device.encode("vandrs", (K, M, W), dobj[i % 2], size, dpar[i % 2],
                                 stream=s.cuda_stream)
                hpar[c0:c0 + chunk].copy_(dpar[i % 2], non_blocking=True)
        torch.cuda.synchronize()

    run()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        run()
    t = (time.perf_counter() - t0) / reps
    h2d = total * size
    d2h = total * M * bs
    print(json.dumps({"path": "pinned batched H2D+encode+D2H (2 streams, 64-object chunks)",
                      "GiBps_payload": round(total * size / t / 2**30, 2),
                      "pcie_GBps": round((h2d + d2h) / t / 1e9, 2), "ms": round(t * 1e3, 2)}))
    # spot-check one object's parity against a fresh device encode
    dev = host[:1].cuda()
    p = torch.empty((1, M * bs), dtype=torch.uint8, device="cuda")
    le.device.encode("vandrs", (K, M, W), dev, size, p)
    torch.cuda.synchronize()
    assert torch.equal(p.cpu(), hpar[:1])


if __name__ == "__main__":
    main()
