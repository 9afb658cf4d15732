"""End-to-end (host memory) rates, RS(10,4,8) 1 MiB objects.

The reference path starts and ends in host memory (Erlang binaries,
c_src/rscoding.cpp:41,73-81), called once per object from many scheduler
threads (basho_bench {concurrent, 4}), so the PCIe-inclusive rate is
recorded in DESIGN.md (never as the bench value):

  C ABI leoec_encode / leoec_decode per object from pageable memory, T
  concurrent caller threads, under
    batch       the default: calls that arrive while the GPU is busy are
                packed into one H2D / launch / D2H (hostq.cpp)
    per-thread  LEOEC_HOST_BATCH=0: each call its own copies on its
                thread's stream (the round-1 path)
  plus the Python mirror (NIF-equivalent term handling) at one caller, and
  the pinned, batched device-API path (H2D -> leoec_encode_dev -> D2H on two
  streams) as the link ceiling.

    python tools/e2e_bench.py [--quick] [--spread]

--spread: host calls spread over every gfx950 device of the node
(leoec_host_spread), for the node-level host rate.
"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

K, M, W, SIZE = 10, 4, 8, 1 << 20
LOST = [0, 1, 2, 3]


def callers(le, T, per, op, bs, filled, tag):
    """T threads calling leoec_{op} back to back: 3 trials of `per` seconds
    (after a warm-up trial); the median trial's rate."""
    import ctypes

    import numpy as np
    bsz = (K + M - filled) * bs
    rng = np.random.default_rng(T)
    srcs = [rng.integers(0, 256, SIZE, dtype=np.uint8) for _ in range(T)]
    outs = [np.empty(bsz, dtype=np.uint8) for _ in range(T)]
    for t in range(T):
        assert le.lib.leoec_encode(2, K, M, W, srcs[t].ctypes.data, SIZE, outs[t].ctypes.data, bsz) == 0
    # decode inputs: blocks 4..13 of each thread's object (pointers into src / out)
    ids = list(range(4, K + M))
    ptrs, idv, decs = [], (ctypes.c_int * len(ids))(*ids), []
    for t in range(T):
        p = []
        for i in ids:
            if i < filled:
                p.append(srcs[t].ctypes.data + i * bs)
            else:
                p.append(outs[t].ctypes.data + (i - filled) * bs)
        ptrs.append((ctypes.c_void_p * len(ids))(*p))
        decs.append(np.empty(SIZE, dtype=np.uint8))

    def call(t):
        if op == "encode":
            return le.lib.leoec_encode(2, K, M, W, srcs[t].ctypes.data, SIZE, outs[t].ctypes.data, bsz)
        return le.lib.leoec_decode(2, K, M, W, ptrs[t], idv, len(ids), bs, SIZE, decs[t].ctypes.data)

    errs = []
    stats = getattr(le._lib._current, "leoec_measure_hostq_stats", None)
    buf = (ctypes.c_double * 14)()

    cpu = []

    def trial():
        """All T threads call back to back for `per` seconds; calls/s (and
        the process's CPU time over the trial, in cores)."""
        ready = threading.Barrier(T + 1)
        go = threading.Event()
        counts = [0] * T
        box = {}

        def work(t):
            if call(t) != 0:  # warm this thread outside the timed region
                errs.append(t)
            ready.wait()
            go.wait()
            n = 0
            while time.perf_counter() < box["end"]:
                if call(t) != 0:
                    errs.append(t)
                n += 1
            counts[t] = n

        ths = [threading.Thread(target=work, args=(t,)) for t in range(T)]
        for th in ths:
            th.start()
        ready.wait()
        c0 = time.process_time()
        t0 = time.perf_counter()
        box["end"] = t0 + per
        go.set()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        cpu.append((time.process_time() - c0) / dt)
        return sum(counts), dt

    trial()  # warm-up trial (first use of the queue's slots)
    if stats:
        stats(buf)  # reset
    runs = [trial() for _ in range(3)]
    assert not errs, errs
    if op == "decode":
        for t in range(T):
            assert np.array_equal(decs[t], srcs[t]), "decode mismatch"
    rates = sorted(n * SIZE / dt / 2**30 for n, dt in runs)
    calls = sum(n for n, _ in runs)
    dt = sum(d for _, d in runs)
    rec = {"path": f"C ABI leoec_{op}, 1 MiB objects, {T} caller threads [{tag}]",
           "GiBps": round(rates[1], 2), "GiBps_min_max": [round(rates[0], 2), round(rates[-1], 2)],
           "us_per_call": round(dt * T / calls * 1e6, 1), "calls": calls,
           "cpu_cores": round(sorted(cpu[1:])[len(cpu[1:]) // 2], 2)}
    if stats:
        stats(buf)
        nb, nj = buf[0], buf[1]
        if nb:
            rec["queue"] = {"batches": int(nb), "jobs_per_batch": round(nj / nb, 2),
                            "launches_per_batch": round(buf[2] / nb, 2),
                            "us_per_batch": {k: round(buf[i] / nb, 1) for i, k in [
                                (6, "open_to_close"), (3, "fill_wait"), (4, "issue"),
                                (5, "gpu_wait"), (7, "done_to_free")]},
                            "issue_us": {"max": round(buf[10], 1), "h2d": round(buf[11] / nb, 1),
                                         "launch": round(buf[12] / nb, 1),
                                         "d2h": round(buf[13] / nb, 1)},
                            "us_per_job": {"reserve_wait": round(buf[9] / nj, 1),
                                           "done_wait": round(buf[8] / nj, 1)}}
    print(json.dumps(rec), flush=True)
    return rec


def mirror(le, tag):
    import numpy as np
    data = np.random.default_rng(1).integers(0, 256, SIZE, dtype=np.uint8).tobytes()
    for _ in range(3):
        le.nif_encode("vandrs", (K, M, W), data, SIZE)
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        st, blocks = le.nif_encode("vandrs", (K, M, W), data, SIZE)
        assert st == "ok"
    t = time.perf_counter() - t0
    print(json.dumps({"path": f"Python mirror nif_encode, 1 caller [{tag}]",
                      "GiBps": round(n * SIZE / t / 2**30, 2), "us_per_call": round(t / n * 1e6, 1)}))
    ids = list(range(4, K + M))
    surv = [blocks[i] for i in ids]
    t0 = time.perf_counter()
    for _ in range(n):
        st, out = le.nif_decode("vandrs", (K, M, W), surv, ids, SIZE)
        assert st == "ok"
    t = time.perf_counter() - t0
    assert out == data
    print(json.dumps({"path": f"Python mirror nif_decode (lose 0-3), 1 caller [{tag}]",
                      "GiBps": round(n * SIZE / t / 2**30, 2), "us_per_call": round(t / n * 1e6, 1)}),
          flush=True)


def pinned_ceiling(le, bs):
    import torch
    total, chunk = 1024, 64
    host = torch.randint(0, 256, (total, SIZE), dtype=torch.uint8).pin_memory()
    hpar = torch.empty((total, M * bs), dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dobj = [torch.empty((chunk, SIZE), dtype=torch.uint8, device="cuda") for _ in streams]
    dpar = [torch.empty((chunk, M * bs), dtype=torch.uint8, device="cuda") for _ in streams]

    def run():
        for i, c0 in enumerate(range(0, total, chunk)):
            s = streams[i % 2]
            with torch.cuda.stream(s):
                dobj[i % 2].copy_(host[c0:c0 + chunk], non_blocking=True)
                le.device.encode("vandrs", (K, M, W), dobj[i % 2], SIZE, dpar[i % 2],
                                 stream=s.cuda_stream)
                hpar[c0:c0 + chunk].copy_(dpar[i % 2], non_blocking=True)
        torch.cuda.synchronize()

    run()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        run()
    t = (time.perf_counter() - t0) / reps
    print(json.dumps({"path": "pinned batched H2D+encode+D2H (device API, 2 streams, 64-object chunks)",
                      "GiBps": round(total * SIZE / t / 2**30, 2),
                      "pcie_GBps": round(total * (SIZE + M * bs) / t / 1e9, 2)}), flush=True)


def main():
    import torch

    os.environ.setdefault("LEOEC_LIBRARY", "measure")  # A/B knobs: libleoec_measure.so
    import leo_erasure_amd as le
    torch.cuda.set_device(0)
    assert le.gf_init() == "ok"
    bs, filled = le.layout("vandrs", (K, M, W), SIZE)
    quick = "--quick" in sys.argv
    if "--spread" in sys.argv:  # every gfx950 device of the node (leoec_host_spread)
        print(json.dumps({"spread_over_devices": le._lib.host_lanes(),
                          "lanes": le._lib.host_spread(le._lib.host_lanes())}), flush=True)
    if "--libs" in sys.argv:  # --libs "tag:path;tag2:path2" [--threads ..] [--rounds R]
        # libraries A/B in one process, interleaved rounds (no knobs)
        libs = [e.partition(":")[::2] for e in sys.argv[sys.argv.index("--libs") + 1].split(";")]
        threads = (1, 8, 32)
        if "--threads" in sys.argv:
            threads = tuple(int(x) for x in sys.argv[sys.argv.index("--threads") + 1].split(","))
        rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 2
        for r in range(rounds):
            for tag, path in libs:
                le._lib.use_library(path)
                assert le.gf_init() == "ok"
                for op in ("encode", "decode"):
                    for T in threads:
                        callers(le, T, 0.4, op, bs, filled, f"{tag} round {r}")
        return
    if "--forms" in sys.argv:  # --forms "tag:K=V,K=V;tag2:..." [--threads 1,8,32]
        spec = sys.argv[sys.argv.index("--forms") + 1]
        forms = []
        for ent in spec.split(";"):
            tag, _, kv = ent.partition(":")
            forms.append((tag, dict(x.split("=", 1) for x in kv.split(",") if x)))
        threads, with_mirror = (1, 8, 32), False
        if "--threads" in sys.argv:
            threads = tuple(int(x) for x in sys.argv[sys.argv.index("--threads") + 1].split(","))
    elif "--queue-ab" in sys.argv:  # batching-queue policies (hostq.cpp knobs)
        # default: close when the previous H2D is done, poll events, depth 3
        # default: idle queue -> up to 4 calls direct, else batched; a batch
        # closes when the previous H2D is done; events polled; depth 3
        forms = [("default", {}),
                 ("always-batch", {"LEOEC_HOSTQ_DIRECT": "0", "LEOEC_HOSTQ_DIRECT_MAP": "0"}),
                 ("direct<=2", {"LEOEC_HOSTQ_DIRECT": "2"}),
                 ("direct<=8", {"LEOEC_HOSTQ_DIRECT": "8", "LEOEC_HOSTQ_DIRECT_MAP": "8"}),
                 ("sync-wait", {"LEOEC_HOSTQ_SYNC": "0"}),
                 ("close-asap", {"LEOEC_HOSTQ_CLOSE": "0"}),
                 ("depth2", {"LEOEC_HOSTQ_DEPTH": "2"})]
        threads, with_mirror = (1, 2, 4, 8, 16, 32), False
    else:
        forms = [("batch", {}), ("per-thread", {"LEOEC_HOST_BATCH": "0"})]
        threads, with_mirror = ((1, 8) if quick else (1, 2, 4, 8, 16, 32)), True
    for tag, env in forms:
        # knobs live in the measurement build, set through its setter (the
        # environment is never written while the library's threads run)
        le._lib.measure_reset_knobs()
        for k, v in env.items():
            le._lib.measure_set_knob(k, v)
        if with_mirror:
            mirror(le, tag)
        for op in ("encode", "decode"):
            for T in threads:
                callers(le, T, 0.4, op, bs, filled, tag)
    le._lib.measure_reset_knobs()
    if "--no-ceiling" not in sys.argv:
        pinned_ceiling(le, bs)


if __name__ == "__main__":
    main()
