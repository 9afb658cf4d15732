"""Headline benchmark: device-resident encode+decode GiB/s, vandrs RS(10,4,8),
1 MiB objects (BASELINE.json metric / configs[1..2]), plus the configs[4]
partitioned 64 MiB batch.

One step = encode every object of this rank's batch (10 data blocks read, 4
coding blocks written per object) + in-place decode of the same batch with
data blocks {0,1,2,3} erased (6 data + 4 coding read, 4 data written).  The
reference's unit of work is one independent object per call
(`c_src/rscoding.cpp:36-85`), so N GPUs = N processes with their own objects
and no collective on the data path:

* ``--workload 1MiB`` (default): every rank owns ``--objects`` 1 MiB objects
  (weak scaling, the BASELINE metric);
* ``--workload 64MiB``: one global batch of 64 x 64 MiB objects split over the
  ranks with `shard_range` (strong scaling, BASELINE configs[4]).

Control traffic (a barrier around the timed region, the max over ranks of
the elapsed time, each rank's verification verdict) goes over gloo on the
host: the data path has no collective and the bench needs no RCCL.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload 1MiB|64MiB]
  N > 1 without WORLD_SIZE in the environment: this process starts N ranks
  (torch.distributed.run) before touching the GPU and exits with their
  status; under a launcher each rank maps LOCAL_RANK to one device.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident encode+decode, vandrs RS(10,4,w=8) 1 MiB objects"
METRIC_64 = "GiB/s device-resident encode+decode, vandrs RS(10,4,w=8) 64 MiB objects, partitioned batch"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
K, M, W = 10, 4, 8
ERASED = [0, 1, 2, 3]          # the timed decode: worst case, 4 data blocks rebuilt
VERIFY_ERASED = [4, 7, 9, 10]  # a second pattern for the check: tail block, parity 11..13 used
POISON = 0xA5
WORKLOADS = {
    # name: (object bytes, objects per rank or None, global objects or None)
    "1MiB": (1 << 20, 2048, None),
    "64MiB": (64 << 20, None, 64),
}
# The GPU box grants one GPU's process 16 CPUs (the harness's CPU share);
# nproc / affinity there show the whole host.  Used when no cgroup quota says.
BOX_CPU_SHARE = 16


def shard_range(rank, world, total):
    """Objects [lo, hi) owned by `rank` when `total` objects split evenly."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--warmup-s", type=float, default=1.0,
                   help="minimum warm-up wall time (clock ramp); at least --warmup steps run")
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="1MiB")
    p.add_argument("--objects", type=int, default=None,
                   help="1MiB: objects per GPU (one launch); 64MiB: global batch")
    p.add_argument("--size", type=int, default=None, help="object bytes (default: the workload's)")
    p.add_argument("--oversubscribe", action="store_true",
                   help="allow more ranks than devices (ranks share devices; rehearsal only)")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="target CPU time of the bounded cpu_baseline sample")
    p.add_argument("--cpu-objects", type=int, default=1024,
                   help="objects in the cpu_baseline sample (copied from rank 0's batch)")
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    p.add_argument("--no-ceiling", action="store_true",
                   help="skip the live access-pattern ceiling of the headline kernel")
    p.add_argument("--no-host", action="store_true",
                   help="skip the host-memory (C ABI, PCIe-inclusive) leg")
    p.add_argument("--host-callers", type=int, default=32,
                   help="caller threads of the host-memory leg (one 1 MiB object each)")
    p.add_argument("--host-seconds", type=float, default=1.0,
                   help="timed seconds per op of the host-memory leg")
    # internal: the pattern-ceiling child process (GpuBackend.pattern_ceiling_child)
    p.add_argument("--pattern-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--host-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--host-data", default="", help=argparse.SUPPRESS)
    p.add_argument("--pattern-device", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--pattern-seed", type=int, default=0x1E0E, help=argparse.SUPPRESS)
    p.add_argument("--traffic", default=",".join(
        os.path.join(ROOT, "profiles", f) for f in ("pmc_traffic.json", "pmc_traffic_64MiB.json")),
                   help="PMC-derived HBM bytes per launch, comma-separated files; the one whose "
                        "objects / object_bytes match the run is used (tools/pmc_traffic.py)")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------
# Device backend: the measured path.
class GpuBackend:
    """libleoec's device entry points (leoec_encode_dev / leoec_decode_dev) on
    this rank's GPU; work is enqueued on torch's current stream."""

    def __init__(self, local_rank, world, oversubscribe=False):
        import torch

        import leo_erasure_amd as le

        ndev = torch.cuda.device_count()
        if ndev <= 0:
            raise SystemExit("bench.py: no GPU visible")
        if world > ndev and not oversubscribe:
            raise SystemExit(f"bench.py: {world} ranks but {ndev} device(s); "
                             "pass --oversubscribe to share devices")
        self.index = local_rank % ndev
        torch.cuda.set_device(self.index)
        st = le.gf_init()
        if st != "ok":
            raise SystemExit(f"bench.py: gf_init -> {st}")
        self.torch = torch
        self.le = le
        self.device = torch.device("cuda", self.index)
        self.name = f"cuda:{self.index} {torch.cuda.get_device_name(self.index)}"
        self.lib_path = le._lib.library_path()

    def random_batch(self, n, size, seed):
        t = self.torch
        gen = t.Generator(device=self.device).manual_seed(seed)
        return t.randint(0, 256, (n, size), dtype=t.uint8, device=self.device, generator=gen)

    def empty(self, n, cols):
        return self.torch.empty((n, cols), dtype=self.torch.uint8, device=self.device)

    def encode(self, objs, size, parity):
        self.le.device.encode("vandrs", (K, M, W), objs, size, parity)

    def decode(self, objs, size, parity, erased):
        self.le.device.decode("vandrs", (K, M, W), objs, size, parity, erased)

    def sync(self):
        self.torch.cuda.synchronize()

    def event(self):
        return self.torch.cuda.Event(enable_timing=True)

    def pattern_ceiling(self, objs, size, parity, enc_bytes, rounds=5, reps=20):
        """SURVEY §8(d)'s achievable-copy figures for the headline kernel, live
        on this batch: (1) the encode's access pattern without its arithmetic
        (every lane loads its 16-byte column of the 10 data blocks, stores 4
        parity columns, each their XOR: same bytes, 64-lane tile-major
        workgroups; measurement library `leoec_measure_xor_pattern_dev`,
        csrc/xor_pattern.hip, not a code), timed in alternating rounds with
        the shipped encode; (2) a device-to-device copy of the batch (torch
        copy_, read + write bytes); (3) the pattern's reads alone and its
        writes alone, timed in the same rounds (`halves`).  Overwrites
        `parity`.  Median per-launch times."""
        import ctypes
        import os
        import statistics
        lib = self.le._lib
        if not os.path.exists(lib.MEASURE_LIB_PATH):
            return {"achieved": None, "error": "measurement build absent (make -C leo_erasure_amd/csrc measure)"}
        mlib = lib.measure_library()  # (run by pattern_child: the library in use)
        stream = self.torch.cuda.current_stream().cuda_stream
        n = objs.shape[0]

        def xor_pattern():
            rc = mlib.leoec_measure_xor_pattern_dev(
                objs.data_ptr(), objs.stride(0), size, n, parity.data_ptr(), parity.stride(0),
                ctypes.c_void_p(stream))
            if rc != 0:
                raise RuntimeError(f"leoec_measure_xor_pattern_dev -> {rc}")

        def timed(fn):
            for _ in range(3):
                fn()
            ev = [self.event() for _ in range(reps + 1)]
            self.sync()
            ev[0].record()
            for i in range(reps):
                fn()
                ev[i + 1].record()
            self.sync()
            return [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]

        def half(h):
            def go():
                rc = mlib.leoec_measure_stream_half_dev(
                    h, objs.data_ptr(), objs.stride(0), size, n, parity.data_ptr(),
                    parity.stride(0), ctypes.c_void_p(stream))
                if rc != 0:
                    raise RuntimeError(f"leoec_measure_stream_half_dev({h}) -> {rc}")
            return go

        times = {"shipped": [], "pattern": [], "reads": [], "writes": []}
        for _ in range(rounds):
            times["shipped"] += timed(lambda: self.encode(objs, size, parity))
            times["pattern"] += timed(xor_pattern)
            times["reads"] += timed(half(0))
            times["writes"] += timed(half(1))
        med = {k: statistics.median(v) for k, v in times.items()}
        ship = enc_bytes / (med["shipped"] * 1e-3) / 1e9
        patt = enc_bytes / (med["pattern"] * 1e-3) / 1e9
        # the encode's bytes split as its reads (K blocks) and writes (M)
        rd_bytes, wr_bytes = enc_bytes * K // (K + M), enc_bytes * M // (K + M)
        serial = enc_bytes / ((med["reads"] + med["writes"]) * 1e-3) / 1e9
        halves = {"what": "the pattern's reads alone and its writes alone "
                          "(leoec_measure_stream_half_dev); `serial` = the encode's bytes at "
                          "those two rates back to back, an upper bound for a kernel that "
                          "mixes them (HBM read/write turnarounds)",
                  "reads_achieved": round(rd_bytes / (med["reads"] * 1e-3) / 1e9, 1),
                  "writes_achieved": round(wr_bytes / (med["writes"] * 1e-3) / 1e9, 1),
                  "serial_achieved": round(serial, 1),
                  "serial_frac": round(serial / HBM_PEAK_GBS, 4),
                  "shipped_over_serial": round(ship / serial, 4)}
        dst = self.torch.empty_like(objs)
        copy_ms = statistics.median(timed(lambda: dst.copy_(objs)))
        del dst
        copy_bytes = 2 * objs.numel()
        copy = copy_bytes / (copy_ms * 1e-3) / 1e9
        return {"kernel": "xor_pattern (measurement library): the encode's loads and stores, "
                          "XOR for the GF product, 64-lane tile-major; not a code",
                "achieved": round(patt, 1), "frac": round(patt / HBM_PEAK_GBS, 4),
                "shipped_achieved": round(ship, 1),
                "shipped_over_ceiling": round(ship / patt, 4),
                "copy": {"what": "device-to-device copy of the batch (torch copy_), "
                                 "read + write bytes", "bytes": copy_bytes,
                         "achieved": round(copy, 1), "frac": round(copy / HBM_PEAK_GBS, 4)},
                "shipped_over_copy": round(ship / copy, 4),
                "halves": halves,
                "sample": f"{rounds} alternating rounds x {reps} launches each, medians"}


    def pattern_ceiling_child(self, n, size, seed, timeout=300):
        """pattern_ceiling in a child process that loads libleoec_measure.so
        alone (LEOEC_LIBRARY=measure) and regenerates this rank's seeded batch
        on the same device: the bench process maps only libleoec.so (one HIP
        library per process, DESIGN §Product library and measurement
        library).  Started after the timed region and the CPU leg; a new
        process (subprocess), never an exec of this GPU-initialised one."""
        env = {k: v for k, v in os.environ.items()
               if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
        env["LEOEC_LIBRARY"] = "measure"
        cmd = [sys.executable, os.path.abspath(__file__), "--pattern-child",
               "--pattern-device", str(self.index), "--objects", str(n), "--size", str(size),
               "--pattern-seed", str(seed)]
        try:
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
        except subprocess.TimeoutExpired:
            return {"achieved": None, "error": f"pattern child timed out after {timeout} s"}
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not lines:
            return {"achieved": None,
                    "error": f"pattern child rc {r.returncode}: {r.stderr.strip()[-400:]}"}
        return json.loads(lines[-1])

    def host_path(self, objs, parity, size, bs, callers=32, seconds=1.0, timeout=240):
        """The NIF's path end to end (PCIe-inclusive; never the bench value):
        `host_rates` in a child process that keeps torch out
        (LEOEC_NO_TORCH=1), so libleoec.so binds the system HIP runtime, as
        in an Erlang VM that loads the NIF — the torch wheel's bundled
        runtime does not overlap the link's two directions (DESIGN.md
        End-to-end).  The child gets this rank's first `callers` objects and
        their GPU parity through files, and measures on this rank's device.
        The same leg in this process (the torch runtime) stays beside it as
        `torch_runtime`."""
        import tempfile

        import numpy as np
        n = min(callers, objs.shape[0])
        srcs = np.ascontiguousarray(objs[:n, :size].cpu().numpy())
        gpar = np.ascontiguousarray(parity[:n].cpu().numpy())
        inproc = host_rates(self.le, srcs, gpar, size, bs, self.index, seconds)
        inproc["link"] = self.link_rates()
        inproc["link_busy"] = link_busy(inproc, inproc["link"], size, bs)
        env = {k: v for k, v in os.environ.items()
               if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                            "LEOEC_LIBRARY")}
        env["LEOEC_NO_TORCH"] = "1"
        with tempfile.TemporaryDirectory(prefix="leoec_host_") as d:
            np.save(os.path.join(d, "srcs.npy"), srcs)
            np.save(os.path.join(d, "gpar.npy"), gpar)
            cmd = [sys.executable, os.path.abspath(__file__), "--host-child", "--host-data", d,
                   "--pattern-device", str(self.index), "--size", str(size),
                   "--host-seconds", str(seconds)]
            try:
                r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
                lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
                child = json.loads(lines[-1]) if r.returncode == 0 and lines else {
                    "error": f"host child rc {r.returncode}: {r.stderr.strip()[-400:]}"}
            except subprocess.TimeoutExpired:
                child = {"error": f"host child timed out after {timeout} s"}
        torch_rt = {k: inproc[k] for k in ("encode_GiBps", "decode_GiBps", "link", "link_busy",
                                           "parity_vs_gpu")}
        torch_rt["what"] = "the same leg in the bench process, on the torch wheel's HIP runtime"
        if "error" in child:  # the in-process figures stand, with the child's failure named
            out = dict(inproc)
            out["runtime"] = "torch wheel's (the system-runtime child failed)"
            out["child_error"] = child["error"]
            return out
        child["torch_runtime"] = torch_rt
        return child

    def link_rates(self, mib=256, reps=5):
        """This device's PCIe copy rates from / to pinned host memory (GB/s,
        median of `reps` copies of `mib` MiB) through torch: host -> device
        alone, device -> host alone, and both directions at once on two
        streams (bytes of both / time)."""
        t = self.torch
        n = mib << 20
        hsrc = t.empty(n, dtype=t.uint8, pin_memory=True)
        hdst = t.empty(n, dtype=t.uint8, pin_memory=True)
        dsrc = t.empty(n, dtype=t.uint8, device=self.device)
        ddst = t.empty(n, dtype=t.uint8, device=self.device)
        cur = t.cuda.current_stream(self.device)
        up, down = t.cuda.Stream(device=self.device), t.cuda.Stream(device=self.device)

        def timed(h2d, d2h):
            ms = []
            for i in range(reps + 1):
                a, b = self.event(), self.event()
                a.record(cur)
                for on, s, dst, src in ((h2d, up, ddst, hsrc), (d2h, down, hdst, dsrc)):
                    if on:
                        s.wait_stream(cur)
                        with t.cuda.stream(s):
                            dst.copy_(src, non_blocking=True)
                        cur.wait_stream(s)
                b.record(cur)
                self.sync()
                if i:
                    ms.append(a.elapsed_time(b))
            return (h2d + d2h) * n / (sorted(ms)[len(ms) // 2] * 1e-3) / 1e9

        out = {"h2d_GBps": round(timed(True, False), 1), "d2h_GBps": round(timed(False, True), 1),
               "both_GBps": round(timed(True, True), 1),
               "what": f"pinned {mib} MiB copies, median of {reps}; both = the two directions "
                       "at once on two streams, bytes of both / time, on this process's HIP "
                       "runtime (the torch wheel's, whose two copies do not overlap)"}
        del hsrc, hdst, dsrc, ddst
        return out


HOST_CALLERS_LIB = os.path.join(ROOT, "tools", "libhost_callers.so")


def host_rates(le, srcs, gpar, size, bs, device, seconds):
    """host-memory leoec_encode / leoec_decode through the C ABI from one
    thread per object of `srcs` (pageable numpy rows), back to back for
    `seconds` per op, on `device` (leoec_host_spread([device]): the threads'
    own current device would be device 0).  The caller threads are native
    (tools/libhost_callers.so, built by build(): as a VM's schedulers call
    the NIF), and the same loops from Python threads stay beside them as
    `python_threads` (each ctypes call takes and drops the interpreter lock,
    which costs 4-5 GiB/s at 32 threads).  Checked, outside the timed loops:
    every thread's encode parity equals `gpar` (the GPU's device parity of
    its object) and every decode (data blocks ERASED lost) returns the
    object.  No torch: bench.py runs it in the bench process and in the
    system-runtime child (host_child)."""
    import ctypes
    import threading

    import numpy as np
    L = le.lib
    n = srcs.shape[0]
    srcs = [np.ascontiguousarray(srcs[t]) for t in range(n)]
    filled = min(size // bs, K)
    out_bytes = (K + M - filled) * bs
    outs = [np.empty(out_bytes, dtype=np.uint8) for _ in range(n)]
    decs = [np.empty(size, dtype=np.uint8) for _ in range(n)]
    ids = list(range(len(ERASED), K + M))  # survivors: blocks 4..13
    idv = (ctypes.c_int * len(ids))(*ids)

    def block(t, i):
        if i < filled:
            return srcs[t].ctypes.data + i * bs
        return outs[t].ctypes.data + (i - filled) * bs

    def enc(t):
        return L.leoec_encode(2, K, M, W, srcs[t].ctypes.data, size, outs[t].ctypes.data,
                              out_bytes)

    ptrs = []

    def dec(t):
        return L.leoec_decode(2, K, M, W, ptrs[t], idv, len(ids), bs, size,
                              decs[t].ctypes.data)

    def check():
        enc_ok = all(np.array_equal(outs[t][(K - filled) * bs:], gpar[t]) for t in range(n))
        dec_ok = all(np.array_equal(decs[t], srcs[t]) for t in range(n))
        return enc_ok, dec_ok

    def timed(fn):
        errs, counts, box = [], [0] * n, {}
        ready = threading.Barrier(n + 1)
        go = threading.Event()

        def work(t):
            if fn(t) != 0:  # this thread's first call, outside the clock
                errs.append(t)
            ready.wait()
            go.wait()
            c = 0
            while time.perf_counter() < box["end"]:
                if fn(t) != 0:
                    errs.append(t)
                c += 1
            counts[t] = c

        ths = [threading.Thread(target=work, args=(t,)) for t in range(n)]
        for th in ths:
            th.start()
        ready.wait()
        t0 = time.perf_counter()
        box["end"] = t0 + seconds
        go.set()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        if errs:
            raise RuntimeError(f"host-path calls failed on threads {sorted(set(errs))[:8]}")
        return sum(counts) * size / dt / 2**30, sum(counts)

    native = None
    if os.path.exists(HOST_CALLERS_LIB):
        native = ctypes.CDLL(HOST_CALLERS_LIB)
        vp = ctypes.c_void_p
        native.host_callers_run.restype = ctypes.c_long
        native.host_callers_run.argtypes = [
            vp, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_uint64, ctypes.c_uint64, vp, vp,
            ctypes.c_int, ctypes.c_uint64, vp, vp]

    def native_timed(op):
        """the same loop from native threads (host_callers_run)"""
        fn = ctypes.cast(L.leoec_encode if op == 0 else L.leoec_decode, ctypes.c_void_p)
        src_p = (ctypes.c_void_p * n)(*[srcs[t].ctypes.data for t in range(n)])
        out_p = (ctypes.c_void_p * n)(*[(outs if op == 0 else decs)[t].ctypes.data
                                        for t in range(n)])
        flat = (ctypes.c_void_p * (n * len(ids)))(*[block(t, i) for t in range(n) for i in ids])
        counts = (ctypes.c_long * n)()
        elapsed = ctypes.c_double()
        bad = native.host_callers_run(fn, op, n, seconds, 2, K, M, W, src_p, out_p, size,
                                      out_bytes, flat, idv, len(ids), bs, counts,
                                      ctypes.byref(elapsed))
        if bad:
            raise RuntimeError(f"host-path calls failed: {bad} (native callers)")
        total = sum(counts)
        return total * size / elapsed.value / 2**30, total

    le._lib.host_spread([device])
    try:
        for t in range(n):
            if enc(t) != 0:
                raise RuntimeError("leoec_encode failed")
        ptrs[:] = [(ctypes.c_void_p * len(ids))(*[block(t, i) for i in ids]) for t in range(n)]
        py_enc, py_enc_calls = timed(enc)
        py_dec, py_dec_calls = timed(dec)
        py_ok = check()
        if native is not None:
            enc_gibs, enc_calls = native_timed(0)
            dec_gibs, dec_calls = native_timed(1)
            enc_ok, dec_ok = check()
            enc_ok, dec_ok = enc_ok and py_ok[0], dec_ok and py_ok[1]
        else:
            enc_gibs, enc_calls, dec_gibs, dec_calls = py_enc, py_enc_calls, py_dec, py_dec_calls
            enc_ok, dec_ok = py_ok
    finally:
        le._lib.host_spread([])
    kind = ("native threads (tools/libhost_callers.so), as a VM's schedulers call the NIF"
            if native is not None else "Python threads (tools/libhost_callers.so not built)")
    return {"encode_GiBps": round(enc_gibs, 2), "decode_GiBps": round(dec_gibs, 2),
            "callers": n, "callers_kind": kind, "seconds_per_op": seconds,
            "calls": [enc_calls, dec_calls],
            "python_threads": {"encode_GiBps": round(py_enc, 2), "decode_GiBps": round(py_dec, 2),
                               "calls": [py_enc_calls, py_dec_calls],
                               "what": "the same loops from Python threads through ctypes"},
            "parity_vs_gpu": {"objects": n, "encode_equal": enc_ok, "decode_equal": dec_ok},
            "what": f"C ABI leoec_encode / leoec_decode (data blocks {ERASED} lost) of "
                    f"{size} B host objects from {n} threads, PCIe-inclusive "
                    "(pageable caller buffers; batching queue), this rank's device; "
                    "GiB/s of object payload"}


def link_busy(rates, link, size, bs):
    """The share of each second the op's bytes keep the link busy at the
    one-direction copy rates measured alone (an encode: its object host ->
    device, its m parity blocks back; a decode: its K survivors in, the
    rebuilt blocks back); above 1 the two directions overlap."""
    e = len(ERASED)
    per = {"encode": (1.0, M * bs / size), "decode": (K * bs / size, e * bs / size)}
    rate = {"encode": rates["encode_GiBps"], "decode": rates["decode_GiBps"]}
    return {op: round(rate[op] * 2**30 / 1e9 * (h / link["h2d_GBps"] + d / link["d2h_GBps"]), 3)
            for op, (h, d) in per.items()}


def hip_link_rates(device, mib=256, reps=5):
    """link_rates through the HIP runtime the process loaded (ctypes; the
    system runtime in host_child): pinned hipHostMalloc buffers, two
    runtime-created streams."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")  # the one libleoec.so loaded
    vp = ctypes.c_void_p
    hip.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    hip.hipStreamSynchronize.argtypes = [vp]
    hip.hipHostFree.argtypes = [vp]
    hip.hipFree.argtypes = [vp]
    hip.hipStreamDestroy.argtypes = [vp]
    n = mib << 20
    if hip.hipSetDevice(device) != 0:
        raise RuntimeError("hipSetDevice failed")
    hs, hd, ds, dd, up, down = vp(), vp(), vp(), vp(), vp(), vp()
    try:
        for p in (hs, hd):
            if hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(n), ctypes.c_uint(0)) != 0:
                raise RuntimeError("hipHostMalloc failed")
        for p in (ds, dd):
            if hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n)) != 0:
                raise RuntimeError("hipMalloc failed")
        for s in (up, down):
            if hip.hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1)) != 0:
                raise RuntimeError("hipStreamCreateWithFlags failed")
        ctypes.memset(hs, 0x5A, n)
        ctypes.memset(hd, 0, n)

        def timed(h2d, d2h):
            ms = []
            for i in range(reps + 1):
                t0 = time.perf_counter()
                if h2d and hip.hipMemcpyAsync(ds, hs, n, 1, up) != 0:
                    raise RuntimeError("hipMemcpyAsync failed")
                if d2h and hip.hipMemcpyAsync(hd, dd, n, 2, down) != 0:
                    raise RuntimeError("hipMemcpyAsync failed")
                if hip.hipStreamSynchronize(up) != 0 or hip.hipStreamSynchronize(down) != 0:
                    raise RuntimeError("hipStreamSynchronize failed")
                if i:
                    ms.append((time.perf_counter() - t0) * 1e3)
            return round((h2d + d2h) * n / (sorted(ms)[len(ms) // 2] * 1e-3) / 1e9, 1)

        return {"h2d_GBps": timed(True, False), "d2h_GBps": timed(False, True),
                "both_GBps": timed(True, True),
                "what": f"pinned {mib} MiB copies, median of {reps}; both = the two directions "
                        "at once on two streams, bytes of both / time, system HIP runtime"}
    finally:
        for s in (up, down):
            if s.value:
                hip.hipStreamDestroy(s)
        for p in (hs, hd):
            if p.value:
                hip.hipHostFree(p)
        for p in (ds, dd):
            if p.value:
                hip.hipFree(p)


def host_child(args):
    """--host-child: a process without torch (LEOEC_NO_TORCH=1, set by the
    parent), so libleoec.so runs on the system HIP runtime an Erlang VM
    would load; host_rates over the parent's objects and GPU parity, the
    link's copy rates on the same runtime, one JSON line."""
    import numpy as np
    if os.environ.get("LEOEC_NO_TORCH") != "1" or "torch" in sys.modules:
        raise RuntimeError("host child must run without torch (LEOEC_NO_TORCH=1)")
    import leo_erasure_amd as le
    srcs = np.load(os.path.join(args.host_data, "srcs.npy"))
    gpar = np.load(os.path.join(args.host_data, "gpar.npy"))
    size = args.size
    bs = ((size + K * W - 1) // (K * W) + 15) // 16 * 16 * W
    if le.gf_init() != "ok":
        raise RuntimeError("gf_init failed")
    rec = host_rates(le, srcs, gpar, size, bs, args.pattern_device, args.host_seconds)
    rec["link"] = hip_link_rates(args.pattern_device)
    rec["link_busy"] = link_busy(rec, rec["link"], size, bs)
    rec["runtime"] = ("system HIP runtime (/opt/rocm), child process without torch: what an "
                      "Erlang VM loading the NIF gets")
    if "torch" in sys.modules:
        raise RuntimeError("torch was imported in the host child")
    print(json.dumps(rec), flush=True)
    return 0


def pattern_child(args):
    """--pattern-child: this process loads libleoec_measure.so only
    (LEOEC_LIBRARY=measure, set by the parent), regenerates the parent's
    seeded batch on the same device, encodes it once and prints
    pattern_ceiling's record as one JSON line."""
    be = GpuBackend(args.pattern_device, 1, True)
    size = args.size or WORKLOADS["1MiB"][0]
    n = args.objects or WORKLOADS["1MiB"][1]
    bs = ((size + K * W - 1) // (K * W) + 15) // 16 * 16 * W
    objs = be.random_batch(n, size, args.pattern_seed)
    parity = be.empty(n, M * bs)
    be.encode(objs, size, parity)
    be.sync()
    rec = be.pattern_ceiling(objs, size, parity, (K + M) * bs * n)
    rec["process"] = (f"child process, {os.path.basename(be.lib_path)} only (the bench process "
                      "maps libleoec.so only); `shipped_achieved` is that build's copy of the "
                      "shipped kernel")
    print(json.dumps(rec), flush=True)
    return 0


# ---------------------------------------------------------------------------
def cpu_share():
    """Worker threads the CPU baseline may use on this host, and what that
    rests on.  The share is the cgroup's cpu.max quota (whole CPUs) or, with
    no quota, the affinity mask capped at the GPU box's per-GPU share; one
    CPU of it is left to the process's other threads (main, torch, HIP
    runtime): with workers = quota they compete with those for the quota and
    the cgroup's CFS bandwidth control throttles whole passes (round 3's
    driver run lost 0.88 s to it)."""
    host = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = host
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        quota = None
    if quota:
        share, basis = max(1, min(aff, int(math.floor(quota)))), "cgroup cpu.max quota"
    else:
        share, basis = min(aff, BOX_CPU_SHARE), (
            f"affinity, capped at {BOX_CPU_SHARE} = the GPU box's CPU share per GPU")
    threads = headroom_workers(share)
    return threads, {"host_cpus": host, "affinity_cpus": aff, "cgroup_cpus": quota,
                     "threads_basis": basis, "share_cpus": share,
                     "reserved_cpus": share - threads}


def headroom_workers(share):
    """Workers for a share of `share` whole CPUs: one CPU is left for the
    process's own threads whenever the share has more than one."""
    return max(1, share - 1)


def _cpu_list(text):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    out = []
    for part in text.strip().split(","):
        if part:
            lo, _, hi = part.partition("-")
            out.extend(range(int(lo), int(hi or lo) + 1))
    return out


def _cpu_snap():
    """{cpu: (total jiffies, idle jiffies)} from /proc/stat, {} if unreadable."""
    out = {}
    try:
        with open("/proc/stat") as fh:
            for line in fh:
                f = line.split()
                if f and f[0].startswith("cpu") and f[0] != "cpu":
                    v = [int(x) for x in f[1:]]
                    out[int(f[0][3:])] = (sum(v), v[3] + (v[4] if len(v) > 4 else 0))
    except (OSError, ValueError):
        return {}
    return out


def _busy_between(a, b):
    busy = {}
    for c in a.keys() & b.keys():
        tot, idle = b[c][0] - a[c][0], b[c][1] - a[c][1]
        busy[c] = 1.0 - idle / tot if tot > 0 else 0.0
    return busy


def _cpu_busy(window_s=0.25):
    """Fraction of time each CPU was busy over a short window (/proc/stat),
    or {} where /proc/stat is unreadable."""
    a = _cpu_snap()
    time.sleep(window_s)
    return _busy_between(a, _cpu_snap())


def pick_cpus(threads, sysfs="/sys/devices/system", busy=None):
    """CPUs to pin the baseline's `threads` workers to: one hardware thread
    per physical core (no two workers on SMT siblings), all on one NUMA node
    where it has enough cores, within the affinity mask (the cgroup's
    cpuset).  The host is shared with other tenants, so the cores are the
    least busy ones over a short /proc/stat window (a core counts as busy as
    its busiest sibling), and the node is the one whose `threads` least busy
    cores are idlest.  Returns (cpus, {numa nodes used})."""
    aff = sorted(os.sched_getaffinity(0))
    allowed = set(aff)
    if busy is None:
        busy = _cpu_busy()

    def read(path):
        try:
            with open(path) as fh:
                return fh.read()
        except OSError:
            return None

    node_of = {}
    for nd in range(64):
        t = read(f"{sysfs}/node/node{nd}/cpulist")
        if t is None:
            continue
        for c in _cpu_list(t):
            node_of[c] = nd
    cores = {}  # physical core -> (its allowed cpus, busiest sibling's load)
    for c in aff:
        sib = read(f"{sysfs}/cpu/cpu{c}/topology/thread_siblings_list")
        sibs = _cpu_list(sib) if sib else [c]
        core = min(sibs)
        load = max(busy.get(x, 0.0) for x in sibs)
        cpu_list, _ = cores.get(core, ([], 0.0))
        cores[core] = (cpu_list + [c], load)
    by_node = {}
    for core, (cl, load) in cores.items():
        by_node.setdefault(node_of.get(cl[0], 0), []).append((load, cl[0]))
    for v in by_node.values():
        v.sort()
    full = [nd for nd, v in by_node.items() if len(v) >= threads]
    if full:  # the node whose `threads` least busy cores are idlest
        nd = min(full, key=lambda n: (sum(x for x, _ in by_node[n][:threads]), n))
        cpus = [c for _, c in by_node[nd][:threads]]
    else:  # no node has enough cores: the least busy cores anywhere
        cpus = [c for _, c in sorted(x for v in by_node.values() for x in v)][:threads]
    if len(cpus) < threads:  # fewer physical cores than threads: reuse siblings
        cpus += [c for c in aff if c not in cpus][: threads - len(cpus)]
    cpus = [c for c in cpus if c in allowed]
    return cpus, sorted({node_of.get(c, 0) for c in cpus})


def _cgroup_throttled_us():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as fh:
            for line in fh:
                k, _, v = line.partition(" ")
                if k == "throttled_usec":
                    return int(v)
    except (OSError, ValueError):
        pass
    return None


THROTTLE_EPS_S = 1e-3  # a pass the cgroup throttled for longer than this is flagged


def summarize_passes(rates, throttled):
    """Median GiB/s of a baseline's passes, over the passes the cgroup did
    not throttle when at least 3 of them were not (throttling only ever slows
    a pass), otherwise over all; with the spreads of the passes used."""
    flagged = [t is not None and t > THROTTLE_EPS_S for t in throttled] if throttled else []
    flagged += [False] * (len(rates) - len(flagged))
    clean = [r for r, f in zip(rates, flagged) if not f]
    used = sorted(clean if len(clean) >= 3 else rates)
    med = used[len(used) // 2]
    return {
        "value": round(med, 3),
        "passes_used": "unthrottled" if len(clean) >= 3 else "all (fewer than 3 unthrottled)",
        "throttled_passes": sum(flagged),
        "best_pass_GiBps": round(used[-1], 3),
        "pass_spread": round((used[-1] - used[0]) / med, 4) if med else None,
        "iqr_spread": round((used[(3 * len(used)) // 4] - used[len(used) // 4]) / med, 4)
        if med else None,
    }


def cpu_baseline(objs, parity, size, n_sample, target_s, ref_structure_s=None):
    """The CPU restatement with ISA-L's split-table / GFNI technique
    (oracle/leoec_oracle.c orc_bench_rs8_pinned, structure 0), timed on this
    host's cores over a bounded sample of the SAME workload: the first
    `n_sample` objects of rank 0's batch, copied to host memory.  Its encode
    output is also compared byte for byte with the GPU's parity of those
    objects (outside the timed region), so the line's `verified` covers
    encode parity too.  Then, as a second labelled figure, the reference's
    own CPU structure (Jerasure's per-(row, input) region passes with
    destination read-modify-write, rscoding.cpp:71 / :147; structure 1) on
    the same sample, workers and parity check, for `ref_structure_s`
    seconds (default target_s / 2); and a short scalar leg (the same one
    pass with scalar table lookups, SURVEY §8(d)'s scalar reference)."""
    import numpy as np

    from oracle import oracle as O

    threads, share = cpu_share()
    cpus, nodes = pick_cpus(threads)
    threads = len(cpus) or threads
    n = min(n_sample, objs.shape[0])
    host = objs[:n].to("cpu", copy=True).numpy()
    gpu_par = parity[:n].to("cpu", copy=True).numpy()

    def leg(structure, total_s):
        cpu_par = np.zeros_like(gpu_par)
        # one pool of workers for the whole leg, worker t pinned to cpus[t],
        # each first-touching its own slice of the sample (NUMA-local pages);
        # passes of >= total/12 s each (several encode+decode rounds between
        # barriers); cpu_par receives the workers' encode of the sample,
        # compared with the GPU's parity after the clock
        pass_s = total_s / 12.0
        thr0 = _cgroup_throttled_us()
        snap0 = _cpu_snap()
        throttled, warm = [], []
        t0 = time.perf_counter()
        rates = O.bench_rs8_pinned(K, M, host, size, ERASED, threads, cpus, pass_s, total_s,
                                   min_passes=3, parity_out=cpu_par, structure=structure,
                                   throttled=throttled, warm_s=total_s / 3.0, warmup=warm)
        t_all = time.perf_counter() - t0
        busy = _busy_between(snap0, _cpu_snap())
        thr1 = _cgroup_throttled_us()
        rec = summarize_passes(rates, throttled)
        rec.update({
            "unit": "GiB/s",
            "passes_GiBps": [round(r, 2) for r in rates],
            # untimed: until two consecutive passes agree within 3 % (at most
            # a third of the leg's time); a shared host ramps for seconds
            "warmup_passes_GiBps": [round(r, 2) for r in warm],
            "throttled_s_per_pass": [None if t is None else round(t, 4) for t in throttled],
            "cgroup_throttled_s": None if thr0 is None or thr1 is None else
            round((thr1 - thr0) / 1e6, 3),
            # the host is shared: CPUs busy during the leg, ours included
            # (the workers' `threads`), as a record of the other tenants' load
            "host_busy_cpus": round(sum(busy.values()), 1) if busy else None,
            "parity_vs_gpu": {"objects": n, "equal": bool(np.array_equal(cpu_par, gpu_par))},
            "sample": f"{len(rates)} passes of >= {pass_s:.2f} s over the first {n} x {size} B "
                      f"objects of rank 0's batch: vandrs RS({K},{M},8) encode + in-place "
                      f"decode of data blocks {ERASED}, {threads} threads pinned one per "
                      f"physical core, each first-touching its own slice, after "
                      f"{len(warm)} untimed warm-up passes; {t_all:.2f} s in all; "
                      f"value = median pass",
        })
        return rec

    rec = leg(0, target_s)
    rec.update({
        "cores": threads, "kind": "port",
        "simd": {0: "scalar", 2: "avx2-pshufb (ISA-L split tables)",
                 3: "avx512-gfni (ISA-L gf2p8affine)"}.get(O.simd_level(), "scalar"),
        "structure": "ISA-L ec_encode_data: one pass per object, every output row at once",
        "pinning": {"cpus": cpus, "numa_nodes": nodes, "first_touch": "per worker thread",
                    "choice": "least busy physical cores of one NUMA node (/proc/stat)"},
        "workers": threads,
    })
    rec.update(share)
    rs = leg(1, target_s / 2.0 if ref_structure_s is None else ref_structure_s)
    rs.update({
        "cores": threads, "kind": "port",
        "simd": "avx2-pshufb (gf-complete w=8 split tables)" if O.simd_level() >= 2 else "scalar",
        "structure": ("Jerasure jerasure_matrix_encode / decode_data: per coding row, the "
                      "coefficient-1 inputs copied / xor-ed, then one region multiply pass per "
                      "other input over the whole block with destination read-modify-write "
                      "(rscoding.cpp:71, :147)"),
    })
    # SURVEY §8(d)'s scalar reference: the one pass with scalar split-table
    # lookups (no SIMD), a short leg for scale
    sc = leg(2, target_s / 6.0 if ref_structure_s is None else ref_structure_s / 3.0)
    sc.update({"cores": threads, "kind": "port", "simd": "scalar",
               "structure": "one pass per object, scalar 4-bit split-table lookups"})
    out = headline_cpu(rec, rs)
    out["scalar"] = sc
    return out


CPU_LEGS = ("isa_l_port", "reference_structure")


def headline_cpu(port, ref):
    """The line's cpu_baseline is its strongest CPU figure (round-4 verdict
    item 3): the faster of the ISA-L-technique port and the reference's own
    Jerasure structure among the legs whose parity equals the GPU's, with
    the other leg kept as a sub-field under its name and `headline_leg`
    naming the one on top.  The shared fields (cores, pinning, share) stay
    at the top level.  `full_share_estimate_GiBps` scales the headline to
    the whole CPU share (the workers leave one CPU of it to the process's
    own threads; round-4 advisor)."""
    shared = {k: v for k, v in port.items()
              if k in ("cores", "kind", "pinning", "workers", "host_cpus", "affinity_cpus",
                       "cgroup_cpus", "threads_basis", "share_cpus", "reserved_cpus")}
    legs = {"isa_l_port": dict(port), "reference_structure": dict(ref)}

    def ok(leg):
        return leg.get("value") is not None and leg.get("parity_vs_gpu", {}).get("equal", False)

    cands = [name for name in CPU_LEGS if ok(legs[name])] or ["isa_l_port"]
    top = max(cands, key=lambda name: legs[name].get("value") or 0.0)
    other = [name for name in CPU_LEGS if name != top][0]
    out = dict(legs[top])
    out.update(shared)
    out["headline_leg"] = top
    out["rule"] = ("value = the faster parity-equal leg: the ISA-L-technique port "
                   "(isa_l_port) or the reference's own Jerasure structure "
                   "(reference_structure), both timed on the same cores and sample")
    out[other] = legs[other]
    workers, share = shared.get("workers"), shared.get("share_cpus")
    if out.get("value") and workers and share:
        out["full_share_estimate_GiBps"] = round(out["value"] * share / workers, 3)
    return out


# ---------------------------------------------------------------------------
def read_traffic(paths, n, size, lib_path):
    """PMC HBM bytes per encode launch from the committed measurement whose
    batch shape matches (tools/pmc_traffic.py), or None.  The file carries
    the sha256 of the code object it was measured on (the offload bundle
    defining gf8_apply<10,4>, leo_erasure_amd/codeobj.py); the figure is
    used only if the library this run loaded holds the same code object, so
    a kernel change without a fresh PMC pass prints null, not a stale
    number.  Returns (traffic, what was found)."""
    from leo_erasure_amd import codeobj

    have = None
    for tpath in [t for t in paths.split(",") if t]:
        if not os.path.exists(tpath):
            continue
        try:
            with open(tpath) as fh:
                tr = json.load(fh)
        except (OSError, ValueError):
            continue
        if tr.get("objects") != n or tr.get("object_bytes") != size:
            continue
        want = (tr.get("code_object") or {}).get("sha256")
        if have is None:
            try:
                have = codeobj.kernel_code_object_sha256(lib_path) if lib_path else ""
            except (OSError, ValueError):
                have = ""
        name = os.path.basename(tpath)
        if not want:
            return None, f"{name}: no code-object stamp"
        if want != have:
            return None, f"{name}: stamp {want[:12]} != loaded code object {(have or '?')[:12]}"
        return tr.get("encode_bytes_per_launch"), f"{name} (code object {want[:12]})"
    return None, "no PMC file for this batch shape"


def _poison_decode(be, objs, ref, parity, size, bs, erased):
    """Overwrite the erased data blocks, rebuild them, require the batch to
    equal its pristine copy: a decode that writes nothing fails this."""
    for b in erased:
        if b >= K:
            continue
        lo, hi = b * bs, min((b + 1) * bs, size)
        if lo < hi:
            objs[:, lo:hi] = POISON
    be.decode(objs, size, parity, erased)
    be.sync()
    return bool(objs.equal(ref))


def run_rank(args, be, rank, world, dist=None):
    """One rank of the bench; returns (record-or-None, verified)."""
    size = args.size or WORKLOADS[args.workload][0]
    per_rank, global_n = WORKLOADS[args.workload][1:]
    if args.objects is not None:
        if global_n is None:
            per_rank = args.objects
        else:
            global_n = args.objects
    if global_n is not None:
        lo, hi = shard_range(rank, world, global_n)
    else:
        lo, hi = rank * per_rank, (rank + 1) * per_rank
    n = hi - lo
    bs = ((size + K * W - 1) // (K * W) + 15) // 16 * 16 * W  # rscoding.cpp:44
    if n <= 0:
        raise SystemExit(f"rank {rank}: no objects (global batch {global_n}, {world} ranks)")

    objs = be.random_batch(n, size, 0x1E0E + lo)
    parity = be.empty(n, M * bs)
    ref = objs.clone()

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        be.encode(objs, size, parity)
        if ev is not None:
            ev[1].record()
        be.decode(objs, size, parity, ERASED)
        if ev is not None:
            ev[2].record()

    # warm-up: at least W steps and at least --warmup-s seconds (clock ramp)
    tw = time.perf_counter()
    wsteps = 0
    while wsteps < args.warmup or time.perf_counter() - tw < args.warmup_s:
        step()
        wsteps += 1
        if wsteps % 16 == 0:
            be.sync()
    be.sync()
    warm_s = time.perf_counter() - tw

    events = [[be.event() for _ in range(3)] for _ in range(args.steps)]
    be.sync()
    if dist is not None:
        dist.barrier()
    be.sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    be.sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    enc_t = [e[0].elapsed_time(e[1]) for e in events]
    dec_t = [e[1].elapsed_time(e[2]) for e in events]
    enc_ms = sum(enc_t) / len(enc_t)
    dec_ms = sum(dec_t) / len(dec_t)

    # verification, outside the timed region
    intact = bool(objs.equal(ref))                       # the timed decodes kept the batch
    dec_ok = _poison_decode(be, objs, ref, parity, size, bs, ERASED)
    dec2_ok = _poison_decode(be, objs, ref, parity, size, bs, VERIFY_ERASED)
    mine = {"rank": rank, "device": getattr(be, "name", "?"), "objects": [lo, hi],
            "elapsed_s": elapsed, "enc_ms": enc_ms, "dec_ms": dec_ms,
            "warmup_steps": wsteps, "warmup_s": warm_s,
            "checks": {"timed_batch_intact": intact, "poisoned_decode_0_1_2_3": dec_ok,
                       "poisoned_decode_4_7_9_10": dec2_ok}}
    if not args.no_host and hasattr(be, "host_path"):
        # every rank, its own device: the node's host-memory rate at N > 1
        # (parity holds the last timed encode of the pristine batch `ref`)
        try:
            mine["host_path"] = be.host_path(ref, parity, size, bs, args.host_callers,
                                             args.host_seconds)
        except Exception as e:  # a host problem must not discard the GPU measurement
            mine["host_path"] = {"encode_GiBps": None, "error": f"{type(e).__name__}: {e}"}
    if dist is not None:
        allr = [None] * world
        dist.all_gather_object(allr, mine)
    else:
        allr = [mine]
    verified = all(all(r["checks"].values()) for r in allr)
    if rank != 0:
        return None, verified

    el = max(r["elapsed_s"] for r in allr)
    total_objs = sum(r["objects"][1] - r["objects"][0] for r in allr)
    value = 2.0 * total_objs * size * args.steps / el / 2**30
    enc_bytes = (K + M) * bs * n              # algorithmic bytes per encode launch (rank 0)
    dec_bytes = (K + len(ERASED)) * bs * n    # per decode launch
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_gbs = dec_bytes / (dec_ms * 1e-3) / 1e9
    traffic, traffic_src = read_traffic(args.traffic, n, size, getattr(be, "lib_path", None))

    def rank_frac(r, per_obj, ms):
        return (r["objects"][1] - r["objects"][0]) * per_obj / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS

    # the whole node: every rank's algorithmic bytes per launch over the
    # slowest rank's average launch, against world x the per-GPU peak
    agg = {}
    for op, per_obj, key in (("encode", (K + M) * bs, "enc_ms"),
                             ("decode", (K + len(ERASED)) * bs, "dec_ms")):
        tot = sum((r["objects"][1] - r["objects"][0]) * per_obj for r in allr)
        slow = max(r[key] for r in allr)
        gbs = tot / (slow * 1e-3) / 1e9
        agg[op] = {"alg_bytes_per_launch": tot, "slowest_rank_launch_ms": round(slow, 4),
                   "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS * world,
                   "frac": round(gbs / (HBM_PEAK_GBS * world), 4)}
    strong = global_n is not None
    rec = {
        "metric": METRIC_64 if strong else METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_steps_run": wsteps,
        "warmup_s": round(warm_s, 3),
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (uniform random bytes, torch Philox, seed 0x1E0E + first object index)",
        "config": {
            "workload": (f"vandrs RS(k=10,m=4,w=8) encode + in-place decode of data blocks "
                         f"{{0,1,2,3}}, {size} B objects, device-resident batch"
                         + (f", global batch of {global_n} objects partitioned over the ranks"
                            if strong else "")),
            "objects_per_gpu": n if not strong else None,
            "global_objects": total_objs, "object_bytes": size, "block_size": bs,
            "parallelism": f"object-sharded x{world}, no data-path collective (gloo control only)",
        },
        "roofline": {
            "bound": "hbm", "kernel": "gf8_apply<10,4> (encode)",
            "achieved": round(enc_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(enc_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": traffic_src,
            "alg_bytes_per_launch": enc_bytes, "avg_launch_ms": round(enc_ms, 4),
            "decode": {"achieved": round(dec_gbs, 1), "frac": round(dec_gbs / HBM_PEAK_GBS, 4),
                       "alg_bytes_per_launch": dec_bytes, "avg_launch_ms": round(dec_ms, 4)},
            "scope": "rank 0's GPU (achieved / frac); `aggregate`: all ranks",
            "aggregate": dict(agg, n_gpus=world,
                              what="sum over ranks of algorithmic bytes per launch / the "
                                   "slowest rank's average launch; peak = n_gpus x 8 TB/s"),
        },
        "kernel_ms": {
            "encode_min_med_max": [round(x, 4) for x in (min(enc_t), sorted(enc_t)[len(enc_t) // 2],
                                                         max(enc_t))],
            "decode_min_med_max": [round(x, 4) for x in (min(dec_t), sorted(dec_t)[len(dec_t) // 2],
                                                         max(dec_t))]},
        "per_rank": [{"rank": r["rank"], "device": r["device"], "objects": r["objects"],
                      "elapsed_s": round(r["elapsed_s"], 5),
                      "encode_ms": round(r["enc_ms"], 4), "decode_ms": round(r["dec_ms"], 4),
                      "encode_frac": round(rank_frac(r, (K + M) * bs, r["enc_ms"]), 4),
                      "decode_frac": round(rank_frac(r, (K + len(ERASED)) * bs, r["dec_ms"]), 4),
                      "checks": r["checks"]} for r in allr],
        "cpu_baseline": None,
    }
    hps = [r.get("host_path") for r in allr]
    if all(hps):
        ok = [h for h in hps if h.get("encode_GiBps") is not None]
        rec["host_path"] = {
            "encode_GiBps": round(sum(h["encode_GiBps"] for h in ok), 2) if len(ok) == world else None,
            "decode_GiBps": round(sum(h["decode_GiBps"] for h in ok), 2) if len(ok) == world else None,
            "callers": sum(h.get("callers", 0) for h in ok),
            "scope": "sum over ranks (each rank its own device and callers); PCIe-inclusive, "
                     "never the bench value",
            "per_rank": hps}
        verified = verified and all(h["parity_vs_gpu"]["encode_equal"] and
                                    h["parity_vs_gpu"]["decode_equal"] for h in ok)
    if world == 1 and not args.no_cpu:
        # parity holds the last timed encode of the pristine batch (`ref`)
        try:
            cb = cpu_baseline(ref, parity, size, args.cpu_objects, args.cpu_seconds)
        except Exception as e:  # a host problem must not discard the GPU measurement
            cb = {"value": None, "error": f"{type(e).__name__}: {e}"}
        rec["cpu_baseline"] = cb
        checked = [c for c in [cb] + [cb.get(k) or {} for k in CPU_LEGS + ("scalar",)]
                   if "parity_vs_gpu" in c]
        rec["cpu_parity_checked"] = bool(checked)
        verified = verified and all(c["parity_vs_gpu"]["equal"] for c in checked)
    else:
        rec["cpu_parity_checked"] = False
    if world == 1 and not args.no_ceiling and hasattr(be, "pattern_ceiling_child"):
        # in a child process with the measurement library alone
        try:
            rec["roofline"]["pattern_ceiling"] = be.pattern_ceiling_child(n, size, 0x1E0E + lo)
        except Exception as e:  # never discard the measurement over the ceiling leg
            rec["roofline"]["pattern_ceiling"] = {"achieved": None,
                                                  "error": f"{type(e).__name__}: {e}"}
    rec["verified"] = verified
    return rec, verified


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """Start `--gpus` ranks of this script under torch.distributed.run as a
    child process (this process never touches the GPU) and return its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)]
    cmd += list(sys.argv[1:] if argv is None else argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def main(argv=None, backend=GpuBackend):
    args = parse(argv)
    if args.pattern_child:
        return pattern_child(args)
    if args.host_child:
        return host_child(args)
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            return launch_ranks(args, argv)
        world, rank, local = 1, 0, 0
    else:
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        be = backend(local, world, args.oversubscribe)
        rec, verified = run_rank(args, be, rank, world, dist)
        if rec is not None:
            print(json.dumps(rec), flush=True)
    finally:
        if dist is not None:
            dist.destroy_process_group()
    return 0 if verified else 1


if __name__ == "__main__":
    sys.exit(main())
