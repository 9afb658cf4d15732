"""bench.py's own rank logic on CPU (bench.main -> run_rank), with the device
calls stubbed by the CPU oracle: world_size-2 gloo ranks shard the objects
with no data-path collective, time with a barrier + max over ranks, and the
line's `verified` flag fails for a decode that writes nothing."""
import contextlib
import io
import json
import os
import socket
import sys
import time

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class CpuEvent:
    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class CpuBackend:
    """bench.GpuBackend's interface over host tensors; encode/decode are the
    oracle's batch driver (the same ops the GPU runs)."""

    def __init__(self, local_rank, world, oversubscribe=False):
        self.name = f"cpu-stub:{local_rank}"

    def random_batch(self, n, size, seed):
        g = torch.Generator().manual_seed(seed)
        return torch.randint(0, 256, (n, size), dtype=torch.uint8, generator=g)

    def empty(self, n, cols):
        return torch.empty((n, cols), dtype=torch.uint8)

    def encode(self, objs, size, parity):
        from oracle import oracle as O
        O.bench_rs8(0, bench.K, bench.M, objs.numpy(), objs.stride(0), size, objs.shape[0],
                    parity.numpy(), threads=1)

    def decode(self, objs, size, parity, erased):
        from oracle import oracle as O
        O.bench_rs8(1, bench.K, bench.M, objs.numpy(), objs.stride(0), size, objs.shape[0],
                    parity.numpy(), erased=erased, threads=1)

    def sync(self):
        pass

    def event(self):
        return CpuEvent()

    def host_path(self, objs, parity, size, bs, callers=32, seconds=1.0):
        """bench.GpuBackend.host_path's record over the oracle's one-object
        calls (the host-memory API's outputs: tail data block + parity)."""
        from oracle import oracle as O
        n = min(callers, objs.shape[0], 2)
        t0 = time.perf_counter()
        enc_ok = dec_ok = True
        for t in range(n):
            data = objs[t, :size].numpy().tobytes()
            blocks = O.encode("vandrs", bench.K, bench.M, bench.W, data)
            enc_ok &= b"".join(blocks[bench.K:]) == parity[t].numpy().tobytes()
            dec_ok &= b"".join(blocks[:bench.K])[:size] == data
        dt = max(time.perf_counter() - t0, 1e-9)
        rate = n * size / dt / 2**30
        return {"encode_GiBps": round(rate, 4), "decode_GiBps": round(rate, 4), "callers": n,
                "seconds_per_op": seconds, "calls": [n, n],
                "parity_vs_gpu": {"objects": n, "encode_equal": enc_ok, "decode_equal": dec_ok},
                "what": "cpu stub"}


class NoopDecode(CpuBackend):
    def decode(self, objs, size, parity, erased):
        pass


class ZeroEncode(CpuBackend):
    def encode(self, objs, size, parity):
        parity.zero_()


class BadHost(CpuBackend):
    """Rank 1's host-memory leg reports parity that differs from the GPU's."""

    def __init__(self, local_rank, world, oversubscribe=False):
        super().__init__(local_rank, world, oversubscribe)
        self.rank = local_rank

    def host_path(self, *a, **kw):
        rec = super().host_path(*a, **kw)
        if self.rank == 1:
            rec["parity_vs_gpu"]["encode_equal"] = False
        return rec


BACKENDS = {"cpu": CpuBackend, "noop_decode": NoopDecode, "zero_encode": ZeroEncode,
            "bad_host": BadHost}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, argv, backend, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      LOCAL_RANK=str(rank), WORLD_SIZE=str(world))
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        rc = bench.main(argv, backend=BACKENDS[backend])
    q.put((rank, rc, out.getvalue()))


def _run_ranks(world, argv, backend="cpu"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, argv, backend, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


SMALL = ["--steps", "3", "--warmup", "1", "--warmup-s", "0", "--size", "65536"]


def test_two_ranks_weak_scaling_through_bench_main():
    res = _run_ranks(2, ["--gpus", "2", "--objects", "5"] + SMALL)
    (r0, rc0, out0), (r1, rc1, out1) = res
    assert rc0 == 0 and rc1 == 0
    assert out1 == ""                       # one line, from rank 0
    rec = json.loads(out0)
    assert rec["n_gpus"] == 2 and rec["scaling"] == "weak" and rec["verified"] is True
    assert [r["objects"] for r in rec["per_rank"]] == [[0, 5], [5, 10]]
    assert rec["config"]["global_objects"] == 10
    assert rec["cpu_baseline"] is None      # rank 0 at N=1 only
    # value = all ranks' objects / the slowest rank's time
    el = max(r["elapsed_s"] for r in rec["per_rank"])
    assert rec["value"] == pytest.approx(2 * 10 * 65536 * 3 / el / 2**30, rel=2e-2)
    assert all(all(r["checks"].values()) for r in rec["per_rank"])
    # the whole node's roofline: every rank's bytes over the slowest launch
    bs = rec["config"]["block_size"]
    agg = rec["roofline"]["aggregate"]
    assert agg["n_gpus"] == 2
    for op, per_obj, key, fkey in (("encode", 14 * bs, "encode_ms", "encode_frac"),
                                   ("decode", 14 * bs, "decode_ms", "decode_frac")):
        a = agg[op]
        slow = max(r[key] for r in rec["per_rank"])
        assert a["alg_bytes_per_launch"] == 10 * per_obj
        assert a["slowest_rank_launch_ms"] == pytest.approx(slow, abs=1e-4)
        assert a["peak"] == 2 * bench.HBM_PEAK_GBS
        assert a["frac"] == pytest.approx(a["achieved"] / a["peak"], rel=1e-3, abs=6e-5)
        for r in rec["per_rank"]:  # each rank against one GPU's peak
            assert r[fkey] == pytest.approx(5 * per_obj / (r[key] * 1e-3) / 1e9 / 8000.0,
                                            rel=1e-2, abs=6e-5)
    assert rec["cpu_parity_checked"] is False
    # the host-memory leg: every rank its own, the node's rate their sum
    hp = rec["host_path"]
    assert len(hp["per_rank"]) == 2
    for op in ("encode_GiBps", "decode_GiBps"):
        assert hp[op] == pytest.approx(sum(h[op] for h in hp["per_rank"]), abs=0.006)
    assert all(h["parity_vs_gpu"]["encode_equal"] and h["parity_vs_gpu"]["decode_equal"]
               for h in hp["per_rank"])
    assert hp["callers"] == sum(h["callers"] for h in hp["per_rank"])


def test_host_leg_parity_failure_fails_the_line():
    """A host-path leg whose outputs differ from the GPU's fails `verified`."""
    res = _run_ranks(2, ["--gpus", "2", "--objects", "3"] + SMALL, backend="bad_host")
    (r0, rc0, out0), (r1, rc1, out1) = res
    rec = json.loads(out0)
    assert rec["verified"] is False and rc0 == 1
    assert rec["host_path"]["per_rank"][1]["parity_vs_gpu"]["encode_equal"] is False


def test_host_leg_can_be_skipped():
    res = _run_ranks(2, ["--gpus", "2", "--objects", "3", "--no-host"] + SMALL)
    rec = json.loads(res[0][2])
    assert "host_path" not in rec and rec["verified"] is True


def test_two_ranks_partitioned_batch():
    """configs[4]: one global batch split with shard_range (strong scaling)."""
    res = _run_ranks(2, ["--gpus", "2", "--workload", "64MiB", "--objects", "7"] + SMALL)
    rec = json.loads(res[0][2])
    assert rec["scaling"] == "strong" and rec["verified"] is True
    assert [r["objects"] for r in rec["per_rank"]] == [[0, 3], [3, 7]]
    assert rec["config"]["global_objects"] == 7


def test_noop_decode_fails_verification_on_a_rank():
    res = _run_ranks(2, ["--gpus", "2", "--objects", "3"] + SMALL, backend="noop_decode")
    rec = json.loads(res[0][2])
    assert rec["verified"] is False
    assert res[0][1] == 1 and res[1][1] == 1
    assert not rec["per_rank"][1]["checks"]["poisoned_decode_0_1_2_3"]


def test_single_rank_cpu_leg_checks_parity(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    argv = ["--objects", "4", "--cpu-seconds", "0.05", "--cpu-objects", "3"] + SMALL
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        rc = bench.main(argv, backend=CpuBackend)
    rec = json.loads(out.getvalue())
    assert rc == 0 and rec["verified"] is True and rec["n_gpus"] == 1
    cb = rec["cpu_baseline"]
    assert cb["parity_vs_gpu"] == {"objects": 3, "equal": True}
    assert cb["cores"] >= 1 and cb["host_cpus"] >= cb["cores"] and cb["affinity_cpus"] >= 1
    # one CPU of the share left to the process's other threads
    assert cb["workers"] == cb["cores"] and cb["cores"] <= max(1, cb["share_cpus"] - 1)
    assert len(cb["throttled_s_per_pass"]) == len(cb["passes_GiBps"])
    assert len(cb["warmup_passes_GiBps"]) >= 1
    # both SIMD legs (the ISA-L-technique port and the reference's own CPU
    # structure), same sample, same parity check; the faster one on top
    top = cb["headline_leg"]
    assert top in bench.CPU_LEGS
    other = cb[[x for x in bench.CPU_LEGS if x != top][0]]
    assert other["parity_vs_gpu"] == {"objects": 3, "equal": True}
    assert other["value"] > 0 and other["cores"] == cb["cores"] and cb["value"] >= other["value"]
    rs = cb if top == "reference_structure" else other
    assert "Jerasure" in rs["structure"]
    sc = cb["scalar"]
    assert sc["parity_vs_gpu"] == {"objects": 3, "equal": True} and sc["simd"] == "scalar"
    assert rec["cpu_parity_checked"] is True


def test_single_rank_failed_cpu_leg_is_recorded(monkeypatch):
    """A CPU leg that raises keeps the GPU measurement, and the line says
    that no CPU-vs-GPU parity check ran."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)

    def boom(*a, **k):
        raise OSError("no host cores")

    monkeypatch.setattr(bench, "cpu_baseline", boom)
    argv = ["--objects", "3", "--no-ceiling"] + SMALL
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        rc = bench.main(argv, backend=CpuBackend)
    rec = json.loads(out.getvalue())
    assert rc == 0 and rec["cpu_baseline"]["value"] is None
    assert "no host cores" in rec["cpu_baseline"]["error"]
    assert rec["cpu_parity_checked"] is False


class WithCeiling(CpuBackend):
    calls = []

    def pattern_ceiling_child(self, n, size, seed):
        WithCeiling.calls.append((n, size, seed))
        return {"achieved": 1.0, "shipped_over_ceiling": 0.5}


class BrokenCeiling(CpuBackend):
    def pattern_ceiling_child(self, n, size, seed):
        raise RuntimeError("no measurement build")


def test_single_rank_pattern_ceiling_leg(monkeypatch):
    """The live pattern-ceiling leg runs once at N = 1 after the timed region
    (in a child process that regenerates the rank's seeded batch: the bench
    process loads one HIP library) and lands in `roofline`; a failing leg is
    recorded and never fails the measurement."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    argv = ["--objects", "3", "--no-cpu"] + SMALL
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        rc = bench.main(argv, backend=WithCeiling)
    rec = json.loads(out.getvalue())
    assert rc == 0 and rec["verified"] is True
    assert rec["roofline"]["pattern_ceiling"] == {"achieved": 1.0, "shipped_over_ceiling": 0.5}
    assert WithCeiling.calls == [(3, 65536, 0x1E0E)]  # the batch's own seed
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        rc = bench.main(argv, backend=BrokenCeiling)
    rec = json.loads(out.getvalue())
    assert rc == 0 and rec["verified"] is True
    assert rec["roofline"]["pattern_ceiling"]["achieved"] is None
    assert "no measurement build" in rec["roofline"]["pattern_ceiling"]["error"]
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        bench.main(argv + ["--no-ceiling"], backend=WithCeiling)
    assert "pattern_ceiling" not in json.loads(out.getvalue())["roofline"]


def test_single_rank_wrong_parity_fails(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    argv = ["--objects", "3", "--cpu-seconds", "0.01", "--cpu-objects", "2"] + SMALL
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        rc = bench.main(argv, backend=ZeroEncode)
    rec = json.loads(out.getvalue())
    assert rc == 1 and rec["verified"] is False
    assert rec["cpu_baseline"]["parity_vs_gpu"]["equal"] is False


def test_gpus_flag_launches_ranks(monkeypatch):
    """--gpus N without a launcher starts N ranks in a child process (before
    any GPU call) and returns its status."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    assert bench.main(["--gpus", "4", "--steps", "5"]) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-3:] == ["--gpus", "4", "--steps", "5"][-3:]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_gpus_must_match_world(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.main(["--gpus", "4"], backend=CpuBackend) == 2


@pytest.mark.parametrize("world,total", [(2, 1024), (2, 7), (8, 64), (3, 2)])
def test_shard_range_tiles_the_batch(world, total):
    spans = [bench.shard_range(r, world, total) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
