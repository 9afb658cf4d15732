"""bench.py's CPU-baseline placement (CPU only): workers go one per physical
core, on one NUMA node, on the least busy cores of a shared host; and the
pinned, first-touch timed baseline reproduces the oracle's parity."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _fake_sysfs(tmp_path, nodes, smt):
    """nodes x cores-per-node x smt hardware threads; cpu id = sibling-major
    (cpu c and c + ncores are siblings, as on the MI355X boxes' EPYC hosts)."""
    per, n = nodes[0], len(nodes)
    ncores = per * n
    for nd in range(n):
        cpus = [c for c in range(ncores * smt) if (c % ncores) // per == nd]
        d = tmp_path / "node" / f"node{nd}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(",".join(map(str, cpus)))
    for c in range(ncores * smt):
        d = tmp_path / "cpu" / f"cpu{c}" / "topology"
        d.mkdir(parents=True)
        sib = [c % ncores + i * ncores for i in range(smt)]
        (d / "thread_siblings_list").write_text(",".join(map(str, sib)))
    return str(tmp_path)


def test_one_worker_per_core_on_one_node(tmp_path, monkeypatch):
    sysfs = _fake_sysfs(tmp_path, [8, 8], 2)  # 2 nodes x 8 cores x 2 threads = 32 cpus
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(32)))
    busy = {c: 0.0 for c in range(32)}
    for c in range(0, 8):  # node 0 busy (another tenant)
        busy[c] = 0.9
    cpus, nodes = bench.pick_cpus(6, sysfs=sysfs, busy=busy)
    assert nodes == [1] and len(cpus) == 6
    cores = {c % 16 for c in cpus}
    assert len(cores) == 6  # no two workers on SMT siblings
    assert all(8 <= c % 16 < 16 for c in cpus)


def test_busy_sibling_makes_the_core_busy(tmp_path, monkeypatch):
    sysfs = _fake_sysfs(tmp_path, [4], 2)  # one node, 4 cores, cpus 0-7
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(8)))
    busy = {c: 0.0 for c in range(8)}
    busy[4] = 1.0  # sibling of cpu 0
    cpus, _ = bench.pick_cpus(3, sysfs=sysfs, busy=busy)
    assert 0 not in cpus and 4 not in cpus and len(cpus) == 3


def test_more_threads_than_cores_of_a_node(tmp_path, monkeypatch):
    sysfs = _fake_sysfs(tmp_path, [4, 4], 1)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(8)))
    cpus, nodes = bench.pick_cpus(6, sysfs=sysfs, busy={})
    assert len(set(cpus)) == 6 and nodes == [0, 1]


def test_pinned_baseline_parity(oracle):
    n, size = 24, 300001
    objs = np.random.default_rng(7).integers(0, 256, (n, size), dtype=np.uint8)
    bs = oracle.block_size(10, 8, size)
    par = np.zeros((n, 4 * bs), np.uint8)
    ref = np.zeros_like(par)
    cpus, _ = bench.pick_cpus(3)
    rates = oracle.bench_rs8_pinned(10, 4, objs, size, [0, 1, 2, 3], 3, cpus, 0.05, 0.2,
                                    parity_out=par)
    oracle.bench_rs8(0, 10, 4, objs, size, size, n, ref, threads=2)
    assert len(rates) >= 3 and all(r > 0 for r in rates)
    assert np.array_equal(par, ref)


def test_pinned_baseline_queue_ragged(oracle):
    """The baseline's shared object queue (chunks of 2): an odd object count,
    more workers than chunks; several rounds of encode + in-place decode keep
    the objects intact, so the last round's parity still equals the oracle's."""
    n, size = 5, 70001
    objs = np.random.default_rng(11).integers(0, 256, (n, size), dtype=np.uint8)
    bs = oracle.block_size(10, 8, size)
    par = np.zeros((n, 4 * bs), np.uint8)
    ref = np.zeros_like(par)
    cpus, _ = bench.pick_cpus(4)
    rates = oracle.bench_rs8_pinned(10, 4, objs, size, [0, 1, 2, 3], 4, cpus, 0.02, 0.1,
                                    parity_out=par)
    oracle.bench_rs8(0, 10, 4, objs, size, size, n, ref, threads=1)
    assert len(rates) >= 3 and all(r > 0 for r in rates)
    assert np.array_equal(par, ref)


@pytest.mark.parametrize("share,workers", [(16, 15), (8, 7), (2, 1), (1, 1)])
def test_headroom_rule(share, workers):
    """A share of N whole CPUs runs N - 1 workers (at least 1): the quota's
    last CPU is for the process's main, torch and HIP threads, so CFS
    bandwidth control does not throttle the passes."""
    assert bench.headroom_workers(share) == workers


@pytest.mark.parametrize("quota,threads,share_cpus", [("1600000 100000", 15, 16),
                                                     ("50000 100000", 1, 1),
                                                     ("max 100000", 15, 16)])
def test_cpu_share_leaves_one_cpu(tmp_path, monkeypatch, quota, threads, share_cpus):
    """16-CPU quota: 15 workers; a quota under one CPU still runs one worker
    (no negative reservation); no quota: the box's per-GPU share of 16."""
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(64)))
    real_open = open

    def fake_open(path, *a, **k):
        if path == "/sys/fs/cgroup/cpu.max":
            f = tmp_path / "cpu.max"
            f.write_text(quota + "\n")
            return real_open(f, *a, **k)
        return real_open(path, *a, **k)

    monkeypatch.setattr("builtins.open", fake_open)
    t, share = bench.cpu_share()
    assert t == threads and share["share_cpus"] == share_cpus
    assert share["reserved_cpus"] == share_cpus - threads >= 0


def test_throttled_passes_are_excluded():
    rates = [100.0, 101.0, 60.0, 99.0, 102.0, 70.0]
    thr = [0.0, 0.0, 0.4, 0.0, None, 0.2]
    s = bench.summarize_passes(rates, thr)
    assert s["throttled_passes"] == 2 and s["passes_used"] == "unthrottled"
    assert s["value"] == 101.0  # median of 99, 100, 101, 102
    # fewer than 3 clean passes: all passes, flagged
    s = bench.summarize_passes([50.0, 90.0, 91.0], [0.3, 0.0, 0.2])
    assert s["passes_used"].startswith("all") and s["value"] == 90.0


@pytest.mark.parametrize("structure", [1, 2])
def test_reference_structure_parity(oracle, structure):
    """The Jerasure-structure leg (per-(row, input) region passes, 1) and the
    scalar leg (2) write the same parity as the one-pass leg and the oracle."""
    n, size = 6, 200003
    objs = np.random.default_rng(3).integers(0, 256, (n, size), dtype=np.uint8)
    bs = oracle.block_size(10, 8, size)
    par = np.zeros((n, 4 * bs), np.uint8)
    ref = np.zeros_like(par)
    thr = []
    rates = oracle.bench_rs8_pinned(10, 4, objs, size, [0, 1, 2, 3], 2, None, 0.02, 0.06,
                                    parity_out=par, structure=structure, throttled=thr)
    oracle.bench_rs8(0, 10, 4, objs, size, size, n, ref, threads=1)
    assert len(rates) >= 3 and len(thr) == len(rates)
    assert np.array_equal(par, ref)


def test_warmup_passes_precede_the_timed_ones(oracle):
    """Untimed warm-up passes (a shared host ramps for seconds): at least one
    when warm_s > 0, at most until two agree within 3 % or warm_s elapses;
    none when warm_s = 0; parity unaffected."""
    n, size = 4, 100003
    objs = np.random.default_rng(5).integers(0, 256, (n, size), dtype=np.uint8)
    bs = oracle.block_size(10, 8, size)
    par = np.zeros((n, 4 * bs), np.uint8)
    ref = np.zeros_like(par)
    warm = []
    rates = oracle.bench_rs8_pinned(10, 4, objs, size, [0, 1, 2, 3], 2, None, 0.02, 0.06,
                                    parity_out=par, warm_s=0.1, warmup=warm)
    oracle.bench_rs8(0, 10, 4, objs, size, size, n, ref, threads=1)
    assert 1 <= len(warm) <= 64 and len(rates) >= 3 and all(r > 0 for r in warm + rates)
    # no two consecutive warm-up passes agree within 3 % before the last pair
    for a, b in zip(warm[:-2], warm[1:-1]):
        assert abs(b - a) > 0.03 * a
    assert np.array_equal(par, ref)
    warm0 = []
    oracle.bench_rs8_pinned(10, 4, objs, size, [0, 1, 2, 3], 2, None, 0.02, 0.06,
                            warm_s=0.0, warmup=warm0)
    assert warm0 == []


def _leg(value, equal=True, structure="x"):
    return {"value": value, "parity_vs_gpu": {"objects": 4, "equal": equal},
            "structure": structure, "cores": 15, "workers": 15, "share_cpus": 16,
            "kind": "port", "pinning": {"cpus": [0]}}


@pytest.mark.parametrize("port,ref,top", [
    (108.6, 113.5, "reference_structure"),  # the round-4 driver box: Jerasure's structure faster
    (117.7, 92.0, "isa_l_port"),
    (100.0, 130.0, "isa_l_port"),            # a faster leg whose parity differs never heads
])
def test_headline_is_the_faster_parity_equal_leg(port, ref, top):
    """cpu_baseline.value is the strongest CPU figure of the line (round-4
    verdict item 3): the faster of the two SIMD legs whose output equals the
    GPU's, the other kept under its name; the full-share estimate scales it
    by share / workers (round-4 advisor)."""
    ref_ok = not (port == 100.0)
    rec = bench.headline_cpu(_leg(port, structure="ISA-L"), _leg(ref, ref_ok, "Jerasure"))
    assert rec["headline_leg"] == top
    want = {"isa_l_port": port, "reference_structure": ref}
    assert rec["value"] == want[top]
    other = [x for x in bench.CPU_LEGS if x != top][0]
    assert rec[other]["value"] == want[other]
    assert rec["structure"] == ("ISA-L" if top == "isa_l_port" else "Jerasure")
    assert rec["cores"] == 15 and rec["pinning"] == {"cpus": [0]}
    assert rec["full_share_estimate_GiBps"] == pytest.approx(want[top] * 16 / 15, rel=1e-3)


def test_link_busy_counts_both_directions():
    """bench.link_busy: the share of a second an op's bytes keep the link
    busy at the one-direction rates (an encode moves its object in and m
    parity blocks out); 1.0 = serial copies back to back, above 1 the two
    directions overlap (the batching queue's copy streams)."""
    size, bs = 1 << 20, 104960
    link = {"h2d_GBps": 50.0, "d2h_GBps": 50.0}
    # encode at the rate where the object's bytes alone fill the H2D direction
    full_in = 50e9 / 2**30  # GiB/s of payload whose input bytes take 1 s per second
    busy = bench.link_busy({"encode_GiBps": full_in, "decode_GiBps": full_in}, link, size, bs)
    assert busy["encode"] == pytest.approx(1.0 + bench.M * bs / size, rel=1e-3)
    assert busy["decode"] == pytest.approx((bench.K + len(bench.ERASED)) * bs / size, rel=1e-3)


def test_host_child_refuses_torch(monkeypatch):
    """The host leg's child must run on the system HIP runtime: it refuses
    to run in a process that has torch (LEOEC_NO_TORCH unset)."""
    monkeypatch.delenv("LEOEC_NO_TORCH", raising=False)

    class A:
        host_data, size, pattern_device, host_seconds = "", 1 << 20, 0, 0.1
    with pytest.raises(RuntimeError, match="without torch"):
        bench.host_child(A())


def test_native_host_callers():
    """tools/libhost_callers.so (bench.py's host leg, built by build()):
    every thread calls the entry point back to back for the window, one call
    each outside it; failures are counted.  Driven here with a ctypes
    callback in place of leoec_encode (no GPU)."""
    import ctypes
    import bench
    if not os.path.exists(bench.HOST_CALLERS_LIB):
        pytest.skip("tools/libhost_callers.so not built")
    lib = ctypes.CDLL(bench.HOST_CALLERS_LIB)
    vp = ctypes.c_void_p
    lib.host_callers_run.restype = ctypes.c_long
    lib.host_callers_run.argtypes = [
        vp, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int,
        ctypes.c_int, vp, vp, ctypes.c_uint64, ctypes.c_uint64, vp, vp, ctypes.c_int,
        ctypes.c_uint64, vp, vp]
    ENC = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           vp, ctypes.c_uint64, vp, ctypes.c_uint64)
    seen = []

    for rc in (0, 3):
        def enc(coding, k, m, w, src, size, out, out_bytes, rc=rc):
            seen.append((coding, k, m, w, size, out_bytes))
            return rc
        cb = ENC(enc)
        n = 4
        srcs = (vp * n)(*range(1, n + 1))
        outs = (vp * n)(*range(11, 11 + n))
        counts = (ctypes.c_long * n)()
        el = ctypes.c_double()
        bad = lib.host_callers_run(ctypes.cast(cb, vp), 0, n, 0.05, 2, 10, 4, 8, srcs, outs, 1000,
                                   2000, None, None, 0, 0, counts, ctypes.byref(el))
        assert el.value >= 0.05
        assert all(c > 0 for c in counts), list(counts)
        assert bad == (0 if rc == 0 else sum(counts) + n)  # every call fails, first calls too
    assert seen[0] == (2, 10, 4, 8, 1000, 2000)
