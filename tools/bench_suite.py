"""Device-resident throughput of every BASELINE.json config (not the headline
line — bench.py is — but the same methodology): HIP events around each
launch on the launch stream, median of `reps`, algorithmic bytes / time.

    python tools/bench_suite.py [--reps 10] > profiles/<round>_suite.jsonl
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK = 8000.0


def timed(torch, fn, reps, warmup_s=0.2):
    """Median launch time with the launches back to back on one stream (as in
    bench.py), after at least `warmup_s` seconds of untimed launches: a short
    warmup after an idle gap (allocation, verification) measures the GPU
    still ramping its clocks — the first op of a config read ~12 % low."""
    stream = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warmup_s:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
    evs = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn()
        b.record(stream)
        evs.append((a, b))
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in evs)


def row(name, op, ms, alg, payload, extra=None):
    gbs = alg / ms / 1e6
    r = {"config": name, "op": op, "ms": round(ms, 4), "alg_GBps": round(gbs, 1),
         "frac_of_8TBps": round(gbs / PEAK, 4), "payload_GiBps": round(payload / ms * 1e3 / 2**30, 1)}
    if extra:
        r.update(extra)
    print(json.dumps(r), flush=True)
    return r


def stripe_case(torch, le, cls, k, m, w, size, n, reps, erased, repair_ids, name, verify=True,
                layout="object"):
    """layout "object" (bench.py's): objects at a k*bs row stride (zero pad after
    `size`), parity in its own buffer at the same row stride (leoec_repair_dev takes one
    stride for all k+m blocks).  layout "stripe": full stripes [n][(k+m)*bs],
    data blocks then coding blocks in one row — parity written next to the
    data it is read from, which costs HBM efficiency (tools/layout_exp.py)."""
    bs, _ = le.layout(cls, (k, m, w), size)
    g = torch.Generator(device="cuda").manual_seed(0x1E0E)
    if layout == "stripe":
        stride = (k + m) * bs
        buf = torch.zeros((n, stride), dtype=torch.uint8, device="cuda")
        objs, parity = buf, buf[:, k * bs:]
    else:
        stride = max(k, m) * bs  # >= size; the tail block's zero pad lies inside the row
        objs = torch.zeros((n, stride), dtype=torch.uint8, device="cuda")
        parity = torch.zeros((n, stride), dtype=torch.uint8, device="cuda")
    objs[:, :size] = torch.randint(0, 256, (n, size), dtype=torch.uint8, device="cuda", generator=g)
    ref = objs[:, :size].clone()
    extra = {"layout": layout}
    enc = lambda: le.device.encode(cls, (k, m, w), objs, size, parity)  # noqa: E731
    t_enc = timed(torch, enc, reps)
    out = []
    out.append(row(name, "encode", t_enc, (k + m) * bs * n, size * n, extra))
    if erased:
        dec = lambda: le.device.decode(cls, (k, m, w), objs, size, parity, erased)  # noqa: E731
        t_dec = timed(torch, dec, reps)
        e = len([x for x in erased if x < k])
        out.append(row(name, "decode%s" % erased, t_dec, (k + e) * bs * n, size * n, extra))
        out.append(row(name, "encode+decode", t_enc + t_dec, (2 * k + m + e) * bs * n,
                       2 * size * n, extra))
        if verify:
            objs[:, :e * bs] = 0
            dec()
            torch.cuda.synchronize()
            assert torch.equal(objs[:, :size], ref), f"{name}: decode mismatch"
    if repair_ids:
        def blk(b):
            return objs[:, b * bs:] if b < k else parity[:, (b - k) * bs:]
        blocks = [None if b in repair_ids else blk(b) for b in range(k + m)]
        r = len(repair_ids)
        # outputs per object, one [n, r*bs] buffer (as encode's parity), and
        # as r separate [n, bs] tensors: the same launch reads 4-5 % slower
        # into separate tensors (profiles/r05_s7_repair_probe.log,
        # r05_s8_repair_probe.log; not the HBM address aliasing of their
        # 2 MiB-aligned bases: end to end in one buffer reads the same)
        rows = torch.empty((n, r * bs), dtype=torch.uint8, device="cuda")
        forms = [("per-object rows", [rows[:, i * bs:] for i in range(r)]),
                 ("separate tensors", [torch.empty((n, bs), dtype=torch.uint8, device="cuda")
                                       for _ in repair_ids])]
        for form, outs in forms:
            rep = lambda: le.device.repair(cls, (k, m, w), blocks, bs, repair_ids, outs, n)  # noqa
            t_rep = timed(torch, rep, reps)
            out.append(row(name, "repair%s" % repair_ids, t_rep, (k + r) * bs * n, r * bs * n,
                           dict(extra, repair_out=form)))
            if verify:
                for i, b in enumerate(repair_ids):
                    assert torch.equal(outs[i][:, :bs], blk(b)[:, :bs]), f"{name}: repair {b}"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--variants", action="store_true", help="also the cauchyrs A/B forms")
    args = ap.parse_args()
    import torch

    os.environ.setdefault("LEOEC_LIBRARY", "measure")  # A/B knobs: libleoec_measure.so
    import leo_erasure_amd as le
    torch.cuda.set_device(0)
    assert le.gf_init() == "ok"
    MiB = 1 << 20
    R = args.reps
    stripe_case(torch, le, "vandrs", 4, 2, 8, MiB, 1024, R, [0, 1], [0, 5],
                "cfg0: vandrs RS(4,2,8) 1 MiB x1024 (GPU)")
    stripe_case(torch, le, "vandrs", 10, 4, 8, MiB, 1024, R, [0, 1, 2, 3], [0, 5, 10, 13],
                "cfg1/2: vandrs RS(10,4,8) 1 MiB x1024")
    stripe_case(torch, le, "vandrs", 10, 4, 8, MiB, 1024, R, [0, 1, 2, 3], [0, 5, 10, 13],
                "cfg1/2: vandrs RS(10,4,8) 1 MiB x1024", layout="stripe")
    stripe_case(torch, le, "cauchyrs", 10, 4, 8, MiB, 1024, R, [0, 1, 2, 3], [0, 5, 10, 13],
                "cfg3: cauchyrs(10,4,8) bitmatrix 1 MiB x1024")
    if args.variants:
        for env, label in [({"LEOEC_GFBIT_LW": "1"}, "lane 4 B"),
                           ({"LEOEC_GFBIT_LW": "4"}, "lane 16 B"),
                           ({"LEOEC_BITMATRIX": "1"}, "masked bitmatrix kernel")]:
            for k, v in env.items():  # knobs live in the measurement build
                le._lib.measure_set_knob(k, v)
            stripe_case(torch, le, "cauchyrs", 10, 4, 8, MiB, 1024, R, [0, 1, 2, 3], None,
                        "cfg3 variant (%s): cauchyrs(10,4,8) 1 MiB x1024" % label)
            le._lib.measure_reset_knobs()
    stripe_case(torch, le, "cauchyrs", 4, 2, 3, MiB, 1024, R, [0, 1], [0, 5],
                "cauchyrs(4,2,3) 1 MiB x1024 (the reference's default cauchyrs parameters)")
    stripe_case(torch, le, "vandrs", 10, 4, 8, 64 * MiB, 64, R, [0, 1, 2, 3], None,
                "cfg4: vandrs RS(10,4,8) 64 MiB x64 per GPU")
    stripe_case(torch, le, "isars", 10, 4, 8, MiB, 1024, R, [0, 1, 2, 3], [0, 5, 10, 13],
                "isars(10,4,8) 1 MiB x1024")
    stripe_case(torch, le, "liberation", 7, 2, 7, MiB, 1024, R, [0, 1], [0, 7],
                "liberation(7,2,7) 1 MiB x1024")
    stripe_case(torch, le, "liberation", 4, 2, 7, MiB, 1024, R, [0, 1], None,
                "liberation(4,2,7) 1 MiB x1024")
    stripe_case(torch, le, "liberation", 10, 2, 11, MiB, 1024, R, [0, 1], None,
                "liberation(10,2,11) 1 MiB x1024")
    stripe_case(torch, le, "vandrs", 10, 4, 8, 16 * MiB, 64, R, [0, 1, 2, 3], None,
                "vandrs RS(10,4,8) 16 MiB x64")
    stripe_case(torch, le, "vandrs", 10, 4, 16, MiB, 1024, R, [0, 1, 2, 3], None,
                "vandrs RS(10,4,16) 1 MiB x1024")
    stripe_case(torch, le, "vandrs", 10, 4, 32, MiB, 1024, R, [0, 1, 2, 3], None,
                "vandrs RS(10,4,32) 1 MiB x1024")
    if not args.skip_cpu:
        import bench
        # config 0 of BASELINE.json: RS(4,2,8) 1 MiB encode+decode on the CPU,
        # bench.py's baseline (pinned, first-touch, median pass) with k, m = 4, 2
        bench.K, bench.M, bench.ERASED = 4, 2, [0, 1]
        n = 1024
        g = torch.Generator(device="cuda").manual_seed(0x1E0E)
        objs = torch.randint(0, 256, (n, MiB), dtype=torch.uint8, device="cuda", generator=g)
        bs, _ = le.layout("vandrs", (4, 2, 8), MiB)
        parity = torch.empty((n, 2 * bs), dtype=torch.uint8, device="cuda")
        le.device.encode("vandrs", (4, 2, 8), objs, MiB, parity)
        torch.cuda.synchronize()
        t0 = time.time()
        cpu = bench.cpu_baseline(objs, parity, MiB, n, args.cpu_seconds)
        print(json.dumps({"config": "cfg0: vandrs RS(4,2,8) 1 MiB encode+decode, CPU port",
                          "cpu": cpu, "wall_s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
