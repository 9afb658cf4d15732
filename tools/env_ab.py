"""A/B of kernel-selection environment variables on one config, interleaved
rounds in one process (the engine reads its LEOEC_* knobs per launch).

    python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 \\
        --variants "LEOEC_GFBIT_PF=1;LEOEC_GFBIT_PF=0;LEOEC_GFBIT_LW=1"

Each variant is `;`-separated, its settings `,`-separated (empty = defaults).
Objects are laid out as in bench.py's family (object rows, separate parity),
after a >=0.3 s time-based warmup per variant.  Output: one JSON line per
(variant, op) with the median over rounds of the median launch time.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--coding", default="cauchyrs")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--w", type=int, default=8)
    ap.add_argument("--size", type=int, default=1 << 20)
    ap.add_argument("--objects", type=int, default=1024)
    ap.add_argument("--erased", default="0,1,2,3")
    ap.add_argument("--repair", default="",
                    help="block ids rebuilt by a timed repair (leoec_repair_dev from the other "
                         "blocks, outputs in one [n][r*bs] buffer); empty: no repair op")
    ap.add_argument("--variants", default="")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--par-offset", type=int, default=0,
                    help="bytes (multiple of 16) the parity rows start past their allocation's base")
    ap.add_argument("--obj-pad", type=int, default=0,
                    help="extra bytes (multiple of 16) per object row beyond max(k, m) * block size")
    args = ap.parse_args()
    import torch
    os.environ.setdefault("LEOEC_LIBRARY", "measure")  # A/B knobs: libleoec_measure.so
    import leo_erasure_amd as le
    torch.cuda.set_device(0)
    assert le.gf_init() == "ok"
    k, m, w = args.k, args.m, args.w
    p = (k, m, w)
    bs, _ = le.layout(args.coding, p, args.size)
    n = args.objects
    stride = max(k, m) * bs + args.obj_pad
    objs = torch.zeros((n, stride), dtype=torch.uint8, device="cuda")
    objs[:, :args.size].random_(0, 256)
    par_buf = torch.zeros(n * stride + args.par_offset, dtype=torch.uint8, device="cuda")
    par = par_buf[args.par_offset:].view(n, stride)
    ref = objs[:, :args.size].clone()
    er = [int(x) for x in args.erased.split(",") if x]
    e = len([x for x in er if x < k])
    variants = [v.strip() for v in args.variants.split(";")]
    keys = {kv.split("=")[0] for v in variants for kv in v.split(",") if kv}

    def setenv(v):
        for key in keys:  # knobs live in the measurement build (its setter)
            le._lib.measure_set_knob(key, None)
        for kv in v.split(","):
            if kv:
                a, b = kv.split("=")
                le._lib.measure_set_knob(a, b)

    ops = {"encode": (lambda: le.device.encode(args.coding, p, objs, args.size, par),
                      (k + m) * bs * n)}
    if er:
        ops["decode%s" % er] = (lambda: le.device.decode(args.coding, p, objs, args.size, par, er),
                                (k + e) * bs * n)
    rep = [int(x) for x in args.repair.split(",") if x]
    if rep:
        blocks = [objs[:, j * bs:] if j < k else par[:, (j - k) * bs:] for j in range(k + m)]
        for i in rep:
            blocks[i] = None
        rout = torch.zeros((n, len(rep) * bs), dtype=torch.uint8, device="cuda")
        routs = [rout[:, r * bs:] for r in range(len(rep))]
        ops["repair%s" % rep] = (lambda: le.device.repair(args.coding, p, blocks, bs, rep, routs, n),
                                 (k + len(rep)) * bs * n)
    s = torch.cuda.current_stream()
    res = {(v, o): [] for v in variants for o in ops}
    ok = {}
    for v in variants:  # correctness of every variant before timing
        setenv(v)
        ops["encode"][0]()
        if er:
            for i in er:  # clear the erased data blocks, then rebuild them
                if i < k:
                    objs[:, i * bs:min((i + 1) * bs, args.size)] = 0
            ops["decode%s" % er][0]()
        torch.cuda.synchronize()
        ok[v] = bool(torch.equal(objs[:, :args.size], ref))
        objs[:, :args.size].copy_(ref)
        if rep:
            rout.fill_(0x5A)
            ops["repair%s" % rep][0]()
            torch.cuda.synchronize()
            for r, i in enumerate(rep):
                src = objs[:, i * bs:(i + 1) * bs] if i < k else par[:, (i - k) * bs:(i - k + 1) * bs]
                # a data block past the object's size reads as zero
                want = src.clone()
                if i < k:
                    want[:, max(0, min(bs, args.size - i * bs)):] = 0
                ok[v] = ok[v] and bool(torch.equal(rout[:, r * bs:(r + 1) * bs], want))
    for _ in range(args.rounds):
        for v in variants:
            setenv(v)
            for o, (fn, _) in ops.items():
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 0.3:
                    for _ in range(10):
                        fn()
                    torch.cuda.synchronize()
                evs = []
                for _ in range(args.reps):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    fn()
                    b.record(s)
                    evs.append((a, b))
                torch.cuda.synchronize()
                res[(v, o)].append(statistics.median(x.elapsed_time(y) for x, y in evs))
    for (v, o), ts in res.items():
        ms = statistics.median(ts)
        alg = ops[o][1]
        print(json.dumps({"config": f"{args.coding}{p}", "variant": v or "default", "op": o,
                          "par_offset": args.par_offset, "obj_pad": args.obj_pad,
                          "size": args.size, "ms": round(ms, 4), "alg_GBps": round(alg / ms / 1e6, 1),
                          "frac": round(alg / ms / 1e6 / 8000, 4), "correct": ok[v]}), flush=True)


if __name__ == "__main__":
    main()
