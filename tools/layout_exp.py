"""Does the HBM placement of objects/parity change the encode rate?

RS(10,4,8) 1 MiB x1024 encode with the shipped kernel, same algorithmic bytes,
different buffer layouts, interleaved rounds in one process (A/B fair):

  obj1M+sep     objects at 1 MiB stride, parity in its own buffer (bench.py)
  stripe        full stripes [n][(k+m)*bs], parity inside the stripe (suite)
  obj1.4M+sep   objects at the stripe stride, parity separate
  stripe1.5M    stripes padded to 1.5 MiB
  stripe+4K     stripes padded to a 4 KiB multiple
  obj1M+sep4K   parity stride padded to 4 KiB multiple

    python tools/layout_exp.py [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--alloc", type=int, default=0,
                    help="N separate allocations of one layout (placement effects)")
    ap.add_argument("--sweep", action="store_true",
                    help="object stride x parity stride grid (separate parity buffer)")
    args = ap.parse_args()
    import torch
    import leo_erasure_amd as le
    torch.cuda.set_device(0)
    assert le.gf_init() == "ok"
    K, M, W, size, n = 10, 4, 8, 1 << 20, 1024
    bs, _ = le.layout("vandrs", (K, M, W), size)
    r4k = lambda x: (x + 4095) // 4096 * 4096  # noqa: E731
    alg = (K + M) * bs * n

    def mk(obj_stride, par_stride, inside):
        if inside:
            buf = torch.empty((n, obj_stride), dtype=torch.uint8, device="cuda")
            objs, par = buf, buf[:, K * bs:]
        else:
            objs = torch.empty((n, obj_stride), dtype=torch.uint8, device="cuda")
            par = torch.empty((n, par_stride), dtype=torch.uint8, device="cuda")
        objs[:, :size].random_(0, 256)
        return objs, par

    if args.sweep:
        cases = {}
        for os_ in (size, size + 1024, size + 4096, k_bs := K * bs, size + size // 4, 2 * size):
            for ps in (M * bs, size, K * bs, 2 * size):
                cases[f"obj{os_}+par{ps}"] = mk(os_, ps, False)
    elif args.alloc:
        cases = {}
        for i in range(args.alloc):
            cases[f"alloc{i}:obj{K * bs}+par{K * bs}"] = mk(K * bs, K * bs, False)
            if i % 2:  # a 1 GiB hole between allocations
                cases[f"hole{i}"] = (torch.empty(1 << 30, dtype=torch.uint8, device="cuda"), None)
        cases = {c: v for c, v in cases.items() if v[1] is not None}
    else:
        cases = {}
    cases = cases or {
        "obj1M+sep": mk(size, M * bs, False),
        "stripe": mk((K + M) * bs, None, True),
        "obj1.4M+sep": mk((K + M) * bs, M * bs, False),
        "stripe1.5M": mk(3 << 19, None, True),
        "stripe+4K": mk(r4k((K + M) * bs), None, True),
        "obj1M+sep4K": mk(size, r4k(M * bs), False),
    }
    s = torch.cuda.current_stream()
    res = {c: [] for c in cases}

    def run(objs, par):
        le.device.encode("vandrs", (K, M, W), objs, size, par)

    for c, (o, p) in cases.items():
        for _ in range(10):
            run(o, p)
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for c, (o, p) in cases.items():
            for _ in range(5):
                run(o, p)
            evs = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                run(o, p)
                b.record(s)
                evs.append((a, b))
            torch.cuda.synchronize()
            res[c].append(statistics.median(a.elapsed_time(b) for a, b in evs))
    for c, ts in res.items():
        ms = statistics.median(ts)
        o, p = cases[c]
        print(json.dumps({"layout": c, "ms": round(ms, 4), "alg_GBps": round(alg / ms / 1e6, 1),
                          "frac": round(alg / ms / 1e6 / 8000, 4),
                          "rounds_ms": [round(t, 4) for t in ts],
                          "obj_ptr": hex(o.data_ptr()), "par_ptr": hex(p.data_ptr())}), flush=True)


if __name__ == "__main__":
    main()
