"""Why does repair read below encode on the same kernel?  RS(10,4,8) 1 MiB
x 1,024 (the suite's case), leoec_repair_dev with the output blocks laid out
three ways, and two repair-id sets, in interleaved rounds in one process:

  separate : one [n][bs] tensor per repaired id (bench_suite.py's layout)
  rows4    : one [n][4*bs] buffer, repaired id i at column i*bs (parity-like)
  rows10   : one [n][10*bs] buffer (the objects' row stride)

  ids [0,5,10,13] (the suite's) and [10,11,12,13] (survivors 0..9: the
  encode's coefficient rows, so only the layout differs from an encode)

Every output is checked against the encode's blocks once per layout.
    python tools/repair_layout.py [--rounds 4] [--reps 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tools.bench_suite import timed  # noqa: E402

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=1024)
    args = ap.parse_args()
    import torch
    import leo_erasure_amd as le
    torch.cuda.set_device(0)
    assert le.gf_init() == "ok"
    k, m, w, size, n = 10, 4, 8, 1 << 20, args.n
    bs, _ = le.layout("vandrs", (k, m, w), size)
    g = torch.Generator(device="cuda").manual_seed(0x1E0E)
    objs = torch.zeros((n, k * bs), dtype=torch.uint8, device="cuda")
    parity = torch.zeros((n, k * bs), dtype=torch.uint8, device="cuda")
    objs[:, :size] = torch.randint(0, 256, (n, size), dtype=torch.uint8, device="cuda", generator=g)
    le.device.encode("vandrs", (k, m, w), objs, size, parity)
    torch.cuda.synchronize()

    def blk(b):
        return objs[:, b * bs:] if b < k else parity[:, (b - k) * bs:]

    def outs_for(layout, nr):
        if layout == "separate":
            return [torch.empty((n, bs), dtype=torch.uint8, device="cuda") for _ in range(nr)]
        width = {"rows4": 4, "rows10": 10}[layout] * bs
        buf = torch.empty((n, width), dtype=torch.uint8, device="cuda")
        return [buf[:, i * bs:] for i in range(nr)]

    cases = []
    for ids in ([0, 5, 10, 13], [10, 11, 12, 13]):
        blocks = [None if b in ids else blk(b) for b in range(k + m)]
        for layout in ("separate", "rows4", "rows10"):
            outs = outs_for(layout, len(ids))
            fn = (lambda blocks=blocks, ids=ids, outs=outs:
                  le.device.repair("vandrs", (k, m, w), blocks, bs, ids, outs, n))
            fn()
            torch.cuda.synchronize()
            for i, b in enumerate(ids):
                assert torch.equal(outs[i][:, :bs], blk(b)[:, :bs]), (ids, layout, b)
            cases.append((str(ids), layout, fn))
    enc = lambda: le.device.encode("vandrs", (k, m, w), objs, size, parity)  # noqa: E731
    cases.append(("encode", "parity rows10", enc))
    alg = (k + 4) * bs * n
    res = {}
    for r in range(args.rounds):
        for ids, layout, fn in (cases if r % 2 == 0 else cases[::-1]):
            ms = timed(torch, fn, args.reps)
            res.setdefault((ids, layout), []).append(round(alg / ms / 1e6 / PEAK, 4))
            print(json.dumps({"round": r, "ids": ids, "out_layout": layout, "ms": round(ms, 4),
                              "frac_of_8TBps": round(alg / ms / 1e6 / PEAK, 4)}), flush=True)
    for (ids, layout), fr in res.items():
        fr = sorted(fr)
        print(json.dumps({"summary": True, "ids": ids, "out_layout": layout,
                          "median_frac": fr[len(fr) // 2], "all": fr}), flush=True)


if __name__ == "__main__":
    main()
