"""Where the RS(10,4,8) repair's gap to encode comes from (measurement only).

The suite reads repair {0,5,10,13} at ~0.75 of 8 TB/s against encode ~0.79
and decode ~0.78, all the same gf8_apply<10,4> kernel over 14 block streams.
Two things differ: the map (encode's rows hold 13 coefficients equal to 1,
decode's and repair's are dense) and where the outputs live (encode and
decode write at the objects' row stride, the suite's repair into four dense
[n, bs] tensors).  This times, interleaved in one process, every combination
the two separate:

    python tools/repair_probe.py [--objects 1024] [--rounds 5] [--reps 20]

One JSON line per case (median over rounds of the per-round median launch).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench_suite import timed  # noqa: E402

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch

    import leo_erasure_amd as le
    le.gf_init()
    k, m, w, size, n = 10, 4, 8, 1 << 20, args.objects
    cls = "vandrs"
    bs, _ = le.layout(cls, (k, m, w), size)
    row = k * bs
    g = torch.Generator(device="cuda").manual_seed(0x1E0E)
    objs = torch.zeros((n, row), dtype=torch.uint8, device="cuda")
    parity = torch.zeros((n, row), dtype=torch.uint8, device="cuda")
    objs[:, :size] = torch.randint(0, 256, (n, size), dtype=torch.uint8, device="cuda", generator=g)
    le.device.encode(cls, (k, m, w), objs, size, parity)
    ref_par = parity[:, :m * bs].clone()
    ref_obj = objs.clone()
    work = objs.clone()

    def blk(b):
        return objs[:, b * bs:] if b < k else parity[:, (b - k) * bs:]

    dense = [torch.empty((n, bs), dtype=torch.uint8, device="cuda") for _ in range(4)]
    wide = torch.empty((n, row), dtype=torch.uint8, device="cuda")
    strided = [wide[:, r * bs:] for r in range(4)]
    packed4 = torch.empty((n, 4 * bs), dtype=torch.uint8, device="cuda")
    packed = [packed4[:, r * bs:] for r in range(4)]

    # four [n, bs] outputs in one allocation: end to end (bases n*bs apart),
    # and with each base rounded up to 2 MiB (as four separate allocations of
    # the caching allocator place them)
    nb = n * bs
    al = (nb + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    ends = torch.empty(4 * al, dtype=torch.uint8, device="cuda")
    end_to_end = [ends[r * nb:(r + 1) * nb].view(n, bs) for r in range(4)]
    aligned = [ends[r * al:r * al + nb].view(n, bs) for r in range(4)]
    bases = {"dense": [o.data_ptr() % (2 << 20) for o in dense],
             "end_to_end": [o.data_ptr() % (2 << 20) for o in end_to_end],
             "aligned": [o.data_ptr() % (2 << 20) for o in aligned]}
    print(json.dumps({"output bases mod 2 MiB": bases}), flush=True)

    def rep(ids, outs):
        blocks = [None if b in ids else blk(b) for b in range(k + m)]
        return lambda: le.device.repair(cls, (k, m, w), blocks, bs, ids, outs, n)

    cases = {
        "encode (parity at row stride k*bs)":
            lambda: le.device.encode(cls, (k, m, w), objs, size, parity),
        "decode [0,1,2,3] in place":
            lambda: le.device.decode(cls, (k, m, w), work, size, parity, [0, 1, 2, 3]),
        "repair [0,5,10,13] -> 4 dense [n,bs] (the suite's)": rep([0, 5, 10, 13], dense),
        "repair [0,5,10,13] -> 4 [n,bs] end to end in one buffer": rep([0, 5, 10, 13], end_to_end),
        "repair [0,5,10,13] -> 4 [n,bs] at 2 MiB-aligned bases": rep([0, 5, 10, 13], aligned),
        "repair [0,5,10,13] -> row stride k*bs": rep([0, 5, 10, 13], strided),
        "repair [0,5,10,13] -> row stride 4*bs": rep([0, 5, 10, 13], packed),
        "repair [0,1,2,3] -> 4 dense [n,bs]": rep([0, 1, 2, 3], dense),
        "repair [0,1,2,3] -> row stride k*bs (decode's map)": rep([0, 1, 2, 3], strided),
        "repair [10,11,12,13] -> row stride k*bs (encode's map)": rep([10, 11, 12, 13], strided),
        "repair [10,11,12,13] -> 4 dense [n,bs]": rep([10, 11, 12, 13], dense),
    }
    # every repair form checked once against the encoded object / parity
    for ids, outs in (([0, 5, 10, 13], dense), ([0, 5, 10, 13], strided), ([0, 5, 10, 13], packed),
                      ([0, 5, 10, 13], end_to_end), ([0, 5, 10, 13], aligned),
                      ([0, 1, 2, 3], dense), ([10, 11, 12, 13], strided)):
        rep(ids, outs)()
        torch.cuda.synchronize()
        for i, b in enumerate(ids):
            want = ref_obj[:, b * bs:(b + 1) * bs] if b < k else ref_par[:, (b - k) * bs:(b - k + 1) * bs]
            assert torch.equal(outs[i][:, :bs], want), f"repair {ids} block {b}"
    t = {c: [] for c in cases}
    for _ in range(args.rounds):
        for c, fn in cases.items():
            t[c].append(timed(torch, fn, args.reps))
    alg = (k + 4) * bs * n
    for c in cases:
        ms = statistics.median(t[c])
        print(json.dumps({"case": c, "ms": round(ms, 4), "frac": round(alg / ms / 1e6 / PEAK, 4),
                          "rounds_ms": [round(x, 4) for x in t[c]]}), flush=True)


if __name__ == "__main__":
    main()
