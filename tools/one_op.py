"""Run one device-resident op of one config repeatedly (a clean target for
rocprofv3 --pmc / --kernel-trace passes on a single kernel).

    python tools/one_op.py --coding cauchyrs --k 10 --m 4 --w 8 --op encode --reps 20
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--coding", default="cauchyrs")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--w", type=int, default=8)
    ap.add_argument("--size", type=int, default=1 << 20)
    ap.add_argument("--objects", type=int, default=1024)
    ap.add_argument("--op", choices=["encode", "decode", "repair"], default="encode")
    ap.add_argument("--erased", default="0,1,2,3",
                    help="decode: data blocks lost; repair: block ids rebuilt")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--knobs", default="",
                    help="K=V,K=V: measurement-build knobs (loads libleoec_measure.so)")
    args = ap.parse_args()
    if args.knobs:  # before the package loads its library
        os.environ["LEOEC_LIBRARY"] = "measure"
    import torch
    import leo_erasure_amd as le
    for kv in filter(None, args.knobs.split(",")):
        k, _, v = kv.partition("=")
        le._lib.measure_set_knob(k, v)
    torch.cuda.set_device(0)
    assert le.gf_init() == "ok"
    p = (args.k, args.m, args.w)
    bs, _ = le.layout(args.coding, p, args.size)
    stride = max(args.k, args.m) * bs
    objs = torch.zeros((args.objects, stride), dtype=torch.uint8, device="cuda")
    objs[:, :args.size].random_(0, 256)
    par = torch.zeros((args.objects, stride), dtype=torch.uint8, device="cuda")
    er = [int(x) for x in args.erased.split(",")]
    le.device.encode(args.coding, p, objs, args.size, par)
    if args.op == "repair":
        # survivors: every block but the rebuilt ones, as [n][stride] row
        # views (data blocks in the object rows, coding blocks in the parity
        # rows); the rebuilt blocks go to one [n][r*bs] buffer (repair reads
        # at the encode's rate with its outputs adjacent)
        k, m = args.k, args.m
        blocks = [objs[:, j * bs:] if j < k else par[:, (j - k) * bs:] for j in range(k + m)]
        for i in er:
            blocks[i] = None
        out = torch.empty((args.objects, len(er) * bs), dtype=torch.uint8, device="cuda")
        outs = [out[:, r * bs:] for r in range(len(er))]
    for _ in range(args.reps):
        if args.op == "encode":
            le.device.encode(args.coding, p, objs, args.size, par)
        elif args.op == "decode":
            le.device.decode(args.coding, p, objs, args.size, par, er)
        else:
            le.device.repair(args.coding, p, blocks, bs, er, outs, args.objects)
    torch.cuda.synchronize()
    print("one_op done", args.coding, p, args.op, "bs", bs)


if __name__ == "__main__":
    main()
