"""A/B the gf8_apply<10,4> measurement variants (LEOEC_GF8_VARIANT) on the
bench workload, interleaved round-robin in one process (§5.4 rule 24).

    python tools/kvariants.py [--rounds 8] [--reps 5] [--variants 1,2,3]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = {1: "shipped (lds+paired)", 2: "cpt2", 3: "branchy sgpr", 4: "branchy lds",
         5: "paired sgpr", 7: "copy-xor", 12: "no-nt", 15: "waves>=5", 16: "waves>=6 (spills)",
         17: "waves 8 (spills)", 20: "wg512", 21: "xcd-map", 22: "wg512+xcd-map", 23: "wg1024",
         24: "copy-xor xcd-map", 25: "wg64", 26: "wg128", 27: "copy-xor wg64", 28: "wg64 waves>=4",
         29: "wg64 waves>=6", 30: "buffer ld/st", 31: "copy-xor buffer", 32: "buffer auto-branchy",
         33: "ones row/col folded", 34: "xcd obj-interleave always"}
DEFAULT = [1, 7, 20, 21, 22, 23, 24]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default=",".join(str(v) for v in DEFAULT))
    ap.add_argument("--objects", type=int, default=1024)
    ap.add_argument("--burst", action="store_true",
                    help="launch the reps back to back, synchronise once (bench-like)")
    args = ap.parse_args()
    import torch
    os.environ.setdefault("LEOEC_LIBRARY", "measure")  # A/B knobs: libleoec_measure.so
    import leo_erasure_amd as le

    torch.cuda.set_device(0)
    assert le.gf_init() == "ok"
    K, M, W, size, n = 10, 4, 8, 1048576, args.objects
    bs, _ = le.layout("vandrs", (K, M, W), size)
    g = torch.Generator(device="cuda").manual_seed(7)
    objs = torch.randint(0, 256, (n, size), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((n, M * bs), dtype=torch.uint8, device="cuda")
    ref = objs.clone()
    variants = [int(v) for v in args.variants.split(",")]
    res = {v: {"enc": [], "dec": []} for v in variants}
    res["d2d-copy"] = {"enc": [], "dec": []}
    stream = torch.cuda.current_stream()
    alg = (K + M) * bs * n
    cp_src = torch.empty(alg // 2, dtype=torch.uint8, device="cuda")
    cp_dst = torch.empty_like(cp_src)
    for rnd in range(args.rounds):
        for v in variants:
            le._lib.measure_set_knob("LEOEC_GF8_VARIANT", v)  # measurement build
            evs = []
            for _ in range(args.reps):
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record(stream)
                le.device.encode("vandrs", (K, M, W), objs, size, parity)
                e[1].record(stream)
                le.device.decode("vandrs", (K, M, W), objs, size, parity, [0, 1, 2, 3])
                e[2].record(stream)
                if not args.burst:
                    torch.cuda.synchronize()
                evs.append(e)
            torch.cuda.synchronize()
            for e in evs:
                res[v]["enc"].append(e[0].elapsed_time(e[1]))
                res[v]["dec"].append(e[1].elapsed_time(e[2]))
            if NAMES.get(v, "").startswith("copy"):
                objs.copy_(ref)  # copy variants do not compute real parity
        for _ in range(args.reps):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record(stream)
            cp_dst.copy_(cp_src)
            e[1].record(stream)
            torch.cuda.synchronize()
            res["d2d-copy"]["enc"].append(e[0].elapsed_time(e[1]))
    le._lib.measure_set_knob("LEOEC_GF8_VARIANT", None)
    le.device.encode("vandrs", (K, M, W), objs, size, parity)
    le.device.decode("vandrs", (K, M, W), objs, size, parity, [0, 1, 2, 3])
    torch.cuda.synchronize()
    out = {}
    for v, r in res.items():
        me = statistics.median(r["enc"])
        row = {"name": NAMES.get(v, v), "enc_ms_med": round(me, 4), "enc_ms_min": round(min(r["enc"]), 4),
               "enc_GBps": round(alg / me / 1e6, 1)}
        if r["dec"]:
            md = statistics.median(r["dec"])
            row.update(dec_ms_med=round(md, 4), dec_GBps=round(alg / md / 1e6, 1))
        out[str(v)] = row
        print(json.dumps(row))
    print("intact_after_shipped_roundtrip", bool(torch.equal(objs, ref)))


if __name__ == "__main__":
    main()
