"""HBM bytes per launch of the bench kernels from rocprofv3 PMC passes.

FETCH_SIZE and WRITE_SIZE are collected in separate passes (TCC slots:
FETCH_SIZE takes 3, WRITE_SIZE 2) by tools/gpu_exp.sh, each over
`bench.py --steps 3 --warmup 1 --no-cpu`.  Both counters are in KiB.
Per MI355X_MICROARCH.md §HBM, on gfx950 FETCH_SIZE reports exactly half the
bytes of a wide (16 B/lane) coalesced streaming read: it is doubled here.
WRITE_SIZE reads 16-B-per-lane streaming stores exactly.  gf8_apply
dispatches alternate encode, decode (one bench step each).

    python tools/pmc_traffic.py gpurun_out > profiles/pmc_traffic.json
"""
import csv
import json
import os
import sys


def per_dispatch(path, counter, match):
    vals = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter or match not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return [vals[d] for d in sorted(vals)]


def main(out_dir, objects=1024, object_bytes=1048576, block_size=104960):
    match = "gf8_apply<10, 4, false"
    fetch = per_dispatch(os.path.join(out_dir, "pmc_fetch", "run_counter_collection.csv"),
                         "FETCH_SIZE", match)
    write = per_dispatch(os.path.join(out_dir, "pmc_write", "run_counter_collection.csv"),
                         "WRITE_SIZE", match)
    assert fetch and write and len(fetch) == len(write), (len(fetch), len(write))
    enc = [2 * f * 1024 + w * 1024 for f, w in zip(fetch[0::2], write[0::2])]
    dec = [2 * f * 1024 + w * 1024 for f, w in zip(fetch[1::2], write[1::2])]
    alg = 14 * block_size * objects
    rec = {
        "objects": objects, "object_bytes": object_bytes, "kernel": match + ">",
        "encode_bytes_per_launch": round(sum(enc) / len(enc)),
        "decode_bytes_per_launch": round(sum(dec) / len(dec)),
        "algorithmic_bytes_per_launch": alg,
        "encode_traffic_over_alg": round(sum(enc) / len(enc) / alg, 4),
        "decode_traffic_over_alg": round(sum(dec) / len(dec) / alg, 4),
        "raw_fetch_kib": fetch, "raw_write_kib": write,
        "method": "FETCH_SIZE*2*1024 + WRITE_SIZE*1024 (gfx950 streaming-read correction), "
                  "separate rocprofv3 --pmc passes over bench.py --steps 3 --warmup 1",
    }
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out",
         int(sys.argv[2]) if len(sys.argv) > 2 else 2048)
