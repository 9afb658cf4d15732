"""HBM bytes per launch of the bench kernels from rocprofv3 PMC passes.

FETCH_SIZE and WRITE_SIZE are collected in separate passes (TCC slots:
FETCH_SIZE takes 3, WRITE_SIZE 2) by tools/gpu_exp.sh, each over
`bench.py --steps 3 --warmup 1 --no-cpu`.  Both counters are in KiB.
Per MI355X_MICROARCH.md §HBM, on gfx950 FETCH_SIZE reports exactly half the
bytes of a wide (16 B/lane) coalesced streaming read: it is doubled here.
WRITE_SIZE reads 16-B-per-lane streaming stores exactly.  gf8_apply
dispatches alternate encode, decode (one bench step each).

    python tools/pmc_traffic.py gpurun_out > profiles/pmc_traffic.json

The record is stamped with the sha256 of the code object that defines
gf8_apply<10,4> in the library the passes ran on (leo_erasure_amd/codeobj.py):
bench.py prints the figure only while the loaded library holds that code.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from leo_erasure_amd import codeobj  # noqa: E402


def per_dispatch(path, counter, match):
    vals = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter or match not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return [vals[d] for d in sorted(vals)]


def main(out_dir, objects=2048, object_bytes=1048576, lib="leo_erasure_amd/libleoec.so",
         fetch_dir="pmc_fetch", write_dir="pmc_write", k=10, w=8):
    block_size = ((object_bytes + k * w - 1) // (k * w) + 15) // 16 * 16 * w  # rscoding.cpp:44
    match = "gf8_apply<10, 4, false"
    fetch = per_dispatch(os.path.join(out_dir, fetch_dir, "run_counter_collection.csv"),
                         "FETCH_SIZE", match)
    write = per_dispatch(os.path.join(out_dir, write_dir, "run_counter_collection.csv"),
                         "WRITE_SIZE", match)
    assert fetch and write and len(fetch) == len(write), (len(fetch), len(write))
    # bench.py --steps 3 --warmup 1: 4 steps of (encode, decode), then the
    # verification decodes, which are not counted
    fetch, write = fetch[:8], write[:8]
    enc = [2 * f * 1024 + w_ * 1024 for f, w_ in zip(fetch[0::2], write[0::2])]
    dec = [2 * f * 1024 + w_ * 1024 for f, w_ in zip(fetch[1::2], write[1::2])]
    alg = 14 * block_size * objects
    rec = {
        "objects": objects, "object_bytes": object_bytes, "block_size": block_size,
        "kernel": match + ">",
        "encode_bytes_per_launch": round(sum(enc) / len(enc)),
        "decode_bytes_per_launch": round(sum(dec) / len(dec)),
        "algorithmic_bytes_per_launch": alg,
        "encode_traffic_over_alg": round(sum(enc) / len(enc) / alg, 4),
        "decode_traffic_over_alg": round(sum(dec) / len(dec) / alg, 4),
        "code_object": {"kernel": "gf8_apply<10, 4>", "library": os.path.basename(lib),
                        "sha256": codeobj.kernel_code_object_sha256(lib)},
        "raw_fetch_kib": fetch, "raw_write_kib": write,
        "method": "FETCH_SIZE*2*1024 + WRITE_SIZE*1024 (gfx950 streaming-read correction), "
                  "separate rocprofv3 --pmc passes over bench.py (encode, decode alternate)",
    }
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir", nargs="?", default="gpurun_out")
    ap.add_argument("--objects", type=int, default=2048)
    ap.add_argument("--object-bytes", type=int, default=1048576)
    ap.add_argument("--fetch", default="pmc_fetch")
    ap.add_argument("--write", default="pmc_write")
    ap.add_argument("--lib", default="leo_erasure_amd/libleoec.so")
    a = ap.parse_args()
    main(a.out_dir, a.objects, a.object_bytes, a.lib, a.fetch, a.write)
