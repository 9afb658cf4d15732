"""Summarise tools/pmc_ops.sh output: per op, the median per-dispatch value of
every counter over the op's kernel dispatches (the first dispatch, a warm-up
encode, is dropped), plus HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B;
gfx950 streaming-read correction, MI355X_MICROARCH.md §HBM).

    python tools/pmc_summary.py gpurun_out/pmc_ops
"""
import csv
import glob
import json
import os
import statistics
import sys


def load(d):
    per = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
                per.setdefault(key, {}).setdefault(r["Counter_Name"], 0.0)
                per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    return per


def main(root):
    names = sorted({os.path.basename(p).rsplit("_g", 1)[0] for p in glob.glob(os.path.join(root, "*_g*"))
                    if os.path.isdir(p)})
    for name in names:
        out = {"op": name}
        for d in sorted(glob.glob(os.path.join(root, name + "_g*"))):
            if not os.path.isdir(d):
                continue
            per = load(d)
            keys = sorted(per)[1:]  # drop the warm-up dispatch
            if not keys:
                continue
            out["kernel"] = keys[-1][1][:90]
            for c in per[keys[0]]:
                out[c] = statistics.median(per[k][c] for k in keys if c in per[k])
        if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
            out["hbm_bytes"] = 2 * out["FETCH_SIZE"] * 1024 + out["WRITE_SIZE"] * 1024
        if "SQ_ACTIVE_INST_VALU" in out and "SQ_BUSY_CYCLES" in out:
            out["valu_active_per_busy"] = out["SQ_ACTIVE_INST_VALU"] / max(1.0, out["SQ_BUSY_CYCLES"])
        print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_ops")
