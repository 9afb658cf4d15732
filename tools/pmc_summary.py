"""Summarise tools/pmc_passes.sh output: per counter, the value of the last
dispatch of the kernel matching a name fragment (summed over the dimensions
rocprofv3 reports), plus the kernel-trace average duration.

    python tools/pmc_summary.py gpurun_out/pmc_<tag> <kernel-name-fragment>
"""
import collections
import csv
import glob
import json
import os
import sys


def summarise(d, frag):
    out = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if frag not in r["Kernel_Name"]:
                continue
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        if per:
            out.update(per[max(per)])
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True):
        best = None  # the matching kernel launched most often (not a warm-up launch)
        for r in csv.DictReader(open(f)):
            if frag in r["Name"] and (best is None or int(r["Calls"]) > int(best["Calls"])):
                best = r
        # a 1-call match is a warm-up launch, not the launch the counters
        # (the last dispatch) describe: no duration then
        if best and int(best["Calls"]) > 1:
            out["avg_ns"] = float(best["AverageNs"])
            out["calls"] = int(best["Calls"])
            out["kernel"] = best["Name"]
    return out


if __name__ == "__main__":
    print(json.dumps(summarise(sys.argv[1], sys.argv[2]), indent=1, sort_keys=True))
