"""Median GiB/s per (variant, op, callers) over the rounds of a
`tools/capi_bench few|mid` A/B whose logs are named <prefix>_{few,mid}_<variant>_<round>.log
(tools/gpu_r5_s26.sh).  Measurement only.

    python tools/summ_caps.py gpurun_out/r05_s26
"""
import collections
import glob
import json
import re
import statistics
import sys


def main():
    prefix = sys.argv[1]
    res = collections.defaultdict(list)
    for f in sorted(glob.glob(prefix + "_*.log")):
        m = re.match(r".*_(few|mid)_(.*)_(\d+)\.log$", f)
        if not m:
            continue
        v = m.group(2)
        for line in open(f):
            if line.startswith('{"path"'):
                d = json.loads(line)
                op = "enc" if "encode" in d["path"] else "dec"
                t = int(re.search(r"(\d+) caller", d["path"]).group(1))
                res[(v, op, t)].append(d["GiBps"])
    vs = sorted({k[0] for k in res})
    for op in ("enc", "dec"):
        for t in (1, 2, 4, 8, 16, 32):
            row = [f"{v.replace('LEOEC_HOSTQ_', '')}: {statistics.median(res[(v, op, t)]):.1f}"
                   for v in vs if res[(v, op, t)]]
            if row:
                print(op, t, " | ".join(row))


if __name__ == "__main__":
    main()
