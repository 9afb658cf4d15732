"""Summarise a rocprofv3 kernel trace (rocpd .db or *_kernel_stats.csv /
*_kernel_trace.csv) into a per-kernel stats table.

    python tools/rocprof_summary.py gpurun_out/prof > profiles/<name>.txt
"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def from_db(path):
    c = sqlite3.connect(path)
    return [(r[0], r[1], r[2]) for r in c.execute("select name, start, end from kernels")]


def from_trace_csv(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return rows


def main(d):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        rows += from_db(p)
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += from_trace_csv(p)
    stats = defaultdict(list)
    for name, s, e in rows:
        stats[name].append(e - s)
    total = sum(sum(v) for v in stats.values()) or 1
    print(f"{'calls':>6} {'avg_us':>10} {'min_us':>10} {'max_us':>10} {'total_us':>12} {'pct':>6}  kernel")
    for name, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):6d} {sum(v)/len(v)/1e3:10.2f} {min(v)/1e3:10.2f} {max(v)/1e3:10.2f} "
              f"{sum(v)/1e3:12.1f} {100*sum(v)/total:6.1f}  {name[:140]}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
