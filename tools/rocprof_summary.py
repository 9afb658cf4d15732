"""Summarise a rocprofv3 kernel trace (rocpd .db or *_kernel_stats.csv /
*_kernel_trace.csv) into a per-kernel stats table.

    python tools/rocprof_summary.py gpurun_out/prof > profiles/<name>.txt
    python tools/rocprof_summary.py --by-launch gpurun_out/prof   # per (kernel, grid, VGPRs)

--by-launch (rocpd .db, or a kernel_trace.csv) splits a kernel's launches by grid size, so one
kernel run over several configs (objects x block sizes) reads per config.
"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def from_db(path, by_launch=False):
    c = sqlite3.connect(path)
    if not by_launch:
        return [(r[0], r[1], r[2]) for r in c.execute("select name, start, end from kernels")]
    q = "select name, start, end, grid_x, workgroup_x, vgpr_count, accum_vgpr_count from kernels"
    return [(f"{r[0][:110]} | grid {r[3]} wg {r[4]} vgpr {r[5] + (r[6] or 0)}", r[1], r[2])
            for r in c.execute(q)]


def from_trace_csv(path, by_launch=False):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"]
            if by_launch:
                vg = int(r.get("VGPR_Count") or 0) + int(r.get("Accum_VGPR_Count") or 0)
                name = f"{name[:110]} | grid {r['Grid_Size_X']} wg {r['Workgroup_Size_X']} vgpr {vg}"
            rows.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return rows


def main(d, by_launch=False):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        rows += from_db(p, by_launch)
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += from_trace_csv(p, by_launch)
    stats = defaultdict(list)
    for name, s, e in rows:
        stats[name].append(e - s)
    total = sum(sum(v) for v in stats.values()) or 1
    print(f"{'calls':>6} {'avg_us':>10} {'min_us':>10} {'max_us':>10} {'total_us':>12} {'pct':>6}  kernel")
    for name, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):6d} {sum(v)/len(v)/1e3:10.2f} {min(v)/1e3:10.2f} {max(v)/1e3:10.2f} "
              f"{sum(v)/1e3:12.1f} {100*sum(v)/total:6.1f}  {name[:170]}")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--by-launch"]
    main(args[0] if args else "gpurun_out/prof", "--by-launch" in sys.argv)
