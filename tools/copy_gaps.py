"""Where the host path's link time goes: the H2D direction's busy fraction,
the gaps between consecutive batch H2D copies, and the batches on the GPU
when each gap opens, from a rocprofv3 copy trace of the C-ABI bench
(round 6, verdict r5 item 3):

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d D -o run \\
        -- tools/capi_bench leo_erasure_amd/libleoec_measure.so trace32
    python tools/copy_gaps.py D

The batching queue (csrc/hostq.cpp) puts every batch's H2D on one copy
stream and every batch's D2H on another, so the H2D stream with the most
busy time is the queue's; its copies are the batches in launch order, and
the D2H stream's copies match them one for one.  The trace is cut into
trials at idle spans longer than --split-ms (capi_bench runs encode trials,
then decode trials, with thread start-up between them).  Per trial: the
H2D stream's busy fraction, gap percentiles, the share of idle time in gaps
of each size, and for each gap the number of batches whose H2D had started
and whose D2H had not ended when it opened (batches on the GPU).
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def col(row, *frags):
    for k in row:
        kl = k.lower()
        if all(f in kl for f in frags):
            return k
    return None


def load_copies(d):
    files = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    if not files:
        raise SystemExit("no memory_copy_trace.csv under %s" % d)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    r0 = rows[0]
    k_dir = col(r0, "direction") or col(r0, "kind")
    k_s, k_e = col(r0, "start"), col(r0, "end")
    k_st = col(r0, "stream")
    k_b = col(r0, "bytes") or col(r0, "size")
    out = []
    for r in rows:
        dirn = r[k_dir].upper()
        kind = "H2D" if ("HOST_TO_DEVICE" in dirn or dirn.endswith("H2D")) else \
               "D2H" if ("DEVICE_TO_HOST" in dirn or dirn.endswith("D2H")) else dirn
        out.append({"kind": kind, "s": int(r[k_s]), "e": int(r[k_e]),
                    "stream": r[k_st] if k_st else "?", "bytes": int(r[k_b]) if k_b and r[k_b] else None})
    return out, list(r0.keys())


def pct(xs, p):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(p / 100.0 * len(xs)))] if xs else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--split-ms", type=float, default=30.0)
    ap.add_argument("--min-bytes", type=int, default=1 << 20)
    a = ap.parse_args()
    copies, cols = load_copies(a.dir)
    busy = collections.Counter()
    for c in copies:
        busy[(c["kind"], c["stream"])] += c["e"] - c["s"]
    h2d_stream = max((k for k in busy if k[0] == "H2D"), key=lambda k: busy[k])[1]
    d2h_stream = max((k for k in busy if k[0] == "D2H"), key=lambda k: busy[k])[1]
    big = lambda c: c["bytes"] is None or c["bytes"] >= a.min_bytes  # noqa: E731
    h = sorted((c for c in copies if c["kind"] == "H2D" and c["stream"] == h2d_stream and big(c)),
               key=lambda c: c["s"])
    dn = sorted((c for c in copies if c["kind"] == "D2H" and c["stream"] == d2h_stream),
                key=lambda c: c["s"])
    d_ends = sorted(c["e"] for c in dn)
    h_starts = [c["s"] for c in h]
    # trials: runs of H2Ds without an idle span longer than split-ms
    trials, cur = [], [h[0]]
    for c in h[1:]:
        if c["s"] - cur[-1]["e"] > a.split_ms * 1e6:
            trials.append(cur)
            cur = []
        cur.append(c)
    trials.append(cur)
    rep = {"columns": cols, "h2d_stream": h2d_stream, "d2h_stream": d2h_stream,
           "streams_busy_ms": {"%s %s" % k: v / 1e6 for k, v in busy.most_common(8)}, "trials": []}
    import bisect
    for t in trials:
        if len(t) < 20:
            continue
        span = t[-1]["e"] - t[0]["s"]
        b = sum(c["e"] - c["s"] for c in t)
        gaps, onq = [], []
        for i in range(len(t) - 1):
            g = t[i + 1]["s"] - t[i]["e"]
            gaps.append(g / 1e3)
            at = t[i]["e"]
            started = bisect.bisect_right(h_starts, at)
            returned = bisect.bisect_right(d_ends, at)
            onq.append(started - returned)
        dur = [(c["e"] - c["s"]) / 1e3 for c in t]
        byt = [c["bytes"] for c in t if c["bytes"]]
        idle = sum(max(g, 0) for g in gaps)
        buckets = collections.OrderedDict()
        for lo, hi in [(-1e9, 5), (5, 20), (20, 50), (50, 100), (100, 1e9)]:
            sel = [g for g in gaps if lo <= g < hi]
            buckets["%g-%g us" % (max(lo, 0), hi)] = {"n": len(sel), "idle_share": sum(max(x, 0) for x in sel) / idle if idle else 0}
        by_q = collections.defaultdict(list)
        for g, q in zip(gaps, onq):
            by_q[q].append(g)
        rep["trials"].append({
            "batches": len(t), "span_ms": span / 1e6, "h2d_busy_frac": b / span,
            "h2d_us_median": statistics.median(dur),
            "h2d_bytes_median": statistics.median(byt) if byt else None,
            "h2d_GBps_median": (statistics.median(byt) / statistics.median(dur) / 1e3) if byt else None,
            "gap_us": {"p10": pct(gaps, 10), "p50": pct(gaps, 50), "p90": pct(gaps, 90),
                       "p99": pct(gaps, 99), "mean": statistics.mean(gaps)},
            "idle_by_gap_size": buckets,
            "batches_on_gpu_at_gap": {str(q): {"gaps": len(v), "mean_gap_us": statistics.mean(v)}
                                      for q, v in sorted(by_q.items())},
        })
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
