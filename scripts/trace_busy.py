"""GPU occupancy of a rocprofv3 kernel trace: the union of ALL kernel dispatch intervals over
the traced span (the middle of the trace: the first and last `skip` fractions of the dispatches
dropped as build / warm-up / checks), the largest idle gaps, and per-kernel totals. Usage: python scripts/trace_busy.py <trace_dir> [skip]"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(f)))
    rows = rows[int(len(rows) * skip):int(len(rows) * (1 - skip))]
    busy, gaps, cb, c0 = 0, [], None, rows[0][0]
    tot = collections.Counter()
    for a, b, name in rows:
        tot[name.split("(")[0][:60]] += b - a
        if cb is None or a > cb:
            if cb is not None:
                gaps.append(a - cb)
            busy += b - a
            cb = b
        elif b > cb:
            busy += b - cb
            cb = b
    span = cb - c0
    gaps.sort(reverse=True)
    print(json.dumps({"trace": d, "kernels": len(rows), "span_ms": round(span / 1e6, 3),
                      "busy_ms": round(busy / 1e6, 3), "busy_frac": round(busy / span, 4),
                      "idle_gaps": len(gaps), "gap_us_top5": [round(g / 1e3, 1) for g in gaps[:5]],
                      "gap_us_total": round(sum(gaps) / 1e3, 1),
                      "top_kernels_ms": {k: round(v / 1e6, 3) for k, v in tot.most_common(8)}}))


if __name__ == "__main__":
    main()
