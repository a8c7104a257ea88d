"""Scan launches in a rocprofv3 kernel trace: true per-launch durations (dispatch begin/end),
how much consecutive scans overlap, the union of their intervals per launch, and the gaps between them (small-shard scan-order study).
Usage: python scripts/scan_overlap.py <trace_dir> [label]"""
import csv
import glob
import json
import os
import sys

import numpy as np


def main():
    d = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else d
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    # the scan launches only (not rescan_kernel, whose name contains "scan_kernel")
    sc = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                if "scan_kernel" in r["Kernel_Name"] and "rescan" not in r["Kernel_Name"])
    sc = sc[len(sc) // 5:]                              # drop build / warm-up launches
    st = np.array([a for a, _ in sc], dtype=np.float64)
    en = np.array([b for _, b in sc], dtype=np.float64)
    dur = (en - st) / 1e3
    ov = np.maximum(0.0, en[:-1] - st[1:]) / 1e3       # overlap with the next launch (us)
    gap = np.maximum(0.0, st[1:] - en[:-1]) / 1e3
    span = (en[-1] - st[0]) / 1e3
    # union of the launch intervals (overlapping launches counted once): bench.py's
    # busy_ms_per_launch, from the trace's own dispatch timestamps
    busy, cb = 0.0, -np.inf
    for a, b in zip(st, en):
        if a > cb:
            busy += b - a
            cb = b
        elif b > cb:
            busy += b - cb
            cb = b
    print(json.dumps({"label": label, "scan_launches": len(sc),
                      "dur_us_mean": round(float(dur.mean()), 2),
                      "dur_us_median": round(float(np.median(dur)), 2),
                      "overlap_us_mean": round(float(ov.mean()), 2),
                      "gap_us_mean": round(float(gap.mean()), 2),
                      "union_us_per_launch": round(busy / 1e3 / len(sc), 2),
                      "us_per_launch_over_span": round(span / len(sc), 2)}))


if __name__ == "__main__":
    main()
