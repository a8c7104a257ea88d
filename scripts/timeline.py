"""Per-step kernel timeline from a rocprofv3 kernel_trace.csv: for the last few search steps
print each kernel's start offset (from the step's first kernel) and duration, and the step
period — shows launch gaps vs kernel time. Usage: python scripts/timeline.py trace.csv [first]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "qprep"
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
starts = [i for i, k in enumerate(ks) if first in k[2]]
for a, b in zip(starts[-4:-1], starts[-3:]):
    t0 = ks[a][0]
    print(f"--- step period {(ks[b][0] - t0) / 1e3:.1f} us")
    for s, e, n in ks[a:b]:
        short = n.split("(")[0].replace("void ragmi::", "").replace("ragmi::", "")[:50]
        print(f"  +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:8.1f} us  {short}")
