"""Per-stage kernel breakdown from a rocprofv3 kernel trace of scripts/bench_stages.py:
kernels are attributed to stages by their order (each stage's launches are contiguous)."""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/st_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# segments separated by >2 ms of idle (host work between stages)
segs, cur, last = [], [], None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if last is not None and s - last > 2_000_000 and cur:
        segs.append(cur)
        cur = []
    cur.append(r)
    last = e
segs.append(cur)
for i, seg in enumerate(segs):
    tot = collections.Counter()
    n = collections.Counter()
    for r in seg:
        k = r["Kernel_Name"].split("(")[0][:70]
        tot[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        n[k] += 1
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    busy = sum(tot.values()) / 1e3
    if span < 50:
        continue
    print(f"segment {i}: {len(seg)} kernels, span {span:.1f} us, busy {busy:.1f} us")
    for k, t in tot.most_common(8):
        print(f"   {t / 1e3:9.1f} us  {n[k]:5d}x  {k}")
