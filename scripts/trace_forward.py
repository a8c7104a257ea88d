"""One forward's kernel sequence from a rocprofv3 kernel trace: the last `n` dispatches (n =
launches per forward), each kernel's duration and the idle gap before it, plus totals by
kernel name. Usage: python scripts/trace_forward.py <trace_dir> <n> [skip_last]"""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
n = int(sys.argv[2])
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) - n - skip:len(rows) - skip]
t0 = int(rows[0]["Start_Timestamp"])
last = None
tot, cnt, gaps = collections.Counter(), collections.Counter(), 0.0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - last) / 1e3 if last is not None else 0.0
    gaps += max(g, 0)
    k = r["Kernel_Name"].split("(")[0]
    k = k[:90]
    print(f"{(s - t0) / 1e3:9.2f} +{g:6.2f} {(e - s) / 1e3:8.2f} us  grid {r.get('Grid_Size', '?'):>8} "
          f"wg {r.get('Workgroup_Size', '?'):>5} lds {r.get('LDS_Block_Size', r.get('Lds_Size', '?')):>6} "
          f"vgpr {r.get('VGPR_Count', r.get('Arch_VGPR_Count', '?')):>4}  {k}")
    tot[k] += (e - s) / 1e3
    cnt[k] += 1
    last = e
span = (int(rows[-1]["End_Timestamp"]) - t0) / 1e3
print(f"span {span:.1f} us, busy {sum(tot.values()):.1f} us, gaps {gaps:.1f} us")
for k, t in tot.most_common():
    print(f"  {t:8.1f} us {cnt[k]:4d}x  {k}")
