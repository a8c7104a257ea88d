"""Summarise rocprofv3 CSV output into profiles/<tag>_*.{csv,json}.

kernel trace -> per-kernel count / total / avg / min / max duration (us);
PMC FETCH_SIZE (kB, per dispatch) -> HBM read bytes per scan launch, corrected x2 for
gfx950 wide streaming reads (MI355X_MICROARCH.md §HBM: FETCH_SIZE reports exactly half the
bytes of 16 B/lane streaming loads). Writes profiles/scan_pmc.json for bench.py.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(d, pat):
    hits = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return hits[0] if hits else None


def main():
    tag, trace_dir, pmc_dir = sys.argv[1], sys.argv[2], sys.argv[3]
    bench_log = sys.argv[4] if len(sys.argv) > 4 else None
    out = os.environ.get("PROFILES_DIR", os.path.join(ROOT, "profiles"))
    os.makedirs(out, exist_ok=True)
    stats = find(trace_dir, "*kernel_stats.csv")
    summary = {}
    if stats:
        rows = list(csv.DictReader(open(stats)))
        with open(os.path.join(out, f"{tag}_kernel_stats.csv"), "w") as f:
            f.write(open(stats).read())
        for r in rows:
            summary[r["Name"][:120]] = {k: r[k] for k in r if k != "Name"}
    trace = find(trace_dir, "*kernel_trace.csv")
    scan_durs = []
    if trace:
        for r in csv.DictReader(open(trace)):
            if "scan_kernel" in r["Kernel_Name"] and "rescan" not in r["Kernel_Name"]:
                scan_durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = find(pmc_dir, "*counter_collection.csv")
    fetch = []
    if pmc:
        for r in csv.DictReader(open(pmc)):
            if ("scan_kernel" in r.get("Kernel_Name", "") and "rescan" not in r.get("Kernel_Name", "")
                    and r.get("Counter_Name") == "FETCH_SIZE"):
                fetch.append(float(r["Counter_Value"]))
        with open(os.path.join(out, f"{tag}_pmc_fetch_size.csv"), "w") as f:
            f.write(open(pmc).read())
    res = {"tag": tag, "scan_launches": len(scan_durs),
           "scan_avg_us": sum(scan_durs) / len(scan_durs) if scan_durs else None,
           "scan_min_us": min(scan_durs) if scan_durs else None}
    if fetch:
        kb = sum(fetch) / len(fetch)
        res.update({"fetch_size_kB_per_launch_raw": kb,
                    "hbm_bytes_per_launch": kb * 1024 * 2,
                    "note": "FETCH_SIZE (kB) x 1024 x 2: gfx950 reports half the bytes of "
                            "16 B/lane streaming reads (MI355X_MICROARCH.md §HBM)"})
        # headline entry updated in place: the by-rows / by-kind tables of earlier passes
        # (scripts/pmc_table.py) are kept
        path = os.path.join(out, "scan_pmc.json")
        base = os.path.join(ROOT, "profiles", "scan_pmc.json")
        table = {}
        for src in (path, base):
            if os.path.exists(src):
                table = json.load(open(src))
                break
        table.update({"hbm_bytes_per_launch": kb * 1024 * 2,
                      "source": f"profiles/{tag}_pmc_fetch_size.csv",
                      "fetch_size_kB_raw": kb, "commit": os.environ.get("COMMIT", "")})
        json.dump(table, open(path, "w"), indent=1)
    if bench_log and os.path.exists(bench_log):
        lines = [l for l in open(bench_log) if l.startswith("{")]
        if lines:
            res["bench"] = json.loads(lines[-1])
            open(os.path.join(out, f"{tag}_bench.json"), "w").write(lines[-1])
    json.dump(res, open(os.path.join(out, f"{tag}_summary.json"), "w"), indent=1)
    print(json.dumps(res)[:2000])


if __name__ == "__main__":
    main()
