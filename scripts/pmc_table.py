"""Merge one rocprofv3 --pmc FETCH_SIZE pass into profiles/scan_pmc.json (bench.py's
`traffic` table), keyed by the scan kind and the rows one launch scans.

usage: python scripts/pmc_table.py KIND ROWS PMC_DIR KERNEL_SUBSTR TAG [ALGO_BYTES]
  KIND: scan_384 (the headline scan_kernel; stored under by_rows_per_gpu), wide_1024
        (config 5's scan_wide_kernel), filtered_384 (the tag-filtered scan_kernel)
Per launch: FETCH_SIZE (kB) x 1024 x 2 (gfx950 reports half the bytes of 16 B/lane streaming
reads, MI355X_MICROARCH.md §HBM), averaged over the pass's launches of KERNEL_SUBSTR. The raw
counter file is copied to profiles/<TAG>_pmc_fetch_size.csv (via PROFILES_DIR on the box)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    kind, rows, pmc_dir, ksub, tag = sys.argv[1:6]
    algo = int(sys.argv[6]) if len(sys.argv) > 6 else None
    out = os.environ.get("PROFILES_DIR", os.path.join(ROOT, "profiles"))
    os.makedirs(out, exist_ok=True)
    hits = glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True)
    if not hits:
        sys.exit(f"no counter_collection.csv under {pmc_dir}")
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(hits[0]))
            if ksub in r.get("Kernel_Name", "") and "rescan" not in r.get("Kernel_Name", "")
            and r.get("Counter_Name") == "FETCH_SIZE"]
    if not vals:
        sys.exit(f"no FETCH_SIZE rows for {ksub}")
    open(os.path.join(out, f"{tag}_pmc_fetch_size.csv"), "w").write(open(hits[0]).read())
    kb = sum(vals) / len(vals)
    entry = {"hbm_bytes_per_launch": kb * 1024 * 2, "fetch_size_kB_raw": kb,
             "launches": len(vals), "kernel": ksub,
             "source": f"profiles/{tag}_pmc_fetch_size.csv",
             "commit": os.environ.get("COMMIT", "")}
    if algo:
        entry["algorithmic_bytes"] = algo
        entry["ratio"] = round(kb * 2048 / algo, 4)
    path = os.path.join(out, "scan_pmc.json")
    base = os.path.join(ROOT, "profiles", "scan_pmc.json")
    table = json.load(open(path if os.path.exists(path) else base))
    key = "by_rows_per_gpu" if kind == "scan_384" else f"by_rows_{kind}"
    table.setdefault(key, {})[str(int(rows))] = entry
    json.dump(table, open(path, "w"), indent=1)
    print(json.dumps({kind: {rows: entry}}))


if __name__ == "__main__":
    main()
