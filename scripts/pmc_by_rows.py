"""Record the HBM bytes of one scan launch over a shard of R rows from a rocprofv3 --pmc
FETCH_SIZE pass (x2: gfx950 reports half the bytes of 16 B/lane streaming reads,
MI355X_MICROARCH.md §HBM) into profiles/scan_pmc.json's by_rows_per_gpu table, which
bench.py reads for the `traffic` of a rank whose shard has R rows.

Usage (GPU box): python scripts/pmc_by_rows.py <pmc_dir> <rows> <tag>
Writes gpurun_out/profiles/<tag>_pmc_fetch_size.csv and gpurun_out/profiles/scan_pmc.json.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    pmc_dir, rows, tag = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    out = os.environ.get("PROFILES_DIR", os.path.join(ROOT, "gpurun_out", "profiles"))
    os.makedirs(out, exist_ok=True)
    f = glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True)[0]
    kb = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
          if "scan_kernel" in r.get("Kernel_Name", "") and r.get("Counter_Name") == "FETCH_SIZE"]
    shutil.copy(f, os.path.join(out, f"{tag}_pmc_fetch_size.csv"))
    cur = os.path.join(out, "scan_pmc.json")
    src = cur if os.path.exists(cur) else os.path.join(ROOT, "profiles", "scan_pmc.json")
    p = json.load(open(src)) if os.path.exists(src) else {}
    avg = sum(kb) / len(kb)
    p.setdefault("by_rows_per_gpu", {})[str(rows)] = {
        "hbm_bytes_per_launch": avg * 1024 * 2, "fetch_size_kB_raw": avg, "launches": len(kb),
        "algorithmic_bytes": rows * 768, "source": f"profiles/{tag}_pmc_fetch_size.csv",
        "commit": os.environ.get("COMMIT", "")}
    json.dump(p, open(cur, "w"), indent=1)
    print(rows, "rows:", len(kb), "launches,", round(avg * 2048 / (rows * 768), 4), "x algorithmic")


if __name__ == "__main__":
    main()
