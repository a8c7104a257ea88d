"""A/B the scan kernel variants (rag_bench_scan) on the 10M x 384 bench corpus, interleaved
rounds in one process (cdna_hip_programming.md §5.4 rule 24). Prints one JSON line per
variant: median / min device ms per launch and the algorithmic HBM rate."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

import bench  # noqa: E402
from ragmi.index import FlatIndex  # noqa: E402

NAMES = {0: "prod (seeded, interleaved, nt, sched-barrier)", 1: "unseeded", 2: "contiguous",
         3: "mfma-only", 4: "loads-only", 5: "no-nt", 6: "no-sb", 7: "top-k never taken",
         8: "VALU v_dot2_f32_f16 (no MFMA), same loads and top-k",
         9: "dynamic tile queue, chunks of 2 (timed per launch)",
         10: "dynamic tile queue, chunks of 1 (timed per launch)",
         11: "dynamic tile queue, chunks of 4 (timed per launch)",
         12: "dynamic (2), loads only (timed per launch)",
         13: "static prod (timed per launch)", 14: "static loads only (timed per launch)",
         15: "prod without the end-of-scan pending sort (probe)",
         16: "prod with the round-1 pending sort (32 lanes x 2 queries)"}


def main():
    rows = int(os.environ.get("ROWS", "10000000"))
    variants = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,3,4,5,6").split(",")]
    rounds = int(os.environ.get("ROUNDS", "5"))
    dev = torch.device("cuda", 0)
    idx = FlatIndex(bench.D, rows, dev, diagnostic=True)
    bench.build_shard(idx, 0, rows, rows, dev)
    qs, _ = bench.make_queries(1, rows, dev)
    res = {v: [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            res[v].append(idx.bench_scan(qs[0], v, reps=5))
    for v in variants:
        ms = np.array(res[v])
        gbs = rows * bench.D * 2 / (np.median(ms) * 1e-3) / 1e9
        print(json.dumps({"variant": v, "name": NAMES[v], "median_ms": round(float(np.median(ms)), 4),
                          "min_ms": round(float(ms.min()), 4), "GB/s": round(gbs, 1),
                          "frac_8TBs": round(gbs / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
