"""Time of one search pass (32 planted queries, bench.py's corpus) at k = 15 (register top-k)
and at k > 32 (the large-k pass: bound sample, candidate collection, exact rescoring and
select), on the same index. One JSON line per k: device ms per pass (HIP events over 20
back-to-back passes) and the HBM rate of the corpus bytes one pass reads.
Usage (GPU box): python scripts/diag/large_k_timing.py [rows] > gpurun_out/large_k.jsonl"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

import bench  # noqa: E402
from ragmi.index import FlatIndex  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    dev = torch.device("cuda", 0)
    idx = FlatIndex(bench.D, n, dev)
    bench.build_shard(idx, 0, n, n, dev)
    qs, _ = bench.make_queries(2, n, dev)
    for k in (15, 33, 100, 1000):
        for q in qs:                      # warm (workspace allocation on first large-k call)
            idx.search(q, k)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for r in range(20):
            idx.search(qs[r % 2], k)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 20
        print(json.dumps({"rows": n, "batch": bench.B, "k": k, "ms_per_pass": round(ms, 4),
                          "qps": round(bench.B / ms * 1e3, 1),
                          "corpus_GBps": round(n * bench.D * 2 / (ms * 1e-3) / 1e9, 1),
                          "unanswered": idx.unanswered()}), flush=True)
    idx.close()


if __name__ == "__main__":
    main()
