"""Cost of the full exact pass (rag_index_search_full, round 6): device ms per query pass
at k = 5000 / 20000 over 1M and 10M x 384 rows (32 queries), and forced at k = 15 for the
comparison with the scan path. One JSON line per case."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
from ragmi.index import FlatIndex  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    for n in (1_000_000, 10_000_000):
        idx = FlatIndex(384, n, dev)
        for r0 in range(0, n, 1_000_000):
            x = torch.randn((1_000_000, 384), generator=g, device=dev)
            idx.upsert(x, torch.arange(r0, r0 + 1_000_000, device=dev), new_count=r0 + 1_000_000)
        q = torch.randn((32, 384), generator=g, device=dev)
        for k, full in ((15, False), (15, True), (5000, False), (20000, False)):
            idx.search(q, k, full=full)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                idx.search(q, k, full=full)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / 3
            print(json.dumps({"rows": n, "k": k, "path": "full" if full or k > 4096 else "scan",
                              "queries": 32, "ms_per_pass": round(ms, 3),
                              "ms_per_query": round(ms / 32, 4)}), flush=True)
        idx.close()


if __name__ == "__main__":
    main()
