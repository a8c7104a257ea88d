"""The unchanged main2.py serving pattern on the drop-in QdrantClient: T threads, each
issuing per-request query_points(limit=15, ticker filter) calls back to back (main2.py's
process_independently -> retrieve_from_qdrant from asyncio.to_thread workers, <= 25 at once,
main2.py:52-53,218,228), with and without query coalescing; plus query_batch_points (the
rewritten batch_processor's one call per micro-batch) for reference. 1M x 384 collection,
16 tickers. One JSON line per mode: requests/s, GPU scans issued, requests per scan."""
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

from ragmi import qdrant_models as m  # noqa: E402
from ragmi.qdrant import QdrantClient  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, d = int(os.environ.get("ROWS", "1000000")), 384
    T, R = int(os.environ.get("THREADS", "25")), int(os.environ.get("REQS", "40"))
    ticks = [f"T{i:02d}" for i in range(16)]
    cl = QdrantClient(url="http://unused", device=dev)
    cl.create_collection("c", m.VectorParams(size=d, distance=m.Distance.COSINE), capacity=n)
    g = torch.Generator(device=dev)
    g.manual_seed(1000)
    x = torch.randn((n, d), generator=g, device=dev)
    cl.upsert("c", m.Batch(ids=list(range(n)), vectors=x,
                           payloads=[{"ticker": ticks[i % 16]} for i in range(n)]))
    col = cl._col("c")
    rng = np.random.default_rng(3)
    qs = rng.standard_normal((T * R, d)).astype(np.float32)
    fl = [m.Filter(must=[m.FieldCondition(key="ticker", match=m.MatchValue(value=ticks[j % 16]))])
          for j in range(T * R)]
    for j in range(4):                                    # warm
        cl.query_points("c", query=qs[j], limit=15, query_filter=fl[j])
    for mode in ("per-request", "coalesced"):
        cl.coalesce = mode == "coalesced"
        b0 = col.coalescer.batches
        bar = threading.Barrier(T + 1)

        def worker(t):
            bar.wait()
            for r in range(R):
                j = t * R + r
                cl.query_points("c", query=qs[j], limit=15, query_filter=fl[j])

        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        [t.start() for t in th]
        bar.wait()
        t0 = time.perf_counter()
        [t.join() for t in th]
        el = time.perf_counter() - t0
        scans = (col.coalescer.batches - b0) if mode == "coalesced" else T * R
        print(json.dumps({"pattern": "main2.py per-request query_points", "mode": mode,
                          "rows": n, "threads": T, "requests": T * R,
                          "requests_per_s": round(T * R / el, 1), "gpu_scans": scans,
                          "requests_per_scan": round(T * R / max(scans, 1), 2)}), flush=True)
    reqs = [m.QueryRequest(query=qs[j], filter=fl[j], limit=15) for j in range(32)]
    cl.query_batch_points("c", reqs)
    t0 = time.perf_counter()
    for _ in range(R):
        cl.query_batch_points("c", reqs)
    el = time.perf_counter() - t0
    print(json.dumps({"pattern": "query_batch_points (32 per call)", "rows": n,
                      "requests_per_s": round(32 * R / el, 1)}), flush=True)
    cl.close()


if __name__ == "__main__":
    main()
