"""GPU test of query coalescing through the QdrantClient drop-in: 32 threads each calling
query_points with their own ticker filter and limit (main2.py's per-request search from
to_thread workers, main2.py:218,228) get ids, scores and payloads identical to the same
calls made one at a time, while sharing a handful of GPU scans."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_32_threads_query_points_bit_equal(gpu):
    from ragmi import qdrant_models as m
    from ragmi.qdrant import QdrantClient
    rng = np.random.default_rng(5)
    n, d = 50_000, 384
    x = rng.standard_normal((n, d)).astype(np.float32)
    tick = ["AAPL", "MSFT", "NVDA", "AMZN"]
    cl = QdrantClient(url="http://unused", device=gpu)
    cl.create_collection("c", m.VectorParams(size=d, distance=m.Distance.COSINE),
                         capacity=n)
    cl.upsert("c", m.Batch(ids=list(range(n)), vectors=x,
                           payloads=[{"ticker": tick[i % 4], "text": f"chunk {i}"}
                                     for i in range(n)]))
    qs = x[rng.choice(n, 32)] + 0.05 * rng.standard_normal((32, d)).astype(np.float32)
    flt = [None if j % 5 == 0 else m.Filter(must=[m.FieldCondition(
        key="ticker", match=m.MatchValue(value=tick[j % 4]))]) for j in range(32)]
    lim = [15 if j % 2 else 7 for j in range(32)]
    want = [cl.query_points("c", query=qs[j], limit=lim[j], query_filter=flt[j]).points
            for j in range(32)]
    col = cl._col("c")
    b0 = col.coalescer.batches
    got = [None] * 32
    bar = threading.Barrier(32)

    def worker(j):
        bar.wait()
        got[j] = cl.query_points("c", query=qs[j], limit=lim[j], query_filter=flt[j]).points

    th = [threading.Thread(target=worker, args=(j,)) for j in range(32)]
    [t.start() for t in th]
    [t.join() for t in th]
    for j in range(32):
        assert [(p.id, p.score, p.payload) for p in got[j]] == \
               [(p.id, p.score, p.payload) for p in want[j]]
    scans = col.coalescer.batches - b0
    print(f"32 concurrent query_points -> {scans} GPU scans")
    assert scans < 32
    cl.close()
