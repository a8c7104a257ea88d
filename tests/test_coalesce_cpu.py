"""CPU tests of the query coalescer (ragmi.qdrant.Coalescer): concurrent single-query
searches — the unchanged main2.py pattern, <= 25 asyncio.to_thread workers each calling
query_points (main2.py:52-53,218,228) — ride shared batched searches; every caller gets
exactly the result of its own individual search; a lone caller is served at once; a
failing batch raises in every rider. The collection here is a host stand-in whose batched
search is an exact numpy top-k with per-query filters (the GPU path: test_coalesce_gpu.py)."""
import threading
import time

import numpy as np
import pytest


class FakeCollection:
    def __init__(self, x, tags, delay=0.002):
        self.x = x / np.linalg.norm(x, axis=1, keepdims=True)
        self.tags, self.delay = tags, delay
        self.calls = []
        self.fail = False

    def search(self, q, limit, filters):
        self.calls.append(len(filters))
        time.sleep(self.delay)                        # a scan's duration: others queue up
        if self.fail:
            raise RuntimeError("device error")
        out = []
        for j, f in enumerate(filters):
            if f is None:
                out.append([])
                continue
            s = self.x @ (q[j] / np.linalg.norm(q[j]))
            s[(self.tags & f[0]) != f[1]] = -np.inf
            o = np.lexsort((np.arange(len(s)), -s))[:limit]
            out.append([(int(r), float(s[r])) for r in o if np.isfinite(s[r])])
        return out


def _paths():
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = os.path.join(root, "financial-rag-system_amd")
    if p not in sys.path:
        sys.path.insert(0, p)


@pytest.mark.parametrize("window", [0.0, 0.003])
def test_concurrent_callers_share_scans_and_match_individual(window):
    _paths()
    from ragmi.qdrant import Coalescer
    rng = np.random.default_rng(0)
    x = rng.standard_normal((3000, 64)).astype(np.float32)
    tags = rng.integers(1, 5, 3000).astype(np.uint32)
    col = FakeCollection(x, tags)
    co = Coalescer(col, window_s=window, max_batch=32)
    qs = rng.standard_normal((40, 64)).astype(np.float32)
    filts = [(0, 0) if j % 3 == 0 else ((0xFFFF, int(1 + j % 4)) if j % 7 else None)
             for j in range(40)]
    limits = [15 if j % 2 else 5 for j in range(40)]
    want = [col.search(qs[j:j + 1], limits[j], [filts[j]])[0] for j in range(40)]
    col.calls.clear()
    got = [None] * 40
    barrier = threading.Barrier(40)

    def worker(j):
        barrier.wait()
        got[j] = co.search(qs[j], limits[j], filts[j])

    th = [threading.Thread(target=worker, args=(j,)) for j in range(40)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert got == want
    assert co.batches == len(col.calls) < 40 and sum(col.calls) == 40
    assert max(col.calls) <= 32


def test_lone_caller_is_not_delayed():
    _paths()
    from ragmi.qdrant import Coalescer
    rng = np.random.default_rng(1)
    col = FakeCollection(rng.standard_normal((500, 32)).astype(np.float32),
                         np.ones(500, np.uint32), delay=0.0)
    co = Coalescer(col)
    t0 = time.perf_counter()
    for _ in range(50):
        co.search(rng.standard_normal(32).astype(np.float32), 5, (0, 0))
    assert time.perf_counter() - t0 < 0.5 and co.batches == 50


def test_failure_reaches_every_rider():
    _paths()
    from ragmi.qdrant import Coalescer
    rng = np.random.default_rng(2)
    col = FakeCollection(rng.standard_normal((500, 32)).astype(np.float32),
                         np.ones(500, np.uint32))
    col.fail = True
    co = Coalescer(col)
    errs = []

    def worker():
        try:
            co.search(rng.standard_normal(32).astype(np.float32), 5, (0, 0))
        except RuntimeError as e:
            errs.append(str(e))

    th = [threading.Thread(target=worker) for _ in range(10)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert errs == ["device error"] * 10
    assert not co.leader_active and not co.pending


def test_base_exception_in_leader_does_not_strand_riders():
    """A BaseException (KeyboardInterrupt here) raised by the leader's search must still hand
    leadership on: riders of that batch see it, later callers are served normally."""
    _paths()
    from ragmi.qdrant import Coalescer
    rng = np.random.default_rng(3)
    col = FakeCollection(rng.standard_normal((500, 32)).astype(np.float32),
                         np.ones(500, np.uint32), delay=0.01)
    orig = col.search
    state = {"n": 0}

    def search(q, limit, filters):
        state["n"] += 1
        if state["n"] == 1:
            time.sleep(0.01)
            raise KeyboardInterrupt
        return orig(q, limit, filters)
    col.search = search
    co = Coalescer(col)
    out = {}

    def worker(j):
        try:
            out[j] = co.search(rng.standard_normal(32).astype(np.float32), 5, (0, 0))
        except KeyboardInterrupt:
            out[j] = "interrupted"

    th = [threading.Thread(target=worker, args=(j,)) for j in range(8)]
    for t in th:
        t.start()
        time.sleep(0.001)
    for t in th:
        t.join(timeout=10)
    assert not any(t.is_alive() for t in th), "a rider was stranded"
    assert "interrupted" in out.values() and len(out) == 8
    # the collection still serves
    assert len(co.search(rng.standard_normal(32).astype(np.float32), 5, (0, 0))) == 5
    assert not co.leader_active and not co.pending
