"""CPU tests of the drop-in host logic: the reference's TESTING stubs (main.py:146-147, 212,
216, 242-243), payload-filter compilation, point ids, ingest point construction. No GPU."""
import hashlib
import importlib
import os
import uuid

import numpy as np
import pytest


@pytest.fixture()
def rag_testing(monkeypatch):
    monkeypatch.setenv("TESTING", "True")
    import ragmi.rag as rag
    rag = importlib.reload(rag)
    for f in (rag.get_embedder, rag.get_reranker, rag.get_qdrant):
        f.cache_clear()
    return rag


def test_testing_stubs_match_reference(rag_testing):
    rag = rag_testing
    assert rag.embed_query("What was Apple's revenue?") == [0.0] * 384
    assert rag.embed(["a", "b"]) == {"embeddings": [[0.0] * 384, [0.0] * 384]}
    assert rag.retrieve_from_qdrant([0.0] * 384, "aapl").points == []
    idx, sc = rag.rerank_documents("q", ["x", "y", "z"], 2)
    assert list(idx) == [0, 1] and np.array_equal(sc, np.zeros(3))
    idx, sc = rag.rerank_documents("q", [], 5)
    assert list(idx) == [] and len(sc) == 0
    assert rag.get_embedder() is None and rag.get_reranker() is None and rag.get_qdrant() is None
    assert rag.embed_query_batch(["a", "b"]) == [[0.0] * 384] * 2
    assert [r.points for r in rag.retrieve_batch([[0.0] * 384] * 2, ["A", "B"])] == [[], []]


def test_payload_tag_filters():
    from ragmi import qdrant_models as m
    from ragmi.qdrant import PayloadTags, UnsupportedFilter
    t = PayloadTags()
    a = t.tag({"ticker": "AAPL", "document_type": "10-K", "text": "x"})
    b = t.tag({"ticker": "MSFT", "document_type": "10-Q"})
    c = t.tag({"ticker": "AAPL"})
    assert a != b and (a & 0xFFFF) == (c & 0xFFFF) and (c >> 16) == 0
    f = lambda *conds: m.Filter(must=[m.FieldCondition(key=k, match=m.MatchValue(value=v))
                                      for k, v in conds])
    mask, val = t.compile(f(("ticker", "AAPL")))
    assert (a & mask) == val and (c & mask) == val and (b & mask) != val
    mask, val = t.compile(f(("ticker", "AAPL"), ("document_type", "10-K")))
    assert (a & mask) == val and (c & mask) != val
    assert t.compile(f(("ticker", "TSLA"))) is None            # never ingested: empty result
    assert t.compile(f(("ticker", "AAPL"), ("ticker", "MSFT"))) is None
    assert t.compile(None) == (0, 0)
    with pytest.raises(UnsupportedFilter):
        t.compile(m.Filter(should=[m.FieldCondition(key="ticker", match=m.MatchValue("A"))]))
    with pytest.raises(UnsupportedFilter):
        t.compile(f(("source_file", "x.html")))


def test_point_ids_like_qdrant():
    from ragmi.qdrant import _norm_id
    h = hashlib.md5(b"AAPL_10-K_primary_document.html_chunk").hexdigest()
    assert _norm_id(h) == str(uuid.UUID(h)) and "-" in _norm_id(h)
    assert _norm_id(str(uuid.UUID(h))) == _norm_id(h)
    assert _norm_id(7) == 7
    with pytest.raises(ValueError):
        _norm_id(-1)


def test_chunk_points_follow_ingest(rag_testing):
    rag = rag_testing
    pts = rag.chunk_points("aapl", "10-k", "primary_document.html", ["c1", "c2"],
                           [[0.1] * 384, [0.2] * 384], ingested_at="T")
    assert pts[0].id == hashlib.md5(b"aapl_10-k_primary_document.html_c1").hexdigest()
    assert pts[0].payload == {"ticker": "AAPL", "document_type": "10-K", "text": "c1",
                              "source_file": "primary_document.html", "ingested_at": "T"}
    again = rag.chunk_points("aapl", "10-k", "primary_document.html", ["c1"], [[0.1] * 384])
    assert again[0].id == pts[0].id                              # idempotent re-ingest


def test_reference_model_constructors():
    from ragmi import qdrant_models as m
    vp = m.VectorParams(size=384, distance=m.Distance.COSINE)
    assert vp.size == 384 and vp.distance == m.Distance.COSINE
    p = m.PointStruct(id="x", vector=[0.0], payload={"ticker": "A"})
    assert p.payload["ticker"] == "A"
    fc = m.FieldCondition(key="ticker", match=m.MatchValue(value="AAPL"))
    assert m.Filter(must=[fc]).must[0].match.value == "AAPL"


def test_retrieve_swallows_like_the_reference(monkeypatch):
    """retrieve_from_qdrant keeps the reference's swallow-to-empty (main.py:232-239): every
    query error gives empty points. Nothing is refused for its size any more — query_points
    answers any limit exactly (k > RAG_MAX_K_LARGE on the full exact pass, round 6)."""
    monkeypatch.setenv("TESTING", "False")
    import ragmi.rag as rag
    rag = importlib.reload(rag)
    import ragmi.qdrant as qd
    assert not hasattr(qd, "LimitTooLarge")

    class Fake:
        def __init__(self, exc):
            self.exc = exc

        def query_points(self, **kw):
            raise self.exc

    monkeypatch.setattr(rag, "get_qdrant", lambda: Fake(RuntimeError("down")))
    assert rag.retrieve_from_qdrant([0.0] * 384, "aapl", limit=5000).points == []


class _StubIndex:
    """FlatIndex stand-in for Collection.search's host logic: the first search leaves query 1
    unanswered (ids -1, unanswered() + 1) as a large-k pass does past 16384 near-ties; the full
    pass answers it."""

    def __init__(self, count, k_full_ids):
        self.count = count
        self.n_un = 0
        self.calls = []
        self.k_full_ids = k_full_ids

    def search(self, q, k, filters=None, full=False):
        import torch
        B = len(q)
        self.calls.append((B, k, full))
        if full:
            ids = torch.tensor([self.k_full_ids[:k]] * B, dtype=torch.int64)
            return torch.full((B, k), 0.5), ids
        ids = torch.arange(k, dtype=torch.int64).repeat(B, 1)
        s = torch.full((B, k), 0.9)
        ids[1] = -1
        s[1] = float("-inf")
        self.n_un += 1
        return s, ids

    def unanswered(self):
        return self.n_un


def test_collection_reanswers_unanswered_queries_on_the_full_pass():
    import numpy as np
    import threading
    from ragmi.qdrant import Collection, PayloadTags
    col = Collection.__new__(Collection)
    col.index = _StubIndex(count=100, k_full_ids=list(range(50, 100)))
    col.lock = threading.RLock()
    col._unanswered = 0
    col.rescued = 0
    col.tags = PayloadTags()
    out = col.search(np.zeros((3, 384), np.float32), 40, [(0, 0)] * 3)
    assert col.index.calls == [(3, 40, False), (1, 40, True)]
    assert [r for r, _ in out[1]] == list(range(50, 90))      # answered, not "no documents"
    assert [r for r, _ in out[0]] == list(range(40))
    assert col.rescued == 1 and col._unanswered == 1
    # padding -1 (fewer matching points than k) with no unanswered query: no second pass
    col.index.n_un = 0
    col._unanswered = 0
    col.index.search = lambda q, k, filters=None, full=False: (
        __import__("torch").tensor([[0.9, float("-inf")]]),
        __import__("torch").tensor([[3, -1]]))
    col.index.unanswered = lambda: 0
    assert col.search(np.zeros((1, 384), np.float32), 2, [(0, 0)]) == [[(3, 0.8999999761581421)]]


def test_limit_range_constants():
    from ragmi import index
    assert index.MAX_K == 32 and index.MAX_K_LARGE == 4096
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "include",
                            "ragmi.h")).read()
    assert "#define RAG_MAX_K 32" in hdr and "#define RAG_MAX_K_LARGE 4096" in hdr


def test_rerank_batch_is_one_forward(monkeypatch):
    """rerank_batch packs every (query, chunk) pair of a micro-batch into ONE predict call
    (batch_size = all pairs), then splits per request like rerank_documents."""
    monkeypatch.setenv("TESTING", "False")
    import ragmi.rag as rag
    rag = importlib.reload(rag)
    calls = []

    class FakeCE:
        def predict(self, pairs, batch_size=32):
            calls.append((len(pairs), batch_size))
            return np.arange(len(pairs), dtype=np.float32)[::-1].copy()

    monkeypatch.setattr(rag, "get_reranker", lambda: FakeCE())
    qs = [f"q{i}" for i in range(32)]
    texts = [[f"t{i}_{j}" for j in range(15)] for i in range(32)]
    out = rag.rerank_batch(qs, texts, 5)
    assert calls == [(480, 480)]
    assert len(out) == 32 and list(out[0][0]) == [0, 1, 2, 3, 4]
