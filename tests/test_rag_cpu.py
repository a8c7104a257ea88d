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


def test_limit_too_large_fails_loudly(monkeypatch):
    """A limit the build cannot answer (> RAG_MAX_K_LARGE over a larger collection) passes the
    reference's swallow-to-empty wrapper (main.py:238-239) as LimitTooLarge: it must not read
    as 'no documents'. Any other query error still gives empty points, as in the reference."""
    monkeypatch.setenv("TESTING", "False")
    import ragmi.rag as rag
    rag = importlib.reload(rag)
    from ragmi.qdrant import LimitTooLarge

    class Fake:
        def __init__(self, exc):
            self.exc = exc

        def query_points(self, **kw):
            raise self.exc

    monkeypatch.setattr(rag, "get_qdrant", lambda: Fake(LimitTooLarge("limit 5000")))
    with pytest.raises(LimitTooLarge):
        rag.retrieve_from_qdrant([0.0] * 384, "aapl", limit=5000)
    monkeypatch.setattr(rag, "get_qdrant", lambda: Fake(RuntimeError("down")))
    assert rag.retrieve_from_qdrant([0.0] * 384, "aapl", limit=5000).points == []


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
