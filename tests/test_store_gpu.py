"""GPU round trip of persistence: FlatIndex -> shard directory -> new
FlatIndex through rag_index_import_rows returns bit-identical stored rows and bit-identical
search results (scores and ids, with and without payload filters); QdrantClient(path=...)
reloads collections with ids, payloads and versions."""
import numpy as np
import pytest
import torch

import oracle_scan as O

pytestmark = pytest.mark.gpu


def test_index_save_load_bit_identical(gpu, tmp_path):
    from ragmi import store
    from ragmi.index import FlatIndex
    rng = np.random.default_rng(5)
    n, d = 7001, 384
    x = rng.standard_normal((n, d)).astype(np.float32)
    tags = rng.integers(0, 4, n).astype(np.uint32)
    a = FlatIndex(dim=d, capacity=n, device=gpu)
    a.upsert(x, np.arange(n), tags)
    store.save_index(a, str(tmp_path / "s"), chunk_rows=3000)
    b = store.load_index(str(tmp_path / "s"), device=gpu)
    assert b.count == n
    np.testing.assert_array_equal(b.export_rows(), a.export_rows())
    np.testing.assert_array_equal(b.export_tags(), tags)
    np.testing.assert_array_equal(a.export_rows(), O.encode_rows(x))
    q = rng.standard_normal((32, d)).astype(np.float32)
    filt = np.stack([np.full(32, 0xFFFFFFFF, np.uint32), rng.integers(0, 4, 32).astype(np.uint32)],
                    1)
    for f in (None, filt):
        sa, ia = a.search(q, 15, filters=f)
        sb, ib = b.search(q, 15, filters=f)
        torch.testing.assert_close(sb, sa, rtol=0, atol=0)
        assert torch.equal(ib, ia)
    # a loaded index keeps accepting writes after the imported rows
    b.reserve(n + 10)
    b.upsert(x[:10], np.arange(n, n + 10))
    assert b.count == n + 10
    np.testing.assert_array_equal(b.export_rows(n, 10), a.export_rows(0, 10))
    # partial range import at an offset
    c = FlatIndex(dim=d, capacity=64, device=gpu)
    store.load_into(c, str(tmp_path / "s"), row0=5, rows=(100, 1100))
    assert c.count == 1005
    np.testing.assert_array_equal(c.export_rows(5, 1000), a.export_rows(100, 1000))
    for idx in (a, b, c):
        idx.close()


def test_qdrant_client_path_persistence(gpu, tmp_path):
    from ragmi import qdrant_models as m
    from ragmi.qdrant import QdrantClient
    rng = np.random.default_rng(6)
    path = str(tmp_path / "storage")
    c1 = QdrantClient(url="http://qdrant:6333", device=gpu, path=path)
    c1.create_collection("financial_documents", m.VectorParams(size=384,
                                                              distance=m.Distance.COSINE))
    c1.create_collection("scratch", m.VectorParams(size=384, distance=m.Distance.COSINE))
    pts = [m.PointStruct(id=f"{i:032x}" if i % 2 else i, vector=rng.standard_normal(384).tolist(),
                         payload={"ticker": ["AAPL", "MSFT"][i % 2],
                                  "document_type": ["10-K", "10-Q", "8-K"][i % 3],
                                  "text": f"chunk {i}"}) for i in range(500)]
    c1.upsert("financial_documents", pts)
    c1.upsert("financial_documents", pts[:7])                  # versions move
    q = rng.standard_normal(384).astype(np.float32)
    flt = m.Filter(must=[m.FieldCondition(key="ticker", match=m.MatchValue(value="MSFT"))])
    before = c1.query_points("financial_documents", q, limit=15, query_filter=flt).points
    c1.delete_collection("scratch")
    c1.close()                                                 # persists
    c2 = QdrantClient(device=gpu, path=path)
    assert [c.name for c in c2.get_collections().collections] == ["financial_documents"]
    assert c2.count("financial_documents").count == 500
    after = c2.query_points("financial_documents", q, limit=15, query_filter=flt).points
    assert [(p.id, p.score, p.payload, p.version) for p in after] == \
        [(p.id, p.score, p.payload, p.version) for p in before]
    rec = c2.retrieve("financial_documents", [pts[3].id, 4])
    assert [r.payload["text"] for r in rec] == ["chunk 3", "chunk 4"]
    # upserts after reload keep the id map and codebooks
    c2.upsert("financial_documents", [m.PointStruct(id=4, vector=pts[4].vector,
                                                    payload={"ticker": "TSLA"})])
    assert c2.count("financial_documents").count == 500
    t = m.Filter(must=[m.FieldCondition(key="ticker", match=m.MatchValue(value="TSLA"))])
    got = c2.query_points("financial_documents", q, limit=5, query_filter=t).points
    assert [p.id for p in got] == [4]
    c2.close()
