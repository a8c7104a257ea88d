"""GPU parity of fp32 storage (RAG_STORE_FP32 — Qdrant's default Float32 vectors, which the
reference gets by setting no `datatype`: database.py:124-130, ingest.py:89-95).

The index keeps the normalised fp32 rows beside the fp16 copy the scan streams; exact scores
read the fp32 rows. Bar: stored fp32 and fp16 rows bit-exact vs the oracle's encode_rows32 /
encode_rows, and top-k ids AND scores bit-exact vs the oracle's search over the fp32 rows —
on random and planted queries, D = 384 / 1024, k = 15 / 32, per-query payload filters,
near-ties below fp16 resolution (ranked by their fp32 values, where fp16 storage ties them),
near-duplicate clusters that need the exactness fallbacks, persistence round trips, and the
QdrantClient default.
"""
import numpy as np
import pytest
import torch

import oracle_scan as O

pytestmark = pytest.mark.gpu


def _index(gpu, x, tags=None, storage="fp32"):
    from ragmi.index import FlatIndex
    idx = FlatIndex(dim=x.shape[1], capacity=max(x.shape[0], 16), device=gpu, storage=storage)
    idx.upsert(x, np.arange(x.shape[0], dtype=np.int64), tags, new_count=x.shape[0])
    return idx


def _search(idx, q, k, filters=None):
    s, i = idx.search(q, k, filters=filters)
    torch.cuda.synchronize()
    return s.cpu().numpy(), i.cpu().numpy()


@pytest.mark.parametrize("dim", [384, 1024])
def test_stored_rows_bit_exact(gpu, dim):
    rng = np.random.default_rng(dim)
    x = rng.standard_normal((777, dim)).astype(np.float32)
    x[5] = 0.0
    idx = _index(gpu, x)
    assert idx.storage == "fp32"
    np.testing.assert_array_equal(idx.export_rows32(), O.encode_rows32(x))
    np.testing.assert_array_equal(idx.export_rows(), O.encode_rows(x))
    idx.close()


@pytest.mark.parametrize("dim,n,b,k", [(384, 5003, 32, 15), (384, 4096, 7, 32), (384, 777, 45, 15),
                                       (1024, 5003, 32, 15), (1024, 4096, 128, 15),
                                       (1024, 3000, 40, 32)])
def test_search_vs_oracle(gpu, dim, n, b, k):
    rng = np.random.default_rng(n + b + dim)
    x = rng.standard_normal((n, dim)).astype(np.float32)
    q = rng.standard_normal((b, dim)).astype(np.float32)
    q[: b // 2] = x[rng.choice(n, b // 2)] + 0.05 * rng.standard_normal((b // 2, dim)).astype(
        np.float32)
    idx = _index(gpu, x)
    s, i = _search(idx, q, k)
    s2, i2 = O.search(O.encode_rows32(x), q, k)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)
    idx.close()


def test_filtered_vs_oracle(gpu):
    rng = np.random.default_rng(8)
    n, b = 6000, 24
    x = rng.standard_normal((n, 384)).astype(np.float32)
    tags = rng.integers(0, 6, n).astype(np.uint32) | (rng.integers(1, 3, n).astype(np.uint32) << 16)
    q = rng.standard_normal((b, 384)).astype(np.float32)
    filt = np.zeros((b, 2), np.uint32)
    filt[:, 0] = np.where(np.arange(b) % 3 == 0, 0xFFFF, 0xFFFFFFFF)
    filt[:, 1] = rng.integers(0, 6, b).astype(np.uint32) | np.where(
        np.arange(b) % 3 == 0, 0, 1 << 16).astype(np.uint32)
    idx = _index(gpu, x, tags)
    s, i = _search(idx, q, 15, filters=filt)
    c32 = O.encode_rows32(x)
    for j in range(b):
        s2, i2 = O.search(c32, q[j:j + 1], 15, tags=tags, mask=int(filt[j, 0]),
                          value=int(filt[j, 1]), use_filter=True)
        np.testing.assert_array_equal(i[j], i2[0])
        np.testing.assert_array_equal(s[j], s2[0])
    idx.close()


@pytest.mark.parametrize("dim", [384, 1024])
def test_sub_fp16_near_ties_ranked_by_fp32(gpu, dim):
    """Rows that differ below fp16 resolution (base + 2e-4 noise): fp32 storage ranks them by
    their fp32 scores exactly as the fp32 oracle; fp16 storage (the oracle over fp16 rows)
    orders them differently — the divergence fp32 storage removes."""
    rng = np.random.default_rng(dim + 1)
    n = 20_000 if dim == 384 else 8_000
    x = rng.standard_normal((n, dim)).astype(np.float32)
    base = x[11].copy()
    rows = np.sort(rng.choice(n, 64, replace=False))
    x[rows] = base + 2e-4 * rng.standard_normal((64, dim)).astype(np.float32)
    q = np.concatenate([base[None] + 1e-3 * rng.standard_normal((6, dim)).astype(np.float32),
                        rng.standard_normal((2, dim)).astype(np.float32)])
    idx = _index(gpu, x)
    for k in (15, 32):
        s, i = _search(idx, q, k)
        s2, i2 = O.search(O.encode_rows32(x), q, k)
        np.testing.assert_array_equal(i, i2)
        np.testing.assert_array_equal(s, s2)
    _, i16 = O.search(O.encode_rows(x), q, 32)
    assert (i16[:6] != i[:6]).any()
    idx.close()


@pytest.mark.parametrize("saturated", [False, True])
def test_near_duplicate_clusters_certified(gpu, saturated):
    """Clusters inside the (larger, fp32-storage) error band: the fallback tiers re-score
    from the fp32 rows and stay bit-exact."""
    rng = np.random.default_rng(40 + saturated)
    n = 200_000 if saturated else 24_000
    base = rng.standard_normal((1, 384)).astype(np.float32)
    x = rng.standard_normal((n, 384)).astype(np.float32)
    rows = np.arange(0, n, 2) if saturated else np.sort(rng.choice(n, 160, replace=False))
    x[rows] = base + 1e-5 * rng.standard_normal((len(rows), 384)).astype(np.float32)
    q = np.concatenate([base + 0.02 * rng.standard_normal((4, 384)).astype(np.float32),
                        rng.standard_normal((2, 384)).astype(np.float32)])
    idx = _index(gpu, x)
    s, i = _search(idx, q, 15)
    _, _, tiers = idx.exactness_stats(6)
    c32 = idx.export_rows32()
    s2, i2 = (O.search_fast if saturated else O.search)(c32, q, 15)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)
    assert (tiers[:4] >= 1).all(), tiers
    idx.close()


def test_million_rows_planted(gpu):
    rng = np.random.default_rng(50)
    n, b = 1_000_000, 32
    x = rng.standard_normal((n, 384)).astype(np.float32)
    src = rng.choice(n, b, replace=False)
    q = x[src] + 0.05 * rng.standard_normal((b, 384)).astype(np.float32)
    idx = _index(gpu, x)
    s, i = _search(idx, q, 15)
    assert (i[:, 0] == src).all()
    s2, i2 = O.search_fast(idx.export_rows32(), q, 15)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)
    idx.close()


def test_persistence_roundtrip(gpu, tmp_path):
    from ragmi import store
    rng = np.random.default_rng(60)
    n = 5000
    x = rng.standard_normal((n, 384)).astype(np.float32)
    tags = rng.integers(0, 4, n).astype(np.uint32)
    q = rng.standard_normal((16, 384)).astype(np.float32)
    idx = _index(gpu, x, tags)
    want = _search(idx, q, 15)
    p = str(tmp_path / "shard32")
    store.save_index(idx, p, chunk_rows=1500)
    idx.close()
    back = store.load_index(p, device=gpu)
    assert back.storage == "fp32"
    np.testing.assert_array_equal(back.export_rows32(), O.encode_rows32(x))
    np.testing.assert_array_equal(back.export_rows(), O.encode_rows(x))
    got = _search(back, q, 15)
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[1], want[1])
    with pytest.raises(Exception, match="fp32-storage"):
        back.import_rows(O.encode_rows(x[:10]), 0)
    back.close()


def test_qdrant_client_default_is_fp32(gpu):
    """VectorParams(size, COSINE) with no datatype (the reference's call) -> fp32 storage;
    datatype float16 -> fp16 storage; both answer query_points with the matching oracle."""
    from ragmi import qdrant_models as models
    from ragmi.qdrant import QdrantClient
    rng = np.random.default_rng(70)
    n = 2000
    x = rng.standard_normal((n, 384)).astype(np.float32)
    q = x[3] + 0.01 * rng.standard_normal(384).astype(np.float32)
    cl = QdrantClient(device=gpu)
    for name, dt, enc in (("f32", None, O.encode_rows32), ("f16", "float16", O.encode_rows)):
        cl.create_collection(name, models.VectorParams(size=384, distance=models.Distance.COSINE,
                                                       datatype=dt))
        cl.upsert(name, [models.PointStruct(id=j, vector=x[j].tolist(), payload={"r": j})
                         for j in range(n)])
        res = cl.query_points(name, query=q.tolist(), limit=15).points
        s2, i2 = O.search(enc(x), q[None], 15)
        assert [p.id for p in res] == i2[0].tolist()
        assert np.array_equal(np.array([p.score for p in res], np.float32), s2[0])
    assert cl._col("f32").index.storage == "fp32" and cl._col("f16").index.storage == "fp16"
    cl.close()
