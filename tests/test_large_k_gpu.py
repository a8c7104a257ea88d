"""Exact top-k for RAG_MAX_K < k <= RAG_MAX_K_LARGE (round 5): Qdrant's
query_points takes any `limit` (/root/reference/main.py:215,232-237), and under the unchanged
reference a refused limit would be swallowed into empty points (main.py:238-239). The large-k
pass (scan_kernels.hip lk_* kernels) must return exactly the oracle's top-k — ids AND scores
bit for bit (oracle/scan_ref.c, canonical fp64 order), ties by row ascending — at D = 384 and
1024, with and without payload filters, with padding where fewer than k rows match, on
near-duplicate clusters whose scores sit inside the MFMA error band, and when a query's first
candidate list overflows (a second, tighter round). Massive exact ties beyond the candidate
capacity are reported as unanswered, never silently truncated, and re-answered by the full
exact pass (round 6), which also serves every k > RAG_MAX_K_LARGE.
"""
import numpy as np
import pytest
import torch

import oracle_scan as O

pytestmark = pytest.mark.gpu


def _index(gpu, x, tags=None, storage="fp16"):
    from ragmi.index import FlatIndex
    idx = FlatIndex(dim=x.shape[1], capacity=x.shape[0], device=gpu, storage=storage)
    idx.upsert(x, np.arange(x.shape[0], dtype=np.int64), tags, new_count=x.shape[0])
    return idx


def _search(idx, q, k, filters=None):
    s, i = idx.search(q, k, filters=filters)
    torch.cuda.synchronize()
    return s.cpu().numpy(), i.cpu().numpy()


def _queries(rng, x, b, dim):
    pick = rng.choice(x.shape[0], b - 3)
    return np.concatenate([x[pick] + 0.05 * rng.standard_normal((b - 3, dim)).astype(np.float32),
                           rng.standard_normal((3, dim)).astype(np.float32)])


@pytest.mark.parametrize("dim,n", [(384, 30_000), (1024, 9_000)])
@pytest.mark.parametrize("k", [33, 64, 100, 500])
def test_large_k_bit_exact(gpu, dim, n, k):
    rng = np.random.default_rng(dim + k)
    x = rng.standard_normal((n, dim)).astype(np.float32)
    q = _queries(rng, x, 12, dim)
    idx = _index(gpu, x)
    s, i = _search(idx, q, k)
    s2, i2 = O.search(O.encode_rows(x), q, k)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)
    assert idx.unanswered() == 0
    idx.close()


@pytest.mark.parametrize("dim", [384, 1024])
def test_large_k_filtered_and_padded(gpu, dim):
    """Per-query payload filters; one ticker holds fewer than k rows (-1 / -inf padding)."""
    rng = np.random.default_rng(7 + dim)
    n, k = 12_000, 100
    x = rng.standard_normal((n, dim)).astype(np.float32)
    tags = rng.integers(1, 5, n).astype(np.uint32)
    tags[rng.choice(n, 60, replace=False)] = 9               # a rare ticker: 60 rows < k
    q = _queries(rng, x, 8, dim)
    vals = [1, 2, 3, 4, 9, 9, 1, 2]
    filters = np.array([[0xffffffff, v] for v in vals], dtype=np.uint32)
    idx = _index(gpu, x, tags)
    s, i = _search(idx, q, k, filters)
    x16 = O.encode_rows(x)
    for b, v in enumerate(vals):
        s2, i2 = O.search(x16, q[b:b + 1], k, tags=tags, mask=0xffffffff, value=v,
                          use_filter=True)
        np.testing.assert_array_equal(i[b], i2[0])
        np.testing.assert_array_equal(s[b], s2[0])
    assert (i[4] >= 0).sum() == 60 and np.all(i[4, 60:] == -1)
    idx.close()


@pytest.mark.parametrize("dim", [384, 1024])
def test_large_k_near_duplicate_cluster(gpu, dim):
    """300 near-duplicates (base + 1e-5 noise) inside the MFMA error band, k = 64 and 100 over
    them, plus 200 exact copies of one row (ties by row ascending)."""
    rng = np.random.default_rng(11 + dim)
    n = 20_000 if dim == 384 else 8_000
    x = rng.standard_normal((n, dim)).astype(np.float32)
    base = rng.standard_normal((1, dim)).astype(np.float32)
    rows = np.sort(rng.choice(n, 300, replace=False))
    x[rows] = base + 1e-5 * rng.standard_normal((300, dim)).astype(np.float32)
    dup = rng.standard_normal((1, dim)).astype(np.float32)
    drows = np.sort(rng.choice(np.setdiff1d(np.arange(n), rows), 200, replace=False))
    x[drows] = dup
    q = np.concatenate([base + 0.01 * rng.standard_normal((4, dim)).astype(np.float32),
                        np.repeat(dup, 2, axis=0), rng.standard_normal((2, dim)).astype(np.float32)])
    idx = _index(gpu, x)
    for k in (64, 100):
        s, i = _search(idx, q, k)
        s2, i2 = O.search(O.encode_rows(x), q, k)
        np.testing.assert_array_equal(i, i2)
        np.testing.assert_array_equal(s, s2)
    assert idx.unanswered() == 0
    idx.close()


def test_large_k_fp32_storage(gpu):
    rng = np.random.default_rng(5)
    n, dim, k = 15_000, 384, 64
    x = rng.standard_normal((n, dim)).astype(np.float32)
    q = _queries(rng, x, 6, dim)
    idx = _index(gpu, x, storage="fp32")
    s, i = _search(idx, q, k)
    s2, i2 = O.search(O.encode_rows32(x), q, k)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)
    idx.close()


def test_large_k_overflow_takes_a_second_round(gpu):
    """1M rows, k = 1000: the first candidate list overflows the per-query capacity for the
    random queries and a tighter round answers them; still bit-exact (certified oracle)."""
    rng = np.random.default_rng(3)
    n, dim, k = 1_000_000, 384, 1000
    x = rng.standard_normal((n, dim)).astype(np.float32)
    q = rng.standard_normal((3, dim)).astype(np.float32)
    idx = _index(gpu, x)
    s, i = _search(idx, q, k)
    s2, i2 = O.search_fast(O.encode_rows(x), q, k)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)
    assert idx.unanswered() == 0
    idx.close()


def test_large_k_massive_ties_are_unanswered_not_truncated(gpu):
    """20000 exact copies of one row and k = 100: every copy ties within the bound of the
    100th best, more than the 16384 candidates a round keeps, so no round can narrow them:
    the query is reported unanswered (-1 ids, rag_index_unanswered) — never a wrong or
    silently truncated list."""
    rng = np.random.default_rng(9)
    n, dim = 24_000, 384
    x = rng.standard_normal((n, dim)).astype(np.float32)
    x[:20_000] = x[0]
    q = np.concatenate([x[:1], rng.standard_normal((1, dim)).astype(np.float32)])
    idx = _index(gpu, x)
    before = idx.unanswered()
    s, i = _search(idx, q, 100)
    assert idx.unanswered() == before + 1
    assert np.all(i[0] == -1)
    s2, i2 = O.search(O.encode_rows(x), q[1:], 100)       # the other query is still exact
    np.testing.assert_array_equal(i[1], i2[0])
    np.testing.assert_array_equal(s[1], s2[0])
    # the full exact pass answers the tied query (round 6): 100 of the 20000
    # copies, the lowest rows first
    sf, i_f = idx.search(q, 100, full=True)
    torch.cuda.synchronize()
    s3, i3 = O.search(O.encode_rows(x), q, 100)
    np.testing.assert_array_equal(i_f.cpu().numpy(), i3)
    np.testing.assert_array_equal(sf.cpu().numpy(), s3)
    assert np.array_equal(i3[0], np.arange(100))
    idx.close()


def test_qdrant_reanswers_massive_ties(gpu):
    """QdrantClient.query_points on the massive-ties collection: the large-k pass leaves the
    tied query unanswered and Collection.search re-runs it on the full pass, so the points come
    back exact instead of empty."""
    from ragmi import qdrant_models as m
    from ragmi.qdrant import QdrantClient
    rng = np.random.default_rng(9)
    n, dim = 24_000, 384
    x = rng.standard_normal((n, dim)).astype(np.float32)
    x[:20_000] = x[0]
    c = QdrantClient(device=gpu)
    c.create_collection("t", m.VectorParams(size=dim, distance=m.Distance.COSINE,
                                            datatype="float16"))
    c.upsert("t", m.Batch(ids=list(range(n)), vectors=x, payloads=[{"ticker": "A"}] * n))
    res = c.query_points("t", query=x[0], limit=100)
    s2, i2 = O.search(O.encode_rows(x), x[:1], 100)
    assert [p.id for p in res.points] == i2[0].tolist()
    assert [p.score for p in res.points] == s2[0].tolist()
    assert c._col("t").rescued == 1
    c.close()


@pytest.mark.parametrize("dim,n,k", [(384, 20_000, 5000), (384, 7_000, 9000), (1024, 9_000, 4500)])
def test_full_pass_any_k(gpu, dim, n, k):
    """k > RAG_MAX_K_LARGE: rag_index_search takes the full exact pass —
    ids and scores bit-exact vs the oracle; k past the row count pads with -1 / -inf."""
    rng = np.random.default_rng(dim + n)
    x = rng.standard_normal((n, dim)).astype(np.float32)
    x[100:140] = x[3]                                       # exact ties: rows ascending
    q = np.concatenate([_queries(rng, x, 6, dim), x[3:4]])
    idx = _index(gpu, x)
    s, i = _search(idx, q, k)
    kk = min(k, n)
    s2, i2 = O.search(O.encode_rows(x), q, kk)
    np.testing.assert_array_equal(i[:, :kk], i2)
    np.testing.assert_array_equal(s[:, :kk], s2)
    assert np.all(i[:, kk:] == -1) and np.all(s[:, kk:] == -np.inf)
    idx.close()


@pytest.mark.parametrize("storage", ["fp16", "fp32"])
def test_full_pass_filtered_and_forced(gpu, storage):
    """Per-query filters with a rare ticker (padding) on the full pass, at k > 4096 and forced
    (full=True) at k = 15 / 100 — the same result as the scan and large-k paths."""
    rng = np.random.default_rng(41)
    n, dim = 15_000, 384
    x = rng.standard_normal((n, dim)).astype(np.float32)
    tags = rng.integers(1, 3, n).astype(np.uint32)
    tags[rng.choice(n, 50, replace=False)] = 7
    q = _queries(rng, x, 5, dim)
    vals = [1, 2, 7, 1, 7]
    filters = np.array([[0xffffffff, v] for v in vals], dtype=np.uint32)
    idx = _index(gpu, x, tags, storage=storage)
    enc = O.encode_rows32(x) if storage == "fp32" else O.encode_rows(x)
    for k, full in ((6000, False), (15, True), (100, True)):
        s, i = idx.search(q, k, filters=filters, full=full)
        torch.cuda.synchronize()
        s, i = s.cpu().numpy(), i.cpu().numpy()
        if k <= 100:
            sp, ip = _search(idx, q, k, filters)                # scan / large-k path
            np.testing.assert_array_equal(i, ip)
            np.testing.assert_array_equal(s, sp)
        for b, v in enumerate(vals):
            s2, i2 = O.search(enc, q[b:b + 1], k, tags=tags, mask=0xffffffff, value=v,
                              use_filter=True)
            np.testing.assert_array_equal(i[b], i2[0])
            np.testing.assert_array_equal(s[b], s2[0])
        assert (i[2] >= 0).sum() == min(50, k)
    idx.close()


def test_large_k_packed_exchange_and_merge(gpu):
    """The multi-GPU form at k > 32: per logical shard rag_index_search_packed with a global
    id offset, then rag_merge_topk_packed (merge_large_kernel) equals the unsharded search."""
    from ragmi.index import merge_topk, merge_topk_packed
    rng = np.random.default_rng(21)
    n, dim, k, parts = 16_000, 384, 100, 3
    x = rng.standard_normal((n, dim)).astype(np.float32)
    q = _queries(rng, x, 8, dim)
    bounds = [0, 5_000, 11_000, n]
    packed = []
    for r in range(parts):
        lo, hi = bounds[r], bounds[r + 1]
        idx = _index(gpu, x[lo:hi])
        packed.append(idx.search_packed(q, k, id_offset=lo))
        torch.cuda.synchronize()
        idx.close()
    s, i = merge_topk_packed(torch.stack(packed), k)
    torch.cuda.synchronize()
    s2, i2 = O.search(O.encode_rows(x), q, k)
    np.testing.assert_array_equal(i.cpu().numpy(), i2)
    np.testing.assert_array_equal(s.cpu().numpy(), s2)
    # the unpacked merge form (rag_merge_topk) of the same lists
    st = torch.stack([p[..., 0].view(torch.float32) for p in packed])
    it = torch.stack([p[..., 1].to(torch.int64) for p in packed])
    s3, i3 = merge_topk(st, it, k)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(i3.cpu().numpy(), i2)
    np.testing.assert_array_equal(s3.cpu().numpy(), s2)


def _np_merge(s, i, k):
    """(score desc, id asc) over the valid entries (id >= 0) of [n_lists, B, k] lists"""
    L, B, _ = s.shape
    out_s = np.full((B, k), -np.inf, np.float32)
    out_i = np.full((B, k), -1, np.int64)
    for b in range(B):
        ss, ii = s[:, b].ravel(), i[:, b].ravel()
        keep = ii >= 0
        ss, ii = ss[keep], ii[keep]
        o = np.lexsort((ii, -ss.astype(np.float64)))[:k]
        out_s[b, :len(o)], out_i[b, :len(o)] = ss[o], ii[o]
    return out_s, out_i


def test_merge_any_k_random_lists(gpu):
    """rag_merge_topk[_packed] past RAG_MAX_K_LARGE (round 6: three stable radix sorts): random
    per-list-sorted inputs whose id ranges interleave across lists, equal scores within and
    across lists, +0 / -0, and padding — equal to the (score desc, id asc) merge."""
    from ragmi.index import MAX_K_LARGE, merge_topk, merge_topk_packed
    rng = np.random.default_rng(17)
    L, B, k = 3, 3, MAX_K_LARGE + 904
    s = np.round(rng.standard_normal((L, B, k)), 2).astype(np.float32)   # many exact ties
    s[0, 0, :50] = 0.0
    s[1, 0, :50] = -0.0
    ids = np.stack([rng.permutation(10 * k)[:k] for _ in range(L * B)]).reshape(L, B, k)
    ids = ids.astype(np.int64)
    ids[2, 1, k // 2:] = -1                                  # a short list (padding)
    s[2, 1, k // 2:] = -np.inf
    for l in range(L):                                       # each list (score desc, id asc)
        for b in range(B):
            v = ids[l, b] >= 0
            o = np.lexsort((ids[l, b][v], -s[l, b][v].astype(np.float64)))
            s[l, b, :v.sum()] = s[l, b][v][o]
            ids[l, b, :v.sum()] = ids[l, b][v][o]
    want_s, want_i = _np_merge(s, ids, k)
    ts, ti = torch.from_numpy(s).to(gpu), torch.from_numpy(ids).to(gpu)
    gs, gi = merge_topk(ts, ti, k)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(gi.cpu().numpy(), want_i)
    np.testing.assert_array_equal(gs.cpu().numpy().view(np.int32), want_s.view(np.int32))
    p = torch.stack([ts.view(torch.int32), torch.where(ti >= 0, ti, -1).to(torch.int32)], -1)
    ps, pi = merge_topk_packed(p.contiguous(), k)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(pi.cpu().numpy(), want_i)
    np.testing.assert_array_equal(ps.cpu().numpy().view(np.int32), want_s.view(np.int32))
    # 64-bit ids (the unpacked form): list 1's ids past 2^33 — the high-word pass orders them
    ids64 = ids.copy()
    ids64[1] = np.where(ids64[1] >= 0, ids64[1] + (1 << 33), -1)
    want_s, want_i = _np_merge(s, ids64, k)
    gs, gi = merge_topk(ts, torch.from_numpy(ids64).to(gpu), k)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(gi.cpu().numpy(), want_i)
    np.testing.assert_array_equal(gs.cpu().numpy().view(np.int32), want_s.view(np.int32))


def test_full_pass_sharded_any_k(gpu):
    """The multi-GPU form past RAG_MAX_K_LARGE: per logical shard the full exact pass with a
    global id offset, then rag_merge_topk's any-k merge equals the unsharded oracle."""
    from ragmi.index import merge_topk
    rng = np.random.default_rng(23)
    n, dim, k = 16_000, 384, 5_500
    x = rng.standard_normal((n, dim)).astype(np.float32)
    x[4_990:5_010] = x[7]                                    # ties straddling a shard bound
    q = np.concatenate([_queries(rng, x, 5, dim), x[7:8]])
    bounds = [0, 5_000, 11_000, n]
    lists_s, lists_i = [], []
    for r in range(3):
        lo, hi = bounds[r], bounds[r + 1]
        idx = _index(gpu, x[lo:hi])
        s, i = idx.search(q, k, id_offset=lo)
        torch.cuda.synchronize()
        lists_s.append(s)
        lists_i.append(i)
        idx.close()
    s, i = merge_topk(torch.stack(lists_s), torch.stack(lists_i), k)
    torch.cuda.synchronize()
    s2, i2 = O.search(O.encode_rows(x), q, k)
    np.testing.assert_array_equal(i.cpu().numpy(), i2)
    np.testing.assert_array_equal(s.cpu().numpy(), s2)
