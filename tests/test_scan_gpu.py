"""GPU parity tests of the flat index (HIP scan + top-k + exact merge) against the oracle.

Bar: bit-exact stored rows, bit-exact top-k ids and scores (the canonical arithmetic of
oracle/scan_ref.c), on the committed golden fixtures and on seeded inputs at sizes the
oracle finishes in seconds; at 1M rows, against the BLAS-shortlist oracle (exact rescoring)
and through size-independent properties (planted neighbours, idempotent re-upsert).
"""
import numpy as np
import pytest
import torch

import oracle_scan as O

pytestmark = pytest.mark.gpu


def make_index(gpu, x, tags=None, capacity=None):
    from ragmi.index import FlatIndex
    n = x.shape[0]
    idx = FlatIndex(dim=x.shape[1], capacity=capacity or max(n, 16), device=gpu)
    if n:
        idx.upsert(x, np.arange(n, dtype=np.int64), tags, new_count=n)
    return idx


def search(idx, q, k, filters=None):
    s, i = idx.search(q, k, filters=filters)
    torch.cuda.synchronize()
    return s.cpu().numpy(), i.cpu().numpy()


def test_upsert_stores_canonical_fp16(gpu, golden_scan):
    g = golden_scan
    idx = make_index(gpu, g["x"], g["tags"])
    np.testing.assert_array_equal(idx.export_rows(), g["enc16"])
    np.testing.assert_array_equal(idx.export_tags(), g["tags"])


@pytest.mark.parametrize("k,key", [(15, "15"), (5, "5")])
def test_search_golden_bit_exact(gpu, golden_scan, k, key):
    g = golden_scan
    idx = make_index(gpu, g["x"], g["tags"])
    s, i = search(idx, g["q"], k)
    np.testing.assert_array_equal(i, g["ids" + key])
    np.testing.assert_array_equal(s, g["s" + key])


def test_search_golden_filtered_per_query(gpu, golden_scan):
    g = golden_scan
    idx = make_index(gpu, g["x"], g["tags"])
    s, i = search(idx, g["q"], 15, filters=g["filt"])
    np.testing.assert_array_equal(i, g["idsf"])
    np.testing.assert_array_equal(s, g["sf"])


@pytest.mark.parametrize("n,b,k", [(5003, 32, 15), (5003, 1, 5), (4096, 7, 32), (777, 45, 15),
                                   (16, 3, 1), (1, 2, 15)])
def test_search_random_vs_oracle(gpu, n, b, k):
    rng = np.random.default_rng(n * 131 + b)
    x = rng.standard_normal((n, 384)).astype(np.float32)
    q = rng.standard_normal((b, 384)).astype(np.float32)
    idx = make_index(gpu, x)
    s, i = search(idx, q, k)
    enc = O.encode_rows(x)
    s2, i2 = O.search(enc, q, k)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)


def test_many_duplicates_tie_break_by_row(gpu):
    rng = np.random.default_rng(3)
    base = rng.standard_normal((1, 384)).astype(np.float32)
    x = rng.standard_normal((3000, 384)).astype(np.float32)
    dup_rows = rng.choice(3000, 80, replace=False)
    x[dup_rows] = base                           # 80 identical rows spread over many waves
    q = base + 0.01 * rng.standard_normal((4, 384)).astype(np.float32)
    idx = make_index(gpu, x)
    s, i = search(idx, q, 32)
    s2, i2 = O.search(O.encode_rows(x), q, 32)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(i[0], np.sort(dup_rows)[:32])


def test_massive_ties_take_exact_fallback(gpu):
    """> kCandCap (256) list heads tie at the threshold: select's exact column-sort fallback."""
    rng = np.random.default_rng(17)
    base = rng.standard_normal((1, 384)).astype(np.float32)
    x = rng.standard_normal((12000, 384)).astype(np.float32)
    x[::2] = base                                 # 6000 identical rows in every tile
    q = base + 0.02 * rng.standard_normal((3, 384)).astype(np.float32)
    idx = make_index(gpu, x)
    s, i = search(idx, q, 32)
    np.testing.assert_array_equal(i, np.tile(np.arange(0, 64, 2), (3, 1)))
    s2, i2 = O.search(O.encode_rows(x), q, 32)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)


def test_empty_and_sparse_filters(gpu):
    rng = np.random.default_rng(5)
    x = rng.standard_normal((2000, 384)).astype(np.float32)
    tags = np.zeros(2000, np.uint32)
    tags[[5, 999, 1500]] = 7
    idx = make_index(gpu, x, tags)
    q = rng.standard_normal((3, 384)).astype(np.float32)
    filt = np.array([[0xFFFF, 7], [0xFFFF, 9], [0, 0]], np.uint32)
    s, i = search(idx, q, 15, filters=filt)
    assert sorted(i[0][:3]) == [5, 999, 1500] and (i[0][3:] == -1).all()
    assert np.isneginf(s[0][3:]).all()
    assert (i[1] == -1).all()
    s2, i2 = O.search(O.encode_rows(x), q[2:], 15)
    np.testing.assert_array_equal(i[2], i2[0])
    # empty index
    from ragmi.index import FlatIndex
    e = FlatIndex(384, 64, gpu)
    s, i = search(e, q, 5)
    assert (i == -1).all()


def test_overwrite_is_idempotent_and_last_write_wins(gpu):
    rng = np.random.default_rng(9)
    x = rng.standard_normal((1000, 384)).astype(np.float32)
    idx = make_index(gpu, x)
    before = idx.export_rows()
    idx.upsert(x[:100], np.arange(100))          # re-ingest: byte-identical
    np.testing.assert_array_equal(idx.export_rows(), before)
    y = rng.standard_normal((10, 384)).astype(np.float32)
    idx.upsert(y, np.arange(500, 510))
    np.testing.assert_array_equal(idx.export_rows(500, 10), O.encode_rows(y))
    assert idx.count == 1000


def test_reserve_grows_and_keeps_rows(gpu):
    rng = np.random.default_rng(11)
    x = rng.standard_normal((100, 384)).astype(np.float32)
    idx = make_index(gpu, x, capacity=100)
    idx.reserve(10000)
    more = rng.standard_normal((2000, 384)).astype(np.float32)
    idx.upsert(more, np.arange(100, 2100))
    allx = np.concatenate([x, more])
    np.testing.assert_array_equal(idx.export_rows(), O.encode_rows(allx))
    q = rng.standard_normal((5, 384)).astype(np.float32)
    s, i = search(idx, q, 15)
    s2, i2 = O.search(O.encode_rows(allx), q, 15)
    np.testing.assert_array_equal(i, i2)


def test_sharded_merge_equals_unsharded(gpu):
    """G logical shards on one device: per-shard exact top-k with id offsets,
    merged by rag_merge_topk, equal the unsharded result id-for-id."""
    from ragmi.index import merge_topk
    rng = np.random.default_rng(13)
    n, b, k = 6000, 32, 15
    x = rng.standard_normal((n, 384)).astype(np.float32)
    q = rng.standard_normal((b, 384)).astype(np.float32)
    full = make_index(gpu, x)
    s_ref, i_ref = search(full, q, k)
    for G in (2, 3, 8):
        bounds = np.linspace(0, n, G + 1).astype(int)
        ss, ii = [], []
        for g in range(G):
            sh = make_index(gpu, x[bounds[g]:bounds[g + 1]])
            s, i = sh.search(q, k, id_offset=int(bounds[g]))
            ss.append(s)
            ii.append(i)
        ms, mi = merge_topk(torch.stack(ss), torch.stack(ii), k)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mi.cpu().numpy(), i_ref)
        np.testing.assert_array_equal(ms.cpu().numpy(), s_ref)


@pytest.mark.parametrize("dim", [384, 1024])
def test_sharded_packed_exchange_equals_unsharded(gpu, dim):
    """The one-collective exchange form (rag_index_search_packed -> all-gather ->
    rag_merge_topk_packed) over G logical shards equals the unsharded search; a shard with
    fewer than k rows contributes -1 entries that the merge skips."""
    from ragmi.index import merge_topk_packed
    rng = np.random.default_rng(14)
    n, b, k = 5000, 40, 15
    x = rng.standard_normal((n, dim)).astype(np.float32)
    q = rng.standard_normal((b, dim)).astype(np.float32)
    full = make_index(gpu, x)
    s_ref, i_ref = search(full, q, k)
    for bounds in ([0, 2500, 5000], [0, 7, 1200, 3000, 5000]):
        packs = []
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            sh = make_index(gpu, x[lo:hi])
            p = sh.search_packed(q, k, id_offset=lo)
            assert p.shape == (b, k, 2) and p.dtype == torch.int32
            packs.append(p)
        ms, mi = merge_topk_packed(torch.stack(packs), k)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mi.cpu().numpy(), i_ref)
        np.testing.assert_array_equal(ms.cpu().numpy(), s_ref)
    with pytest.raises(Exception):
        full.search_packed(q, k, id_offset=2 ** 31 - 10)


def test_one_million_rows_planted_and_exact(gpu):
    """Full-size property test at the config-2 corpus (1M x 384): every planted query finds
    its source row first, and the top-15 equals the exact oracle (BLAS shortlist + canonical
    rescoring) id-for-id: recall@5 = recall@15 = 1.0."""
    n, d, b = 1_000_000, 384, 32
    g = torch.Generator(device=gpu)
    g.manual_seed(0)
    x = torch.randn((n, d), generator=g, device=gpu, dtype=torch.float32)
    from ragmi.index import FlatIndex
    idx = FlatIndex(d, n, gpu)
    idx.upsert(x, torch.arange(n, device=gpu), new_count=n)
    src = torch.randint(0, n, (b,), generator=g, device=gpu)
    q = x[src] + 0.05 * torch.randn((b, d), generator=g, device=gpu)
    s, i = search(idx, q, 15)
    np.testing.assert_array_equal(i[:, 0], src.cpu().numpy())
    enc = idx.export_rows()
    s2, i2 = O.search_fast(enc, q.cpu().numpy(), 15)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)
    # concurrent searches from several threads through the workspace ring stay exact
    import threading
    res = {}

    def worker(t):
        with torch.cuda.stream(torch.cuda.Stream(gpu)):
            res[t] = search(idx, q, 15)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    [t.start() for t in th]
    [t.join() for t in th]
    for t in range(6):
        np.testing.assert_array_equal(res[t][1], i)


@pytest.mark.parametrize("dim,b", [(384, 32), (1024, 128)])
def test_serial_scan_order_across_streams(gpu, dim, b):
    """rag_index_set_scan_order(1): batches issued round-robin on 3 streams without host
    syncs, every scan chained behind the previous one by the handle's event; (2): every scan
    on the handle's own scan stream; each batch's result equals the oracle's (and the
    unordered mode gives the same)."""
    rng = np.random.default_rng(dim + b)
    n = 20_000
    x = rng.standard_normal((n, dim)).astype(np.float32)
    idx = make_index(gpu, x)
    enc = idx.export_rows()
    qs = [x[rng.choice(n, b)] + 0.05 * rng.standard_normal((b, dim)).astype(np.float32)
          for _ in range(6)]
    want = [O.search(enc, q, 15) for q in qs]
    qd = [torch.from_numpy(q).to(gpu) for q in qs]
    streams = [torch.cuda.Stream(gpu) for _ in range(3)]
    for serial in (1, 2, 0):
        idx.set_scan_order(serial)
        torch.cuda.synchronize()
        outs = []
        for j, q in enumerate(qd):
            st = streams[j % 3]
            st.wait_stream(torch.cuda.current_stream(gpu))
            with torch.cuda.stream(st):
                outs.append(idx.search(q, 15))
        torch.cuda.synchronize()
        for (s, i), (s2, i2) in zip(outs, want):
            np.testing.assert_array_equal(i.cpu().numpy(), i2)
            np.testing.assert_array_equal(s.cpu().numpy(), s2)
    idx.close()


# ---- D = 1024 (config 5: bge-large vectors; queries in LDS, scan_lds_kernel)
@pytest.mark.parametrize("n,b,k", [(5003, 32, 15), (4096, 128, 15), (777, 45, 16), (33, 3, 5)])
def test_search_d1024_vs_oracle(gpu, n, b, k):
    rng = np.random.default_rng(n * 7 + b)
    x = rng.standard_normal((n, 1024)).astype(np.float32)
    q = rng.standard_normal((b, 1024)).astype(np.float32)
    idx = make_index(gpu, x)
    enc = O.encode_rows(x)
    np.testing.assert_array_equal(idx.export_rows(), enc)
    s, i = search(idx, q, k)
    s2, i2 = O.search(enc, q, k)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)


def test_search_d1024_filtered_per_query(gpu):
    rng = np.random.default_rng(11)
    n, b = 6000, 40
    x = rng.standard_normal((n, 1024)).astype(np.float32)
    tags = rng.integers(0, 6, n).astype(np.uint32) | (rng.integers(1, 3, n).astype(np.uint32) << 16)
    q = rng.standard_normal((b, 1024)).astype(np.float32)
    filt = np.zeros((b, 2), np.uint32)
    filt[:, 0] = np.where(np.arange(b) % 3 == 0, 0xFFFF, 0xFFFFFFFF)
    filt[:, 1] = rng.integers(0, 6, b).astype(np.uint32) | np.where(
        np.arange(b) % 3 == 0, 0, 1 << 16).astype(np.uint32)
    idx = make_index(gpu, x, tags)
    s, i = search(idx, q, 15, filters=filt)
    enc = O.encode_rows(x)
    for j in range(b):
        s2, i2 = O.search(enc, q[j:j + 1], 15, tags=tags, mask=int(filt[j, 0]),
                          value=int(filt[j, 1]), use_filter=True)
        np.testing.assert_array_equal(i[j], i2[0])
        np.testing.assert_array_equal(s[j], s2[0])


def test_d1024_planted_200k_batch128(gpu):
    """Config-5 shape at a size the oracle shortlist finishes quickly: planted queries find
    their source row first; full top-15 equals the exact oracle."""
    rng = np.random.default_rng(12)
    n, b = 200_000, 128
    x = rng.standard_normal((n, 1024)).astype(np.float32)
    src = rng.choice(n, b, replace=False)
    q = x[src] + 0.05 * rng.standard_normal((b, 1024)).astype(np.float32)
    idx = make_index(gpu, x)
    s, i = search(idx, q, 15)
    assert (i[:, 0] == src).all()
    s2, i2 = O.search_fast(idx.export_rows(), q, 15)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)


def test_d1024_million_rows_batch128(gpu):
    """Config 5's per-rank shape at 1M x 1024, B = 128: corpus generated
    on the device, planted + pure-random queries and a 64-row near-duplicate cluster (its
    queries sit inside the MFMA error band, so the certified select's fallbacks run), every
    query's top-15 ids and scores bit-exact against the certified oracle shortlist
    (oracle_scan.search_fast, exact canonical rescoring), plus a 30-row fp32-encoding pin of
    the stored rows."""
    n, b, d = 1_000_000, 128, 1024
    g = torch.Generator(device=gpu)
    g.manual_seed(1024)
    x = torch.randn((n, d), generator=g, device=gpu)
    rows = torch.arange(900_000, 900_064, device=gpu)
    x[rows] = x[900_000] + 1e-5 * torch.randn((64, d), generator=g, device=gpu)
    src = torch.randint(0, n, (96,), generator=g, device=gpu)
    q = torch.cat([x[src] + 0.05 * torch.randn((96, d), generator=g, device=gpu),
                   torch.randn((24, d), generator=g, device=gpu),
                   x[900_000:900_008] + 1e-4 * torch.randn((8, d), generator=g, device=gpu)])
    from ragmi.index import FlatIndex
    idx = FlatIndex(dim=d, capacity=n, device=gpu)
    idx.upsert(x, torch.arange(n, device=gpu), new_count=n)
    s, i = search(idx, q, 15)
    enc = idx.export_rows()
    pin = np.random.default_rng(3).choice(n, 30, replace=False)
    np.testing.assert_array_equal(enc[pin], O.encode_rows(x[pin].cpu().numpy()))
    del x
    assert (i[:96, 0] == src.cpu().numpy()).mean() > 0.95
    st = {}
    s2, i2 = O.search_fast(enc, q.cpu().numpy(), 15, stats=st)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)
    idx.close()


@pytest.mark.parametrize("dim", [384, 1024])
def test_zero_vectors(gpu, dim):
    """Zero rows and zero queries (COSINE normalisation leaves a zero vector zero, every score
    against it 0): bit-exact vs the oracle, ties by row ascending — for a zero query that is
    the first k rows with the largest score 0 (i.e. every row scoring exactly 0 or above)."""
    rng = np.random.default_rng(dim)
    n = 3000
    x = rng.standard_normal((n, dim)).astype(np.float32)
    x[[0, 7, 100, 2999]] = 0.0
    q = np.concatenate([np.zeros((2, dim), np.float32), rng.standard_normal((3, dim))
                        .astype(np.float32)])
    idx = make_index(gpu, x)
    s, i = search(idx, q, 15)
    s2, i2 = O.search(O.encode_rows(x), q, 15)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)
    np.testing.assert_array_equal(i[0], np.arange(15))
    assert (s[0] == 0).all()
