"""Host logic of bench.py's measurement helpers on CPU tensors (no GPU): recall@5 against
the unrounded fp32 corpus, including a corpus split over two shards whose per-shard lists
are merged the way rank 0 merges them; the certified per-batch exactness check against the
oracle (unsharded and over two shards), which must flag a wrong answer."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


@pytest.fixture
def small_chunks(monkeypatch):
    monkeypatch.setattr(bench, "CHUNK", 1000)

    def gen_chunk(c, dev, rows=1000):
        g = torch.Generator()
        g.manual_seed(1000 + c)
        return torch.randn((rows, bench.D), generator=g)

    monkeypatch.setattr(bench, "gen_chunk", gen_chunk)
    return gen_chunk


def _corpus(gen_chunk, n):
    return torch.cat([gen_chunk(c, None, bench.chunk_rows(c, n))
                      for c in range((n + bench.CHUNK - 1) // bench.CHUNK)])


def test_recall_fp32_exact_and_reversed(small_chunks):
    n = 2500
    x = _corpus(small_chunks, n)
    q = x[[5, 1200, 2400, 77]] + 0.01 * torch.randn(4, bench.D)
    qn = torch.nn.functional.normalize(q, dim=1)
    xn = torch.nn.functional.normalize(x, dim=1)
    ref = torch.topk(qn @ xn.T, 15, dim=1).indices.numpy()
    dev = torch.device("cpu")
    assert bench.recall_fp32(q, ref, 0, n, n, 0, 1, dev).mean() == 1.0
    # the best 5 replaced by ranks 11..15: no overlap
    assert bench.recall_fp32(q, ref[:, ::-1].copy(), 0, n, n, 0, 1, dev).mean() == 0.0


def test_recall_fp32_shard_merge_matches_unsharded(small_chunks, monkeypatch):
    """Two shards [0, 1300) and [1300, 2500): each computes its own top-15 with global row ids;
    merging them as rank 0 does gives the unsharded top-5."""
    n, cut = 2500, 1300
    x = _corpus(small_chunks, n)
    q = x[[10, 1290, 1310, 2499]] + 0.01 * torch.randn(4, bench.D)
    dev = torch.device("cpu")
    qn = torch.nn.functional.normalize(q, dim=1)
    xn = torch.nn.functional.normalize(x, dim=1)
    ref = torch.topk(qn @ xn.T, 15, dim=1).indices.numpy()
    # capture each shard's partial result through a fake all_gather_object
    shard_parts = []
    for lo, hi in ((0, cut), (cut, n)):
        got = {}

        def fake_gather(out, obj, _got=got):
            _got["mine"] = obj
            for i in range(len(out)):
                out[i] = obj
        monkeypatch.setattr(bench.dist, "all_gather_object", fake_gather)
        bench.recall_fp32(q, ref, lo, hi, n, 1, 2, dev)   # rank 1: returns None
        shard_parts.append(got["mine"])

    def merged_gather(out, obj):
        out[0], out[1] = shard_parts
    monkeypatch.setattr(bench.dist, "all_gather_object", merged_gather)
    assert bench.recall_fp32(q, ref, 0, cut, n, 0, 2, dev).mean() == 1.0
    S = np.concatenate([p[0] for p in shard_parts], axis=1)
    I = np.concatenate([p[1] for p in shard_parts], axis=1)
    top5 = np.take_along_axis(I, np.argsort(-S, axis=1, kind="stable")[:, :5], axis=1)
    assert all(set(top5[b]) == set(ref[b, :5]) for b in range(4))


class _Shard:
    """export_rows surface of FlatIndex over oracle-encoded rows."""

    def __init__(self, enc):
        self.enc = enc

    def export_rows(self):
        return self.enc


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_scan as O
    return O


def test_verify_exact_unsharded_flags_wrong_answers():
    O = _oracle()
    rng = np.random.default_rng(4)
    n = 3000
    x = rng.standard_normal((n, bench.D)).astype(np.float32)
    enc = O.encode_rows(x)
    q = np.concatenate([x[[3, 900]] + 0.05 * rng.standard_normal((2, bench.D)).astype(np.float32),
                        rng.standard_normal((2, bench.D)).astype(np.float32)])
    s, i = O.search(enc, q, bench.K_TOP)
    r5, ok = bench.verify_exact(_Shard(enc), q, s, i, 0, 0, 1, torch.device("cpu"))
    assert ok.all() and (r5 == 1.0).all()
    bad_i = i.copy()
    bad_i[1, 0], bad_i[1, 14] = bad_i[1, 14], bad_i[1, 0]      # order swapped
    bad_i[2, 3] = (bad_i[2, 3] + 1) % n                         # a wrong row
    r5, ok = bench.verify_exact(_Shard(enc), q, s, bad_i, 0, 0, 1, torch.device("cpu"))
    assert list(ok) == [True, False, False, True]
    assert r5[2] < 1.0


def test_verify_exact_two_shards(monkeypatch):
    O = _oracle()
    rng = np.random.default_rng(5)
    n, cut = 3000, 1700
    x = rng.standard_normal((n, bench.D)).astype(np.float32)
    enc = O.encode_rows(x)
    q = x[[10, 1650, 1800, 2999]] + 0.05 * rng.standard_normal((4, bench.D)).astype(np.float32)
    s, i = O.search(enc, q, bench.K_TOP)
    shards = [(0, enc[:cut]), (cut, enc[cut:])]
    qn = O.normalize(q)
    # the all-reduce MAX of the per-rank exact scores of the returned rows
    e_all = np.maximum(*[O.rescore(e, qn, np.where((i >= lo) & (i < lo + len(e)), i - lo, -1))
                         for lo, e in shards])
    parts = []
    for rank, (lo, e) in enumerate(shards):
        def fake_reduce(t, op=None):
            t.copy_(torch.from_numpy(e_all))

        def fake_gather(out, obj):
            parts.append(obj)
            for j in range(len(out)):
                out[j] = obj
        monkeypatch.setattr(bench.dist, "all_reduce", fake_reduce)
        monkeypatch.setattr(bench.dist, "all_gather_object", fake_gather)
        bench.verify_exact(_Shard(e), q, s, i, lo, 1, 2, torch.device("cpu"))

    def merged(out, obj):
        out[0], out[1] = parts
    monkeypatch.setattr(bench.dist, "all_gather_object", merged)
    r5, ok = bench.verify_exact(_Shard(shards[0][1]), q, s, i, 0, 0, 2, torch.device("cpu"))
    assert ok.all() and (r5 == 1.0).all()


def test_busy_union_counts_overlap_once():
    """bench.py's device time for overlapped scan launches: the union of their intervals."""
    import numpy as np
    from ragmi.index import busy_union_ms
    assert busy_union_ms(np.array([]), np.array([])) == 0.0
    # disjoint: the plain sum of durations (== the average launch duration x launches)
    assert busy_union_ms(np.array([0.0, 2.0, 5.0]), np.array([1.0, 3.0, 6.5])) == 3.5
    # nested / overlapping / unsorted, negative starts (launches recorded before the first)
    a = np.array([4.0, 0.0, 0.5, -1.0, 10.0])
    b = np.array([6.0, 2.0, 1.0, 0.25, 10.5])
    assert busy_union_ms(a, b) == (2.0 - (-1.0)) + 2.0 + 0.5
