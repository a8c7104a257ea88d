"""Host logic of bench.py's measurement helpers on CPU tensors (no GPU, no oracle library):
recall@5 against the unrounded fp32 corpus, including a corpus split over two shards whose
per-shard lists are merged the way rank 0 merges them."""
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
    assert bench.recall_fp32(q, ref, 0, n, n, 0, 1, dev) == 1.0
    # the best 5 replaced by ranks 11..15: no overlap
    assert bench.recall_fp32(q, ref[:, ::-1].copy(), 0, n, n, 0, 1, dev) == 0.0


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
    assert bench.recall_fp32(q, ref, 0, cut, n, 0, 2, dev) == 1.0
    S = np.concatenate([p[0] for p in shard_parts], axis=1)
    I = np.concatenate([p[1] for p in shard_parts], axis=1)
    top5 = np.take_along_axis(I, np.argsort(-S, axis=1, kind="stable")[:, :5], axis=1)
    assert all(set(top5[b]) == set(ref[b, :5]) for b in range(4))
