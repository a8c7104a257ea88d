"""Searches on CU-partitioned streams (rag_stream_create_cu_partition, bench.py's batches in
flight on small shards): the scan grid is sized to the stream's CU share, the results must not
change — ids and scores equal the default stream's bit for bit, and the oracle's — for plain,
filtered, D = 1024 and k > 32 passes, with the partitions' batches in flight together."""
import numpy as np
import pytest
import torch

import oracle_scan as O

pytestmark = pytest.mark.gpu


def _index(gpu, x, tags=None):
    from ragmi.index import FlatIndex
    idx = FlatIndex(dim=x.shape[1], capacity=x.shape[0], device=gpu)
    idx.upsert(x, np.arange(x.shape[0], dtype=np.int64), tags, new_count=x.shape[0])
    return idx


@pytest.mark.parametrize("whole", [False, True], ids=["quarters", "whole"])
@pytest.mark.parametrize("dim,n,k", [(384, 200_000, 15), (384, 60_000, 100), (1024, 40_000, 15)])
def test_partition_streams_match_default_stream(gpu, dim, n, k, whole):
    """whole=True: full-CU-mask streams (each on a dedicated hardware queue; the config-2/3
    pipelines' batch streams, round 6)"""
    from ragmi.index import PartitionStreams
    rng = np.random.default_rng(dim + k)
    x = rng.standard_normal((n, dim)).astype(np.float32)
    idx = _index(gpu, x)
    qs = [torch.from_numpy(x[rng.choice(n, 32)] + 0.05 * rng.standard_normal((32, dim))
                           .astype(np.float32)).to(gpu) for _ in range(8)]
    ref = [idx.search(q, k) for q in qs]
    torch.cuda.synchronize()
    parts = PartitionStreams(gpu, 4, whole=whole)
    try:
        cur = torch.cuda.current_stream(gpu)
        for s in parts.streams:
            s.wait_stream(cur)
        outs = []
        for i, q in enumerate(qs):                     # all four partitions in flight at once
            with torch.cuda.stream(parts[i % 4]):
                outs.append(idx.search(q, k))
        torch.cuda.synchronize()
        for (s0, i0), (s1, i1) in zip(ref, outs):
            assert torch.equal(i0, i1) and torch.equal(s0, s1)
        s2, i2 = O.search(O.encode_rows(x), qs[0].cpu().numpy(), k)
        np.testing.assert_array_equal(outs[0][1].cpu().numpy(), i2)
        np.testing.assert_array_equal(outs[0][0].cpu().numpy(), s2)
    finally:
        parts.close()
        idx.close()


def test_partition_streams_filtered(gpu):
    from ragmi.index import PartitionStreams
    rng = np.random.default_rng(3)
    n, dim, k = 100_000, 384, 15
    x = rng.standard_normal((n, dim)).astype(np.float32)
    tags = rng.integers(1, 9, n).astype(np.uint32)
    idx = _index(gpu, x, tags)
    q = torch.from_numpy(x[rng.choice(n, 32)]).to(gpu)
    filt = np.array([[0xffffffff, 1 + (i % 8)] for i in range(32)], dtype=np.uint32)
    s0, i0 = idx.search(q, k, filters=filt)
    torch.cuda.synchronize()
    parts = PartitionStreams(gpu, 2)
    try:
        parts[1].wait_stream(torch.cuda.current_stream(gpu))
        with torch.cuda.stream(parts[1]):
            s1, i1 = idx.search(q, k, filters=filt)
        torch.cuda.synchronize()
        assert torch.equal(i0, i1) and torch.equal(s0, s1)
    finally:
        parts.close()
        idx.close()


def test_partition_argument_checks(gpu):
    from ragmi._lib import RagmiError
    from ragmi.index import PartitionStreams
    with pytest.raises(RagmiError):
        PartitionStreams(gpu, 100_000)                  # more parts than CUs
    with pytest.raises(RagmiError):
        PartitionStreams(gpu, 64)       # 4 CUs a part: XCDs without a CU would run on all
    p = PartitionStreams(gpu, 32)       # 8 consecutive CU ids: one CU of every XCD
    p.close()


def test_streams_recreated_at_reused_addresses(gpu):
    """Partition streams closed and new streams created (possibly at the same handles): the
    index re-reads each workspace's CU share (stream generation counter), and the
    results stay the default stream's."""
    from ragmi.index import PartitionStreams
    rng = np.random.default_rng(9)
    n, dim, k = 120_000, 384, 15
    x = rng.standard_normal((n, dim)).astype(np.float32)
    idx = _index(gpu, x)
    q = torch.from_numpy(x[rng.choice(n, 32)]).to(gpu)
    s0, i0 = idx.search(q, k)
    torch.cuda.synchronize()
    try:
        for parts_n, whole in ((4, False), (2, True), (8, False), (4, True)):
            parts = PartitionStreams(gpu, parts_n, whole=whole)
            try:
                for st in parts.streams:
                    st.wait_stream(torch.cuda.current_stream(gpu))
                outs = []
                for st in parts.streams:
                    with torch.cuda.stream(st):
                        outs.append(idx.search(q, k))
                torch.cuda.synchronize()
                for s1, i1 in outs:
                    assert torch.equal(i0, i1) and torch.equal(s0, s1)
            finally:
                parts.close()
    finally:
        idx.close()
