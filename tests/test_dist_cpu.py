"""CPU (gloo) tests of the N > 1 path: contiguous row shards, per-shard top-k
with global id offsets, all-gather, merge by (score desc, id asc) == unsharded result.

The per-shard search here is the oracle (the GPU scan cannot run on CPU) and the merges are
numpy restatements of rag_merge_topk / rag_merge_topk_packed; what is under test is
ragmi.dist's sharding, id offsets and exchange plumbing with world_size 2 and 3 over gloo on
127.0.0.1 — including the production packed exchange (search_packed -> ONE all-gather of
[B, k, 2] int32 (score bits, global row) -> packed merge), the exact bytes RCCL carries."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _paths():
    for p in (ROOT, os.path.join(ROOT, "financial-rag-system_amd"), os.path.join(ROOT, "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)


class OracleShard:
    def __init__(self, enc16, tags=None):
        self.enc16, self.tags = enc16, tags
        self.count = enc16.shape[0]

    def search(self, q, k, filters=None, id_offset=0):
        import oracle_scan as O
        q = q.numpy() if isinstance(q, torch.Tensor) else q
        s = np.empty((q.shape[0], k), np.float32)
        i = np.empty((q.shape[0], k), np.int64)
        for b in range(q.shape[0]):
            m, v = (0, 0) if filters is None else (int(filters[b][0]), int(filters[b][1]))
            s[b], i[b] = [a[0] for a in O.search(self.enc16, q[b:b + 1], k, tags=self.tags,
                                                 mask=m, value=v, use_filter=filters is not None)]
        i = np.where(i >= 0, i + id_offset, -1)
        return torch.from_numpy(s), torch.from_numpy(i)

    def search_packed(self, q, k, filters=None, id_offset=0):
        """rag_index_search_packed's exchange format: int32 [B, k, 2] = (fp32 score bits,
        global row; -1 = none)."""
        s, i = self.search(q, k, filters, id_offset)
        p = np.empty(tuple(s.shape) + (2,), np.int32)
        p[..., 0] = s.numpy().view(np.int32)
        p[..., 1] = np.where(i.numpy() >= 0, i.numpy(), -1).astype(np.int32)
        return torch.from_numpy(p)


def np_merge_packed(p, k):
    """numpy restatement of merge_exact_kernel<PACKED> (csrc/scan_kernels.hip): the union of
    the gathered lists' valid entries (row >= 0), ordered by (score desc, row asc), first k."""
    p = p.numpy()
    W, B = p.shape[:2]
    out_s = np.full((B, k), -np.inf, np.float32)
    out_i = np.full((B, k), -1, np.int64)
    for b in range(B):
        s = p[:, b, :, 0].ravel().view(np.float32)
        i = p[:, b, :, 1].ravel().astype(np.int64)
        keep = i >= 0
        s, i = s[keep], i[keep]
        o = np.lexsort((i, -s.astype(np.float64)))[:k]
        out_s[b, :len(o)], out_i[b, :len(o)] = s[o], i[o]
    return torch.from_numpy(out_s), torch.from_numpy(out_i)


def np_merge(gs, gi, k):
    gs, gi = gs.numpy(), gi.numpy()
    W, B, _ = gs.shape
    out_s = np.full((B, k), -np.inf, np.float32)
    out_i = np.full((B, k), -1, np.int64)
    for b in range(B):
        s = gs[:, b].ravel()
        i = gi[:, b].ravel()
        keep = i >= 0
        s, i = s[keep], i[keep]
        o = np.lexsort((i, -s.astype(np.float64)))[:k]
        out_s[b, :len(o)], out_i[b, :len(o)] = s[o], i[o]
    return torch.from_numpy(out_s), torch.from_numpy(out_i)


def _worker(rank, world, port, n, q, x, tags, filt, result_q, packed=False):
    _paths()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_scan as O
        from ragmi.dist import ShardedIndex, shard_bounds
        lo, hi = shard_bounds(n, rank, world)
        shard = OracleShard(O.encode_rows(x[lo:hi]), tags[lo:hi])
        if packed:
            sh = ShardedIndex(n, local=shard, merge_packed=np_merge_packed)
            assert sh.packed
        else:
            sh = ShardedIndex(n, local=shard, merge=np_merge)
            assert not sh.packed
        assert (sh.lo, sh.hi) == (lo, hi)
        s, i = sh.search(torch.from_numpy(q), 15)
        sf, i_f = sh.search(torch.from_numpy(q), 15, filters=filt)
        if rank == 0:
            result_q.put((s.numpy(), i.numpy(), sf.numpy(), i_f.numpy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("packed", [False, True], ids=["lists", "packed"])
@pytest.mark.parametrize("world,n", [(2, 1001), (3, 1001), (3, 25)])
def test_sharded_search_equals_unsharded_gloo(world, n, packed):
    """n = 25 at world 3: shards of 8-9 rows, fewer than k = 15 (-1 entries in the exchange)."""
    _paths()
    import oracle_scan as O
    rng = np.random.default_rng(world)
    x = rng.standard_normal((n, 384)).astype(np.float32)
    tags = rng.integers(1, 4, n).astype(np.uint32)
    q = x[rng.choice(n, 6)] + 0.05 * rng.standard_normal((6, 384)).astype(np.float32)
    filt = np.array([[0, 0], [0xFFFF, 1], [0xFFFF, 2], [0xFFFF, 3], [0xFFFF, 9], [0, 0]],
                    np.uint32)
    ctx = mp.get_context("spawn")
    result_q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, n, q, x, tags, filt, result_q, packed))
             for r in range(world)]
    [p.start() for p in procs]
    s, i, sf, i_f = result_q.get(timeout=240)
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    enc = O.encode_rows(x)
    s2, i2 = O.search(enc, q, 15)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_array_equal(s, s2)
    for b in range(q.shape[0]):
        a, c = O.search(enc, q[b:b + 1], 15, tags=tags, mask=int(filt[b, 0]),
                        value=int(filt[b, 1]), use_filter=True)
        np.testing.assert_array_equal(i_f[b], c[0])
    assert (i_f[4] == -1).all()     # filter value never ingested: empty on every shard


def test_shard_bounds_cover_and_owner():
    _paths()
    from ragmi.dist import owner_of, shard_bounds
    for n in (0, 1, 7, 10_000_000, 10_000_003):
        for world in (1, 2, 3, 4, 8):
            b = [shard_bounds(n, r, world) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[r][1] == b[r + 1][0] for r in range(world - 1))
            assert max(h - lo for lo, h in b) - min(h - lo for lo, h in b) <= 1
            for row in (0, n // 2, n - 1):
                if 0 <= row < n:
                    r = owner_of(row, n, world)
                    assert b[r][0] <= row < b[r][1]


def _worker_big_k(rank, world, port, n, q, x, k, result_q):
    _paths()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_scan as O
        from ragmi.dist import ShardedIndex, shard_bounds

        class NoPacked(OracleShard):
            def search_packed(self, *a, **kw):
                raise AssertionError("k > MAX_K_LARGE must not use the packed exchange")

        lo, hi = shard_bounds(n, rank, world)
        sh = ShardedIndex(n, local=NoPacked(O.encode_rows(x[lo:hi])), merge=np_merge,
                          merge_packed=np_merge_packed)
        assert sh.packed
        s, i = sh.search(torch.from_numpy(q), k)
        if rank == 0:
            result_q.put((s.numpy(), i.numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_search_any_limit_uses_the_list_exchange_gloo():
    """A `limit` past RAG_MAX_K_LARGE (the packed exchange's bound) goes through the unpacked
    per-shard lists and the any-k merge (rag_merge_topk, stable radix sorts on the GPU;
    its numpy restatement here): the unsharded oracle's result, padded past the row count."""
    _paths()
    import oracle_scan as O
    from ragmi.index import MAX_K_LARGE
    rng = np.random.default_rng(5)
    n, world, k = 4500, 2, MAX_K_LARGE + 500
    x = rng.standard_normal((n, 384)).astype(np.float32)
    x[10:20] = x[0]                                           # exact ties across the shards
    x[3000:3010] = x[0]
    q = np.concatenate([x[:1], rng.standard_normal((2, 384)).astype(np.float32)])
    ctx = mp.get_context("spawn")
    result_q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_big_k, args=(r, world, port, n, q, x, k, result_q))
             for r in range(world)]
    [p.start() for p in procs]
    s, i = result_q.get(timeout=300)
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    s2, i2 = O.search(O.encode_rows(x), q, n)
    np.testing.assert_array_equal(i[:, :n], i2)
    np.testing.assert_array_equal(s[:, :n], s2)
    assert (i[:, n:] == -1).all() and (s[:, n:] == -np.inf).all()
