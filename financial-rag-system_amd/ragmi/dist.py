"""Corpus sharded over the GPUs of one node.

One process per GPU. Rank r holds the contiguous global rows [lo_r, hi_r) of the collection
in its own in-HBM FlatIndex. A search is:
  local scan + per-wave top-k + exact-rescoring select   (libragmi.so, this rank's stream)
  -> ONE all-gather of the per-shard exact top-k, packed as int32 pairs (score bits, global
     row: B*k*8 bytes/rank) over RCCL/xGMI (torch.distributed backend "nccl" = RCCL on ROCm)
  -> GPU merge of world lists by (score desc, id asc)  (rag_merge_topk)
Because every shard reports canonical exact scores, the merged result equals the unsharded
one id-for-id (tests/test_scan_gpu.py::test_sharded_merge_equals_unsharded).

This replaces the per-request HTTP hop to the Qdrant service (reference main.py:232-237);
the reference itself has no multi-GPU component.

Allocation order matters on MI355X: build (or load) the shard BEFORE RCCL's communicator is
created — init the process group without `device_id`, so the communicator appears at the
first collective. Created first, its buffers left the shard with a physical placement that
scans ~8% slower (1.25M-row shard: 184K vs 201K qps; DESIGN §6, profiles/r03w_rccl_probe.jsonl).
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


def shard_bounds(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous row range [lo, hi) of `rank` (sizes differ by at most one row)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return n_total * rank // world, n_total * (rank + 1) // world


def owner_of(row: int, n_total: int, world: int) -> int:
    """Rank holding global row `row` under shard_bounds."""
    r = (row * world) // max(n_total, 1)
    while shard_bounds(n_total, r, world)[0] > row:
        r -= 1
    while shard_bounds(n_total, r, world)[1] <= row:
        r += 1
    return r


def all_gather_lists(scores: torch.Tensor, ids: torch.Tensor, group=None):
    """[B, k] per rank -> [world, B, k] on every rank (RCCL all-gather on GPU tensors,
    gloo list all-gather on CPU tensors)."""
    world = dist.get_world_size(group)
    if scores.is_cuda and dist.get_backend(group) == "nccl":
        out_s = torch.empty((world,) + tuple(scores.shape), dtype=scores.dtype,
                            device=scores.device)
        out_i = torch.empty((world,) + tuple(ids.shape), dtype=ids.dtype, device=ids.device)
        dist.all_gather_into_tensor(out_s, scores.contiguous(), group=group)
        dist.all_gather_into_tensor(out_i, ids.contiguous(), group=group)
        return out_s, out_i
    dev = scores.device
    sc, ic = scores.detach().cpu().contiguous(), ids.detach().cpu().contiguous()   # gloo: host
    ls = [torch.empty_like(sc) for _ in range(world)]
    li = [torch.empty_like(ic) for _ in range(world)]
    dist.all_gather(ls, sc, group=group)
    dist.all_gather(li, ic, group=group)
    return torch.stack(ls).to(dev), torch.stack(li).to(dev)


def _gpu_merge(s, i, k):
    from .index import merge_topk
    return merge_topk(s, i, k)


def _gpu_merge_packed(p, k):
    from .index import merge_topk_packed
    return merge_topk_packed(p, k)


def all_gather_packed(p: torch.Tensor, group=None) -> torch.Tensor:
    """[B, k, 2] int32 per rank -> [world, B, k, 2] on every rank in ONE collective (RCCL
    over xGMI on device tensors; gloo on host tensors). The concatenated output form
    ([world * B, k, 2], the same bytes) is the one every backend implements."""
    world = dist.get_world_size(group)
    out = torch.empty((world * p.shape[0],) + tuple(p.shape[1:]), dtype=p.dtype,
                      device=p.device)
    dist.all_gather_into_tensor(out, p.contiguous(), group=group)
    return out.view((world,) + tuple(p.shape))


class ShardedIndex:
    """A collection of n_total rows sharded over the process group's ranks.

    `local` is this rank's index object: anything with
        search(queries, k, filters=None, id_offset=0) -> (scores [B,k], ids [B,k])
    (a ragmi.index.FlatIndex in production). `merge` combines [world, B, k] lists into the
    global [B, k] (the rag_merge_topk GPU kernel by default).
    """

    def __init__(self, n_total: int, local=None, dim: int = 384, device=None, group=None,
                 merge: Callable | None = None, merge_packed: Callable | None = None,
                 storage: str = "fp16", force_exchange: bool = False,
                 diagnostic: bool = False):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.n_total = int(n_total)
        self.lo, self.hi = shard_bounds(self.n_total, self.rank, self.world)
        if local is None:
            from .index import FlatIndex
            local = FlatIndex(dim=dim, capacity=max(self.hi - self.lo, 16), device=device,
                              storage=storage, diagnostic=diagnostic)
        self.local = local
        self.merge = merge or _gpu_merge
        self.merge_packed = merge_packed or _gpu_merge_packed
        # packed exchange (one collective of (score bits, int32 row) pairs) whenever the
        # local shard offers it and global rows fit int32: the production path on RCCL, and
        # on gloo with a host-side merge_packed (tests/test_dist_cpu.py)
        self.packed = ((merge is None or merge_packed is not None) and
                       hasattr(local, "search_packed") and self.n_total < 2 ** 31 and
                       dist.is_initialized())
        # force_exchange: run the packed all-gather + merge even at world 1 (bench.py's
        # one-GPU RCCL rehearsal, RAGMI_DIST_REHEARSAL; same results as the plain search)
        self.force_exchange = bool(force_exchange) and self.packed

    @property
    def rows(self) -> int:
        return self.hi - self.lo

    def owns(self, global_rows: torch.Tensor) -> torch.Tensor:
        return (global_rows >= self.lo) & (global_rows < self.hi)

    def upsert_global(self, vectors: torch.Tensor, global_rows: torch.Tensor, tags=None):
        """Keep the rows this rank owns (vectors/rows may be the full batch on every rank)."""
        m = self.owns(global_rows)
        if bool(m.any()):
            rows = (global_rows[m] - self.lo).to(torch.int64)
            t = tags[m] if tags is not None else None
            cnt = max(getattr(self.local, "count", 0), int(rows.max()) + 1)
            self.local.upsert(vectors[m], rows, t, new_count=cnt)

    def search(self, queries, k: int, filters=None):
        from .index import MAX_K_LARGE
        # the packed exchange carries k <= MAX_K_LARGE; a larger `limit` (answered by each
        # shard's full exact pass) goes through the unpacked lists and the any-k merge
        if (self.world > 1 or self.force_exchange) and self.packed and k <= MAX_K_LARGE:
            # one all-gather of the packed (score bits, int32 row) lists instead of two
            p = self.local.search_packed(queries, k, filters=filters, id_offset=self.lo)
            return self.merge_packed(all_gather_packed(p, self.group), k)
        s, i = self.local.search(queries, k, filters=filters, id_offset=self.lo)
        if self.world == 1:
            return s, i
        gs, gi = all_gather_lists(s, i, self.group)
        return self.merge(gs, gi, k)

    def save(self, path: str) -> None:
        """Collective: write the whole collection to one shard directory (ragmi.store)."""
        from .store import save_sharded
        save_sharded(self, path)

    def load(self, path: str) -> int:
        """Load this rank's rows from a shard directory saved at any world size."""
        from .store import load_sharded
        return load_sharded(self, path)
