"""Child process of tests/test_dist_rccl_gpu.py (not collected by pytest): the production
multi-GPU exchange of ragmi.dist run over RCCL (torch.distributed backend "nccl") on the one
GPU a test box has.

A world-1 RCCL process group is the most this box can form (RCCL refuses two ranks on one
device), so the N > 1 search is replayed shard by shard: the corpus is split into S contiguous
logical shards (ragmi.dist.shard_bounds), each its own FlatIndex; every shard's
search_packed(id_offset = lo) output goes through ragmi.dist.all_gather_packed — a real
`all_gather_into_tensor` on the RCCL communicator, the call a rank makes at N > 1 — and the
S gathered [1, B, k, 2] blocks are stacked into the [S, B, k, 2] a world-S all-gather returns
and merged by rag_merge_topk_packed (ShardedIndex.search's merge). The result must equal the
unsharded index's search id for id and bit for bit in the scores.

argv: n_rows n_shards k seed. Prints one JSON line."""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))


def main():
    n, shards, k, seed = (int(a) for a in sys.argv[1:5])
    from ragmi.dist import all_gather_packed, shard_bounds
    from ragmi.index import FlatIndex, merge_topk_packed

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        x = torch.randn((n, 384), generator=g, device=dev)
        # near-duplicates across shard boundaries: equal fp16 rows in different shards make
        # the (score desc, row asc) tie-break decide between ranks
        step = n // shards
        for b in range(1, shards):
            x[b * step] = x[b * step - 1]
        q = torch.randn((32, 384), generator=g, device=dev)
        q[:8] = x[(torch.arange(8, device=dev) * step + step - 1) % n] + 1e-3 * q[:8]
        full = FlatIndex(384, n, dev)
        full.upsert(x, torch.arange(n, device=dev))
        ref_s, ref_i = full.search(q, k)
        parts = []
        for r in range(shards):
            lo, hi = shard_bounds(n, r, shards)
            sh = FlatIndex(384, max(hi - lo, 16), dev)
            sh.upsert(x[lo:hi], torch.arange(hi - lo, device=dev))
            p = sh.search_packed(q, k, id_offset=lo)
            parts.append(all_gather_packed(p))          # RCCL all_gather_into_tensor, world 1
            assert parts[-1].shape == (1, 32, k, 2)
            assert torch.equal(parts[-1][0], p)
            sh.close()
        s, i = merge_topk_packed(torch.cat(parts), k)
        torch.cuda.synchronize()
        out = {"backend": dist.get_backend(), "world": dist.get_world_size(),
               "ids_equal": bool(torch.equal(i, ref_i)),
               "scores_bitwise_equal": bool(torch.equal(s.view(torch.int32),
                                                        ref_s.view(torch.int32))),
               "rows": n, "shards": shards, "k": k}
        full.close()
    finally:
        dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
