"""Where does the per-batch exchange of the N > 1 search cost go? (round 3 probe, one GPU)

A world-1 torch.distributed "nccl" (= RCCL) group and a 1.25M-row shard (the 8-GPU shard
size), 4 batches in flight on 4 streams as bench.py runs them, timing K batches of each
variant of the per-batch tail:
  plain       local search (the 1-GPU step)
  packed      search_packed + rag_merge_topk_packed, no collective
  pg          search_packed + dist.all_gather_into_tensor + merge (ragmi.dist's N > 1 path)
  pg_async    the same with async_op=True and work.wait() (the stream wait without the
              process group's own current-stream synchronisation path)
Prints one JSON line per variant and rep: qps, and the host's enqueue time per batch (the
loop's wall time before the final synchronize) — host-bound when it approaches the step."""
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

import bench  # noqa: E402


def main():
    rows = int(os.environ.get("ROWS", "1250000"))
    steps, warm = int(os.environ.get("STEPS", "300")), 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    no_pg = os.environ.get("NO_PG") == "1"          # baseline: no communicator at all
    # PG_MODE: eager (device_id: the communicator is created at init), lazy (no device_id:
    # created at the first collective), late (eager, after the index is built)
    pg_mode = os.environ.get("PG_MODE", "eager")

    def init_pg():
        if pg_mode == "lazy":
            dist.init_process_group("nccl")
        else:
            dist.init_process_group("nccl", device_id=dev)
    if not no_pg and pg_mode != "late":
        init_pg()
    from ragmi.dist import all_gather_packed
    from ragmi.index import FlatIndex, merge_topk_packed
    idx = FlatIndex(bench.D, rows, dev, diagnostic=True)
    bench.build_shard(idx, 0, rows, rows, dev)
    qs, _ = bench.make_queries(warm + steps, rows, dev)
    if not no_pg and pg_mode == "late":
        init_pg()
    S = int(os.environ.get("STREAMS", "4"))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    for s in streams[1:]:
        s.wait_stream(streams[0])
    k = bench.K_TOP

    def tail(mode, q):
        if mode == "plain":
            return idx.search(q, k)
        p = idx.search_packed(q, k)
        if mode == "packed":
            return merge_topk_packed(p.view((1,) + tuple(p.shape)), k)
        if mode == "pg":
            return merge_topk_packed(all_gather_packed(p), k)
        out = torch.empty((p.shape[0],) + tuple(p.shape[1:]), dtype=p.dtype, device=p.device)
        w = dist.all_gather_into_tensor(out, p, async_op=True)
        w.wait()
        return merge_topk_packed(out.view((1,) + tuple(p.shape)), k)

    modes = os.environ.get("MODES", "plain,packed,pg,pg_async").split(",")
    for rep in range(2):
        for mode in modes:
            for i in range(warm):
                with torch.cuda.stream(streams[i % S]):
                    tail(mode, qs[i])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                with torch.cuda.stream(streams[i % S]):
                    tail(mode, qs[warm + i])
            t_enq = time.perf_counter() - t0
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(json.dumps({"mode": mode, "rep": rep, "rows": rows, "streams": S,
                              "pg": "none" if no_pg else pg_mode,
                              "env": os.environ.get("PROBE_ENV_LABEL"),
                              "qps": round(bench.B * steps / el, 1),
                              "us_per_step": round(el / steps * 1e6, 1),
                              "host_enqueue_us_per_step": round(t_enq / steps * 1e6, 1)}),
                  flush=True)
    idx.close()
    if not no_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
