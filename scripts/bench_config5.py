"""Config 5 (BASELINE.json / SURVEY §8d, §8f row 4): queries/sec + recall@5 of cosine top-15
over a 50M x 1024 fp16 corpus (bge-large-en-v1.5 vector width) at batch 128.

One step = one batch of 128 queries: query prep -> seed sampling -> ONE scan launch that
serves all four 32-query groups (scan_wide_kernel: every tile is staged into LDS once and
consumed by all groups' waves) -> exact select. N > 1: same contiguous-shard + RCCL all-gather
merge as bench.py (python -m torch.distributed.run --nproc-per-node N scripts/bench_config5.py).
50M x 1024 fp16 = 102.4 GB: fits one MI355X (288 GB).

recall@5 is measured against a streamed GPU fp32 reference (torch matmul of the fp16-rounded
normalised rows, chunk by chunk with a running top-15) for the first timed batch. Synthetic
data: torch randn corpus in 1M-row chunks seeded 5000+c; planted queries (corpus row +
0.05 N(0,1)), every 4th batch pure random. Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

D = 1024
K_TOP = 15
CHUNK = 1_000_000
HBM_PEAK = 8.0e12


def gen_chunk(c, dev, rows):
    g = torch.Generator(device=dev)
    g.manual_seed(5000 + c)
    return torch.randn((rows, D), generator=g, device=dev, dtype=torch.float32)


def chunk_rows(c, n):
    return min(CHUNK, n - c * CHUNK)


def build_shard(idx, lo, hi, n, dev):
    for c in range(lo // CHUNK, (hi - 1) // CHUNK + 1):
        x = gen_chunk(c, dev, chunk_rows(c, n))
        a, b = max(lo, c * CHUNK), min(hi, c * CHUNK + x.shape[0])
        rows = torch.arange(a - lo, b - lo, device=dev, dtype=torch.int64)
        idx.upsert(x[a - c * CHUNK:b - c * CHUNK], rows, new_count=max(idx.count, b - lo))
        del x
    torch.cuda.synchronize()


def make_queries(nb, batch, n, dev):
    rng = np.random.default_rng(7)
    picks = rng.integers(0, n, (nb, batch))
    rows = {}
    for c in sorted(set((picks // CHUNK).ravel().tolist())):
        x = gen_chunk(c, dev, chunk_rows(c, n))
        for r in np.unique(picks[(picks // CHUNK) == c]):
            rows[int(r)] = x[int(r) - c * CHUNK].clone()
        del x
    g = torch.Generator(device=dev)
    g.manual_seed(8)
    qs = []
    for i in range(nb):
        base = torch.stack([rows[int(r)] for r in picks[i]])
        noise = torch.randn((batch, D), generator=g, device=dev)
        qs.append((base + 0.05 * noise if i % 4 != 3 else noise).contiguous())
    return qs


def reference_top(q, lo, hi, n, dev):
    """fp32 scores of the fp16-rounded normalised rows [lo, hi), streamed, running top-15."""
    qn = torch.nn.functional.normalize(q.double(), dim=1).float()
    best_s = torch.full((q.shape[0], K_TOP), -float("inf"), device=dev)
    best_i = torch.full((q.shape[0], K_TOP), -1, device=dev, dtype=torch.int64)
    for c in range(lo // CHUNK, (hi - 1) // CHUNK + 1):
        x = gen_chunk(c, dev, chunk_rows(c, n))
        a, b = max(lo, c * CHUNK), min(hi, c * CHUNK + x.shape[0])
        xs = x[a - c * CHUNK:b - c * CHUNK].double()
        x16 = (xs / xs.norm(dim=1, keepdim=True)).float().half().float()
        s = qn @ x16.T
        ids = torch.arange(a, b, device=dev, dtype=torch.int64)
        cs = torch.cat([best_s, s], 1)
        ci = torch.cat([best_i, ids.expand(q.shape[0], -1)], 1)
        best_s, o = torch.topk(cs, K_TOP, dim=1)
        best_i = torch.gather(ci, 1, o)
        del x, xs, x16, s
    return best_s, best_i


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=50_000_000)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--no-recall", action="store_true")
    ap.add_argument("--diagnostic", action="store_true",
                    help="create the index with RAG_CREATE_DIAGNOSTIC (RAGMI_* A/B knobs honoured)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group(os.environ.get("RAGMI_DIST_BACKEND", "nccl"))   # lazy comm (bench.py)
    from ragmi.dist import ShardedIndex

    n = args.rows
    sh = ShardedIndex(n, dim=D, device=dev, diagnostic=args.diagnostic)
    idx, lo, hi = sh.local, sh.lo, sh.hi
    t_build = time.perf_counter()
    build_shard(idx, lo, hi, n, dev)
    t_build = time.perf_counter() - t_build
    qs = make_queries(args.warmup + args.steps, args.batch, n, dev)
    for w in range(args.warmup):
        sh.search(qs[w], K_TOP)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    idx.profile(4)
    t0 = time.perf_counter()
    first = None
    for k in range(args.steps):
        out = sh.search(qs[args.warmup + k], K_TOP)
        if k == 0:
            first = out
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    idx.profile(0)
    scan_ms, launches = idx.profile_scan_ms()
    scan_avg = scan_ms / max(launches, 1)
    if world > 1:
        t = torch.tensor([elapsed, scan_avg], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, scan_avg = float(t[0]), float(t[1])

    recall5 = top1_planted = None
    if not args.no_recall:
        q0 = qs[args.warmup]
        rs, ri = reference_top(q0, lo, hi, n, dev)
        if world > 1:
            from ragmi.dist import all_gather_lists
            gs, gi = all_gather_lists(rs, ri, sh.group)
            rs, ri = sh.merge(gs, gi, K_TOP)
        got = first[1].cpu().numpy()
        ref = ri.cpu().numpy()
        recall5 = float(np.mean([len(set(got[b, :5]) & set(ref[b, :5])) / 5
                                 for b in range(got.shape[0])]))
    if rank == 0:
        algo = (hi - lo) * D * 2
        ach = algo / (scan_avg * 1e-3)
        print(json.dumps({
            "metric": "queries/sec + recall@5, batch=128 over 50Mx1024 corpus (config 5)",
            "value": round(args.batch * args.steps / elapsed, 2), "unit": "queries/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "fp16",
            "data": "synthetic (torch randn corpus, 1M-row chunks seeded 5000+c; planted "
                    "queries, every 4th batch pure random)",
            "config": {"workload": f"cosine top-{K_TOP} over {n}x{D} fp16 corpus, "
                                   f"batch={args.batch}, {world} shard(s)",
                       "corpus_rows": n, "dim": D, "batch": args.batch, "k": K_TOP,
                       "rows_per_gpu": hi - lo, "query_groups_per_launch": args.batch // 32},
            "recall_at_5_vs_fp32": recall5,
            "roofline": {"bound": "hbm", "achieved": round(ach / 1e9, 1),
                         "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": round(ach / HBM_PEAK, 4),
                         "kernel": ("scan_wide_kernel<1024>" if args.batch > 32
                                    else "scan_lds_kernel<1024,false,true>"),
                         "avg_ms": round(scan_avg, 4),
                         "algorithmic_bytes_per_launch": algo},
            "build_s": round(t_build, 2),
            "diagnostic_knobs": ({k: v for k, v in os.environ.items() if k.startswith("RAGMI_")}
                                 if args.diagnostic else None),
        }), flush=True)
    idx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
