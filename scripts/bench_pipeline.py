"""End-to-end retrieval pipeline on one MI355X — BASELINE.json configs 2 and 3:

  config 2: batch of 32 queries -> bge-small encode -> cosine top-15 over 1M x 384 fp16
  config 3: ... -> ms-marco-MiniLM cross-encoder rerank of the 32 x 15 (query, chunk) pairs
            -> top-5 per query (main.py:_ask_impl stages 1-3, batched as main2.batch_processor)

Everything after the query token ids stays on the GPU: the chunk token ids of every corpus row
live in HBM (tokenised at ingest; here synthetic, 180-260 tokens per row, uint16), the
(query, chunk) pairs are assembled on the GPU from the search result ([CLS] q [SEP] c [SEP],
token types 0/1, truncated to 512) and fed to the packed cross-encoder forward; the top-5 per
query is a torch.topk over the 15 logits (the reference's np.argsort(...)[::-1][:5]).
Synthetic seeded weights (real checkpoints absent), random token ids; per-stage device times
with HIP events. Precision: fp16x3 (the parity mode: rerank logits within 1e-3) and fp16.
One JSON line per (config, precision).
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

from ragmi import synth as R  # noqa: E402  (model shapes, seeded weights)
from ragmi.encoders import HEAD_CLS_L2, HEAD_POOLER_CLS, BertEncoder  # noqa: E402
from ragmi.index import FlatIndex  # noqa: E402
from ragmi.pairs import build_pairs_gpu  # noqa: E402

N, D, B, K, TOPK = 1_000_000, 384, 32, 15, 5
LC_MAX = 260
CLS, SEP = 101, 102   # query batches carry their own [CLS] ... [SEP] (dropped in pairs)


def chunk_tokens(dev):
    """Synthetic per-row chunk token ids (what ingest would tokenise once), uint16 [N, 260]."""
    g = torch.Generator(device=dev)
    g.manual_seed(77)
    toks = torch.randint(1000, 30000, (N, LC_MAX), generator=g, device=dev, dtype=torch.int32)
    lens = torch.randint(180, LC_MAX + 1, (N,), generator=g, device=dev, dtype=torch.int32)
    return toks.to(torch.int16), lens


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    steps = int(os.environ.get("STEPS", "20"))
    idx = FlatIndex(dim=D, capacity=N, device=dev, diagnostic=True)
    for c in range(N // 1_000_000):
        g = torch.Generator(device=dev)
        g.manual_seed(1000 + c)
        x = torch.randn((1_000_000, D), generator=g, device=dev)
        idx.upsert(x, torch.arange(c * 1_000_000, (c + 1) * 1_000_000, device=dev))
        del x
    c_toks, c_lens = chunk_tokens(dev)
    rng = np.random.default_rng(3)
    batches = []
    for _ in range(steps + 3):
        lens = rng.integers(16, 33, B)
        ids = np.concatenate([np.r_[CLS, rng.integers(1000, 30000, L - 2), SEP] for L in lens])
        batches.append((ids.astype(np.int32), np.zeros(len(ids), np.int32),
                        np.r_[0, np.cumsum(lens)].astype(np.int32)))
    for prec in ("fp16x3", "fp16"):
        bge = BertEncoder(R.BGE_SMALL, R.make_weights(R.BGE_SMALL, 1), HEAD_CLS_L2, dev, prec, diagnostic=True)
        ce = BertEncoder(R.MINILM_CE, R.make_weights(R.MINILM_CE, 2), HEAD_POOLER_CLS, dev, prec, diagnostic=True)
        for cfg in (2, 3):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            acc = np.zeros(3)
            torch.cuda.synchronize()
            t0 = None
            for i, (ids, tt, cu) in enumerate(batches):
                if i == 3:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                ev[0].record()
                q = bge.forward_packed(ids, tt, cu)                  # stage 1
                ev[1].record()
                s, rows = idx.search(q, K)                           # stage 2
                ev[2].record()
                if cfg == 3:                                         # stage 3
                    q_ids = torch.from_numpy(ids).to(dev)
                    q_cu = torch.from_numpy(cu).to(dev)
                    pid, pty, pcu, mx = build_pairs_gpu(q_ids, q_cu, rows, c_toks, c_lens)
                    logits = ce.forward_device(pid, pty, pcu, mx).view(B, K)
                    top = torch.topk(logits, TOPK, dim=1).indices
                    _ = torch.gather(rows, 1, top)
                ev[3].record()
                if i >= 3:
                    torch.cuda.synchronize()
                    acc += [ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]),
                            ev[2].elapsed_time(ev[3])]
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(json.dumps({
                "config": cfg, "precision": prec,
                "workload": f"batch {B} queries (16-32 tokens) -> bge-small -> top-{K} over "
                            f"{N}x{D} fp16" + (f" -> MiniLM-L6 CE rerank of {B}x{K} pairs "
                                               f"(~220-290 tokens) -> top-{TOPK}" if cfg == 3
                                               else ""),
                "qps": round(B * steps / el, 1), "ms_per_batch": round(el / steps * 1e3, 3),
                "stage_ms": {"encode": round(acc[0] / steps, 3),
                             "search": round(acc[1] / steps, 3),
                             "rerank_incl_pair_build": round(acc[2] / steps, 3)},
                "note": "per-batch host sync (stage timing); synthetic weights/tokens"}),
                flush=True)
            # pipelined: batch i on stream i % S, no per-batch sync (a serving loop with S
            # batches in flight; each stream has its own encoder / index workspaces)
            for S in [int(x) for x in os.environ.get("PIPE_STREAMS", "2,4").split(",")]:
                streams = [torch.cuda.Stream(dev) for _ in range(S)]

                def run(i, ids, tt, cu):
                    with torch.cuda.stream(streams[i % S]):
                        q = bge.forward_packed(ids, tt, cu)
                        s_, rows = idx.search(q, K)
                        if cfg == 3:
                            q_ids = torch.from_numpy(ids).to(dev)
                            q_cu = torch.from_numpy(cu).to(dev)
                            pid, pty, pcu, mx = build_pairs_gpu(q_ids, q_cu, rows, c_toks,
                                                                c_lens)
                            logits = ce.forward_device(pid, pty, pcu, mx).view(B, K)
                            top = torch.topk(logits, TOPK, dim=1).indices
                            return torch.gather(rows, 1, top)
                        return rows
                torch.cuda.synchronize()
                for i in range(3):
                    run(i, *batches[i])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(3, len(batches)):
                    run(i, *batches[i])
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                print(json.dumps({"config": cfg, "precision": prec, "batches_in_flight": S,
                                  "qps": round(B * steps / el, 1),
                                  "ms_per_batch": round(el / steps * 1e3, 3)}), flush=True)
        bge.close()
        ce.close()
    idx.close()


if __name__ == "__main__":
    main()
