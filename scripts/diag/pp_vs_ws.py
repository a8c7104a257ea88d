"""Diagnostic: the PP GEMM vs the WS GEMM bitwise at the rerank forward's token count, every
shape / epilogue of a MiniLM layer; prints mismatching rows / columns."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
from ragmi.encoders import linear  # noqa: E402

M = int(os.environ.get("M", 117996))
for (N, K, epi) in [(1152, 384, 0), (384, 384, 2), (1536, 384, 1), (384, 1536, 2), (768, 384, 0)]:
    g = torch.Generator(device="cuda")
    g.manual_seed(N + K)
    a32 = torch.randn((M, K), generator=g, device="cuda")
    w32 = torch.randn((N, K), generator=g, device="cuda") / math.sqrt(K)
    bias = torch.randn((N,), generator=g, device="cuda") * 0.1
    a, w = a32.half(), w32.half()
    al, wl = (a32 - a.float()).half(), (w32 - w.float()).half()
    p = linear(a, w, bias, epi, al, wl, 45)
    q = linear(a, w, bias, epi, al, wl, 19)
    torch.cuda.synchronize()
    pv = p if epi == 2 else p[0].float() + p[1].float()
    qv = q if epi == 2 else q[0].float() + q[1].float()
    bad = pv != qv
    nb = int(bad.sum())
    print(f"M={M} N={N} K={K} epi={epi}: {nb} mismatches", flush=True)
    if nb:
        r, c = torch.nonzero(bad, as_tuple=True)
        print("  rows", sorted(set((r // 256).tolist()))[:20], "panel-rows", sorted(set((r % 256).tolist()))[:40])
        print("  cols", sorted(set((c // 192).tolist()))[:20], "tile-cols", sorted(set((c % 192).tolist()))[:40])
        print("  max diff", float((pv - qv).abs().max()))
