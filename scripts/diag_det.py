"""Determinism check of the fp16x3 cross-encoder forward: the same batches repeated, outputs
compared bitwise, and max |d| vs the oracle per repeat."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bert_ref as R
from ragmi.encoders import HEAD_POOLER_CLS, BertEncoder, linear
G = np.load(os.path.join(ROOT, "tests", "golden", "bert_golden.npz"))
w = R.make_weights(R.MINILM_CE, int(G["ce_seed"]))
enc = BertEncoder(R.MINILM_CE, w, HEAD_POOLER_CLS, 0, "fp16x3")
for seed in (4, 11, 6):
    rng = np.random.default_rng(seed)
    if seed == 11:
        R.random_batch(rng, 32, 32)
    ids, tt, m = R.random_batch(rng, 15, 288, pair=True)
    ref = R.ce_logits(w, R.MINILM_CE, ids, tt, m)
    outs = [enc.forward_padded(ids, tt, m).cpu().numpy() for _ in range(6)]
    same = all(np.array_equal(outs[0], o) for o in outs)
    print(os.environ.get("RAGMI_GEMM", "auto"), seed, "T", int(m.sum()), "deterministic", same,
          "errs", [float("%.2e" % np.abs(o - ref).max()) for o in outs], flush=True)
# GEMM-level: repeat one SMALL split GEMM and compare bitwise
g = torch.Generator(device="cuda"); g.manual_seed(0)
for (M, N, K) in ((2200, 1152, 384), (2200, 384, 1536), (2200, 384, 384), (2200, 1536, 384)):
    a32 = torch.randn((M, K), generator=g, device="cuda"); w32 = torch.randn((N, K), generator=g, device="cuda") / K ** 0.5
    a, wh = a32.half(), w32.half(); al = (a32 - a.float()).half(); wl = (w32 - wh.float()).half()
    b = torch.randn((N,), generator=g, device="cuda")
    for v in (5, 10, 1):
        cs = [linear(a, wh, b, 2, al, wl, v) for _ in range(8)]
        torch.cuda.synchronize()
        ref = (a.double() + al.double()) @ (wh.double() + wl.double()).T + b.double()
        print("gemm", M, N, K, "variant", v, "deterministic", all(torch.equal(cs[0], c) for c in cs),
              "max err", ["%.2e" % float((c.double() - ref).abs().max()) for c in cs[:3]], flush=True)
