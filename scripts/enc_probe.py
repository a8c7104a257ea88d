"""Runs the config-3 rerank forward (480 pairs, ~117K tokens, MiniLM-L6 shape) REPS times in
one precision — a fixed workload for rocprofv3 counter passes over the encoder kernels."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
from ragmi import synth as R  # noqa: E402  (model shapes, seeded weights)
from ragmi.encoders import HEAD_POOLER_CLS, BertEncoder  # noqa: E402

prec = os.environ.get("PREC", "fp16")
reps = int(os.environ.get("REPS", "3"))
dev = torch.device("cuda", 0)
enc = BertEncoder(R.MINILM_CE, R.make_weights(R.MINILM_CE, 2), HEAD_POOLER_CLS, dev, prec, diagnostic=True)
rng = np.random.default_rng(0)
lens = rng.integers(200, 289, 480)
ids = rng.integers(1000, 30000, int(lens.sum())).astype(np.int32)
tt = np.zeros_like(ids)
cu = np.r_[0, np.cumsum(lens)].astype(np.int32)
for _ in range(reps):
    enc.forward_packed(ids, tt, cu)
torch.cuda.synchronize()
print("done", int(cu[-1]), "tokens")
