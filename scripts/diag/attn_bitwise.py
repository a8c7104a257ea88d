"""Bitwise check of attention variants against VAR 42 at the rerank shape (diagnostic build:
RAGMI_LIB_AB=<-DRAGMI_DIAG_BUILD build>). Usage: VARIANTS=554 python scripts/diag/attn_bitwise.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
from ragmi.encoders import attention  # noqa: E402


def main():
    rng = np.random.default_rng(3)
    for lo_len, hi_len in ((200, 289), (5, 40), (280, 512)):
        lens = rng.integers(lo_len, hi_len, 96)
        cu = torch.from_numpy(np.r_[0, np.cumsum(lens)].astype(np.int32)).cuda()
        T = int(lens.sum())
        x = torch.randn((T, 1152), device="cuda") * 2
        hi = x.half()
        lo = (x - hi.float()).half()
        ref = [t.clone() for t in attention(hi, cu, int(lens.max()), lo, 42)]
        for v in [int(s) for s in os.environ.get("VARIANTS", "554").split(",")]:
            out = attention(hi, cu, int(lens.max()), lo, v)
            same = all(torch.equal(a.view(torch.int16), b.view(torch.int16)) for a, b in zip(ref, out))
            print(json.dumps({"variant": v, "lens": [lo_len, hi_len], "bitwise_equal_to_42": same}))
            assert same


if __name__ == "__main__":
    main()
