"""Deferred-LayerNorm GEMM epilogues vs the plain WS epilogues on the same operands (one
MiniLM layer's four GEMMs at M tokens, fp16x3): device ms per call via HIP events over
back-to-back launches (bench_gemm.timeit). One JSON line per GEMM."""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from bench_gemm import timeit  # noqa: E402
from ragmi.encoders import (EPI_F16, EPI_F32, EPI_GELU_F16, EPI_LN_F16,  # noqa: E402
                            EPI_LN_GELU_F16, EPI_RES_LN, linear, linear_dl)

WS = 19


def planes(*shape):
    x = torch.randn(shape, device="cuda")
    h = x.half()
    return h, (x - h.float()).half()


def main():
    M = int(os.environ.get("GEMM_M", "117000"))
    H = 384
    st = torch.rand((M, H // 64, 2), device="cuda")
    st[..., 0] -= 0.5
    st[..., 1] = st[..., 1] * 64 + 8
    gamma, beta = torch.ones(H, device="cuda"), torch.zeros(H, device="cuda")
    for name, N, K, epi, dl in (("qkv", 1152, 384, EPI_F16, EPI_LN_F16),
                                ("ffn1", 1536, 384, EPI_GELU_F16, EPI_LN_GELU_F16),
                                ("o", 384, 384, EPI_F32, EPI_RES_LN),
                                ("ffn2", 384, 1536, EPI_F32, EPI_RES_LN)):
        a, al = planes(M, K)
        w, wl = planes(N, K)
        w, wl = w / math.sqrt(K), wl / math.sqrt(K)
        bias = torch.zeros(N, device="cuda")
        c1 = torch.zeros(N, device="cuda")
        ms_plain = timeit(lambda: linear(a, w, bias, epi, al, wl, WS))
        c, cl = planes(M, N)
        so = torch.empty_like(st)
        if dl == EPI_RES_LN:
            fn = lambda: linear_dl(dl, a, al, w, wl, bias, c, cl, st_in=st, gamma=gamma,  # noqa
                                   beta=beta, st_out=so)
        else:
            fn = lambda: linear_dl(dl, a, al, w, wl, bias, c, cl, c1=c1, st_in=st)  # noqa
        ms_dl = timeit(fn)
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "plain_ms": round(ms_plain, 4),
                          "deferred_ms": round(ms_dl, 4),
                          "delta_us": round((ms_dl - ms_plain) * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
