"""Diagnostic timing of the PP GEMM: per epilogue kind at the rerank size (plain F16 vs GELU
at N = 1536; the deferred-LN epilogues through rag_bert_gemm_dl), against WS."""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from bench_gemm import timeit  # noqa: E402
from ragmi.encoders import linear, linear_dl  # noqa: E402
from ragmi.index import FlatIndex  # noqa: E402

_diag = FlatIndex(384, 16, torch.device("cuda", 0), diagnostic=True)   # honour RAGMI_* knobs
M = int(os.environ.get("M", 117000))
g = torch.Generator(device="cuda")
g.manual_seed(0)
for (name, N, K, epi) in [("qkv_f16", 1152, 384, 0), ("ffn1_f16", 1536, 384, 0),
                          ("ffn1_gelu", 1536, 384, 1)]:
    a = torch.randn((M, K), generator=g, device="cuda").half()
    w = (torch.randn((N, K), generator=g, device="cuda") / math.sqrt(K)).half()
    al = (torch.randn((M, K), generator=g, device="cuda") * 1e-4).half()
    wl = (torch.randn((N, K), generator=g, device="cuda") * 1e-5).half()
    bias = torch.zeros((N,), device="cuda")
    for v, vn in ((19, "ws"), (45, "pp"), (48, "pp_no_store")):
        ms = timeit(lambda: linear(a, w, bias, epi, al, wl, v))
        print(json.dumps({"gemm": name, "variant": vn, "ms": round(ms, 4),
                          "stagger": os.environ.get("RAGMI_PP_STAGGER", "0")}), flush=True)
# deferred-LN epilogues (the forward's QKV / FFN1): WS or PP by RAGMI_GEMM_PP (read once)
for (name, N, epi) in [("qkv_ln", 1152, 4), ("ffn1_ln_gelu", 1536, 5)]:
    K = 384
    a = torch.randn((M, K), generator=g, device="cuda").half()
    al = (torch.randn((M, K), generator=g, device="cuda") * 1e-4).half()
    w = (torch.randn((N, K), generator=g, device="cuda") / math.sqrt(K)).half()
    wl = (torch.randn((N, K), generator=g, device="cuda") * 1e-5).half()
    bias = torch.zeros((N,), device="cuda")
    c1 = torch.randn((N,), generator=g, device="cuda")
    st = torch.stack([torch.zeros((M, 6), device="cuda"), torch.full((M, 6), 64.0, device="cuda")], -1).contiguous()
    c = torch.empty((M, N), dtype=torch.float16, device="cuda")
    cl = torch.empty_like(c)
    ms = timeit(lambda: linear_dl(epi, a, al, w, wl, bias, c, cl, c1=c1, st_in=st))
    print(json.dumps({"gemm": name, "variant": "pp" if os.environ.get("RAGMI_GEMM_PP", "1") != "0" else "ws",
                      "ms": round(ms, 4), "stagger": os.environ.get("RAGMI_PP_STAGGER", "0")}), flush=True)
