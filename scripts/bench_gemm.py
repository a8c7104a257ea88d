"""Encoder GEMM benchmark: TILE (gemm_kernel) vs PIPE (gemm_pipe_kernel) on the encoder
shapes, through rag_bert_gemm. One JSON line per (shape, precision, variant):
device ms per call (HIP events, median of reps), algorithmic TFLOP/s (2 M N K), and the
MFMA-pipe fraction of the 2.5 PF dense fp16 peak (fp16x3 issues 3 MFMAs per product).

Shapes (M = tokens): rerank batch 32 x 15 pairs x ~244 tokens = 117K (config 3), chunk
encode 64 x ~232 = 14.8K (ingest EMBED_BATCH), query batch 32 x ~24 = 782.
"""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

from ragmi.encoders import EPI_F16, EPI_F32, EPI_GELU_F16, linear  # noqa: E402

PEAK = 2.5e15
VNAME = {0: "auto", 1: "tile", 5: "small", 19: "ws", 20: "ws_mfma_only", 21: "ws_no_store",
         22: "ws_dma_only"}
LAYERS = {
    "small": [("qkv", 1152, 384, EPI_F16), ("o", 384, 384, EPI_F32),
              ("ffn1", 1536, 384, EPI_GELU_F16), ("ffn2", 384, 1536, EPI_F32)],
    # bge-large-en-v1.5 (config 5 query encoder): hidden 1024, FFN 4096
    "large": [("qkv", 3072, 1024, EPI_F16), ("o", 1024, 1024, EPI_F32),
              ("ffn1", 4096, 1024, EPI_GELU_F16), ("ffn2", 1024, 4096, EPI_F32)],
}


def timeit(fn, reps=20):
    """Device ms per call: `reps` back-to-back launches between two events (a single launch
    between events would also time the host-side launch latency)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    return min(ts)


def main():
    Ms = [int(x) for x in os.environ.get("GEMM_M", "117000,14800,782").split(",")]
    variants = [int(x) for x in os.environ.get("GEMM_VARIANTS", "1,19").split(",")]
    for M in Ms:
        for prec in os.environ.get("GEMM_PRECS", "fp16,fp16x3").split(","):
            vs = list(variants)
            tot = {v: 0.0 for v in vs}
            for name, N, K, epi in LAYERS[os.environ.get("GEMM_LAYER", "small")]:
                g = torch.Generator(device="cuda")
                g.manual_seed(0)
                a = torch.randn((M, K), generator=g, device="cuda").half()
                w = (torch.randn((N, K), generator=g, device="cuda") / math.sqrt(K)).half()
                bias = torch.zeros((N,), device="cuda")
                al = (torch.randn((M, K), generator=g, device="cuda") * 1e-4).half() \
                    if prec == "fp16x3" else None
                wl = (torch.randn((N, K), generator=g, device="cuda") * 1e-5).half() \
                    if prec == "fp16x3" else None
                for v in vs:
                    ms = timeit(lambda: linear(a, w, bias, epi, al, wl, v))
                    fl = 2.0 * M * N * K
                    pipe_fl = fl * (3 if prec == "fp16x3" else 1)
                    tot[v] += ms
                    print(json.dumps({"M": M, "gemm": name, "N": N, "K": K, "precision": prec,
                                      "variant": VNAME[v],
                                      "ms": round(ms, 4),
                                      "TFLOPs": round(fl / ms / 1e9, 1),
                                      "mfma_frac": round(pipe_fl / ms / 1e-3 / PEAK, 4)}),
                          flush=True)
            print(json.dumps({"M": M, "precision": prec,
                              "layer": os.environ.get("GEMM_LAYER", "small"), "layer_ms":
                              {(VNAME[v]): round(t, 4)
                               for v, t in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
