"""Where a query-batch GEMM's time goes: the SMALL kernel at M = 782 tokens
(32 bge-small queries) timed over K, so the slope is the cost of one 32-deep K step and the
intercept the launch ramp + prologue + epilogue; the same for the split-K fp32 form and the
add_ln384 pass over the rows. One JSON line per point (min over 5 windows of 50 launches).
Usage (GPU box): python scripts/diag/small_gemm_sweep.py > gpurun_out/small_sweep.jsonl"""
import ctypes
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

from ragmi import _lib  # noqa: E402
from ragmi.encoders import EPI_F16, GEMM_SMALL  # noqa: E402


def timeit(fn, reps=50):
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
        ts.append(a.elapsed_time(b) / reps * 1e3)
    return min(ts)


def operands(M, N, K):
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    a32 = torch.randn((M, K), generator=g, device="cuda")
    w32 = torch.randn((N, K), generator=g, device="cuda") / math.sqrt(K)
    a, w = a32.half(), w32.half()
    return a, (a32 - a.float()).half(), w, (w32 - w.float()).half(), \
        torch.randn((N,), generator=g, device="cuda") * 0.1


def main():
    M = int(os.environ.get("SWEEP_M", "782"))
    L = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    for N in (1152, 384):
        for K in [int(k) for k in os.environ.get("SWEEP_K", "64,128,256,384,768,1536").split(",")]:
            a, al, w, wl, b = operands(M, N, K)
            ch = torch.empty((M, N), dtype=torch.float16, device="cuda")
            cl = torch.empty_like(ch)

            def f16():        # preallocated outputs: the device time, not linear()'s host path
                _lib.check(L.rag_bert_gemm(GEMM_SMALL, EPI_F16, a.data_ptr(), al.data_ptr(),
                                           w.data_ptr(), wl.data_ptr(), b.data_ptr(), M, N, K,
                                           ch.data_ptr(), cl.data_ptr(), st))
            us = timeit(f16)
            tag = os.path.basename(os.environ.get("RAGMI_LIB_AB", "in-tree"))
            print(json.dumps({"lib": tag, "kind": "small_f16", "M": M, "N": N, "K": K, "us": round(us, 2)}),
                  flush=True)
            c = torch.empty((4, M, N), device="cuda")
            parts = ctypes.c_int()

            def sk():
                _lib.check(L.rag_bert_gemm_splitk(GEMM_SMALL, a.data_ptr(), al.data_ptr(),
                                                  w.data_ptr(), wl.data_ptr(), b.data_ptr(), M, N,
                                                  K, c.data_ptr(), 4, ctypes.byref(parts), st))
            us = timeit(sk)
            print(json.dumps({"lib": tag, "kind": "splitk_f32", "M": M, "N": N, "K": K, "parts": parts.value,
                              "us": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
