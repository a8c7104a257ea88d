"""Is the config-2 serving loop bound by host-side launches? (round 3 probe)

For the bge-small query forward (32 queries, ~21 tokens each) and the 1M-row search pass:
host microseconds per call to ENQUEUE (ctypes + every hipLaunchKernel inside; the stream is
kept short of full so enqueue never blocks) against device microseconds per call (HIP events
over back-to-back calls). If enqueue >= device time, the GPU idles between kernels whatever
the number of streams. One JSON line per stage.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

from ragmi import synth as R  # noqa: E402
from ragmi.encoders import HEAD_CLS_L2, BertEncoder  # noqa: E402
from ragmi.index import FlatIndex  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(7)
    cfg = R.BGE_SMALL
    enc = BertEncoder(cfg, R.make_weights(cfg, 1), HEAD_CLS_L2, dev, "fp16x3", diagnostic=True)
    lens = rng.integers(16, 27, 32)
    ids = np.concatenate([rng.integers(1000, 30000, L).astype(np.int32) for L in lens])
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    t_ids = torch.from_numpy(ids).to(dev)
    t_tt = torch.zeros_like(t_ids)
    t_cu = torch.from_numpy(cu).to(dev)
    out = enc.forward_packed(ids, np.zeros_like(ids), cu)
    st = torch.cuda.Stream(dev)         # a non-null stream (graph replay needs one)
    torch.cuda.set_stream(st)
    T, B, S = int(cu[-1]), len(lens), int(lens.max())

    def enc_call():
        enc._L.rag_encoder_forward(enc._h, t_ids.data_ptr(), t_tt.data_ptr(), t_cu.data_ptr(),
                                   B, T, S, out.data_ptr(), st.cuda_stream)

    idx = FlatIndex(384, capacity=1_000_000, device=dev, diagnostic=True)
    for c in range(4):
        x = torch.randn(250_000, 384, device=dev)
        idx.upsert(x, torch.arange(c * 250_000, (c + 1) * 250_000, device=dev))
    q = torch.nn.functional.normalize(torch.randn(32, 384, device=dev), dim=1)
    idx.search(q, 15)

    def search_call():
        idx.search(q, 15)

    tt_np = np.zeros_like(ids)

    def enc_api():      # what the serving loop calls: numpy ids in, H2D staging included
        enc.forward_packed(ids, tt_np, cu)

    def enc_null():     # the library's default: the caller's current stream is the null stream
        with torch.cuda.stream(torch.cuda.default_stream(dev)):
            enc.forward_packed(ids, tt_np, cu)

    def graphs(mode):
        def f():
            enc.set_graphs(mode)
        return f

    for name, fn, reps, setup in (
            ("encode_q forward, eager", enc_call, 20, graphs(0)),
            ("encode_q forward, graph replay", enc_call, 20, graphs(1)),
            ("search pass 1M", search_call, 20, graphs(-1)),
            ("encode_q forward_packed (python API), eager", enc_api, 20, graphs(0)),
            ("encode_q forward_packed (python API), graph replay", enc_api, 20, graphs(1)),
            ("encode_q forward_packed (python API), null stream, graph replay", enc_null, 20,
             graphs(1))):
        setup()
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        host = []
        for _ in range(5):
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            host.append((time.perf_counter() - t0) / reps * 1e6)
            torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        es = torch.cuda.default_stream(dev) if fn is enc_null else st
        a.record(es)
        for _ in range(reps):
            fn()
        b.record(es)
        torch.cuda.synchronize(dev)
        devus = a.elapsed_time(b) / reps * 1e3
        print(json.dumps({"stage": name, "host_enqueue_us": round(float(np.median(host)), 1),
                          "device_us": round(devus, 1), "tokens": T if "encode" in name else None}),
              flush=True)


if __name__ == "__main__":
    main()
