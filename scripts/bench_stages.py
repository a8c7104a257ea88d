"""Stage benchmark of the encoders (BASELINE configs 2-3):

  encode_q   bge-small, 32 queries x 16-32 tokens        (main2.py batch_processor stage 1)
  encode_q_large  bge-large shape (1024/16 heads/4096, 24 layers), 128 queries (config 5)
  encode_c   bge-small, 64 chunks x 200-260 tokens       (ingest.py embed_chunks, EMBED_BATCH=64)
  rerank     MiniLM-L6 CE, 32 queries x 15 pairs x ~288 tokens (config 3 stage 2)

Per stage: device ms per call (HIP events on the stream), tokens/s, and MFMA-rate accounting
(GEMM FLOPs = 2 * tokens * params-per-token; attention 4*S*H per token per layer; fp16x3
issues 3 MFMAs per product, so its MFMA-pipe work is 3x the algorithmic FLOPs). Synthetic
seeded weights (real checkpoints absent), random token ids. One JSON line per stage.
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

PEAK_F16 = 2.5e15   # dense fp16 MFMA, MI355X_MICROARCH.md


def flops_per_token(cfg, S):
    H, FF = cfg["hidden"], cfg["inter"]
    gemm = 2 * (4 * H * H + 2 * H * FF)
    attn = 4 * S * H
    return cfg["layers"] * (gemm + attn)


def batch(rng, B, lo, hi, pair=False):
    lens = rng.integers(lo, hi + 1, B)
    ids = np.concatenate([rng.integers(1000, 30000, L).astype(np.int32) for L in lens])
    tt = np.zeros_like(ids)
    if pair:
        off = 0
        for L in lens:
            tt[off + L // 4: off + L] = 1
            off += L
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    return ids, tt, cu


def run(enc, ids, tt, cu, reps):
    out = enc.forward_packed(ids, tt, cu)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # queue everything first so host-side packing is outside the device interval
    t_ids = torch.from_numpy(ids).cuda()
    t_tt = torch.from_numpy(tt).cuda()
    t_cu = torch.from_numpy(cu).cuda()
    L = np.diff(cu)
    a.record(st)
    for _ in range(reps):
        enc._L.rag_encoder_forward(enc._h, t_ids.data_ptr(), t_tt.data_ptr(), t_cu.data_ptr(),
                                   len(L), int(cu[-1]), int(L.max()), out.data_ptr(),
                                   st.cuda_stream)
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def cpu_torch_baseline(cfg, w, ids, tt, cu, head, budget=10.0):
    """The reference stack's arithmetic on CPU: transformers BertModel / ...ForSequence-
    Classification in fp32 torch on the host cores, padded batch (as sentence-transformers)."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden_bert as M
    L = np.diff(cu)
    S = int(L.max())
    B = len(L)
    pid = np.zeros((B, S), np.int64)
    ptt = np.zeros_like(pid)
    pm = np.zeros_like(pid)
    for i in range(B):
        pid[i, :L[i]], ptt[i, :L[i]], pm[i, :L[i]] = ids[cu[i]:cu[i + 1]], tt[cu[i]:cu[i + 1]], 1
    model = M.hf_model(cfg, w, head == HEAD_POOLER_CLS)
    t0 = time.perf_counter()
    n = 0
    with torch.no_grad():
        while True:
            model(input_ids=torch.from_numpy(pid), token_type_ids=torch.from_numpy(ptt),
                  attention_mask=torch.from_numpy(pm))
            n += 1
            if time.perf_counter() - t0 > budget:
                break
    return (time.perf_counter() - t0) / n * 1e3, torch.get_num_threads()


def main():
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    reps = int(os.environ.get("REPS", "20"))
    do_cpu = os.environ.get("CPU", "1") == "1"
    stages = [("encode_q", R.BGE_SMALL, HEAD_CLS_L2, (32, 16, 32, False)),
              ("encode_c", R.BGE_SMALL, HEAD_CLS_L2, (64, 200, 260, False)),
              ("rerank", R.MINILM_CE, HEAD_POOLER_CLS, (480, 200, 288, True)),
              # config 5 query encoder: bge-large-en-v1.5 shape, 128 queries
              ("encode_q_large", R.BGE_LARGE, HEAD_CLS_L2, (128, 16, 32, False))]
    only = os.environ.get("STAGES")          # e.g. STAGES=rerank PRECS=fp16x3
    precs = os.environ.get("PRECS", "fp16,fp16x3").split(",")
    for prec in precs:
        for name, cfg, head, (B, lo, hi, pair) in stages:
            if only and name not in only.split(","):
                continue
            w = R.make_weights(cfg, 1)
            enc = BertEncoder(cfg, w, head, dev, prec, diagnostic=True)
            ids, tt, cu = batch(rng, B, lo, hi, pair)
            # DEFERS=-1,0: the deferred LayerNorm (rag_encoder_set_defer_ln) auto, then off
            for defer in [int(v) for v in os.environ.get("DEFERS", "-1").split(",")]:
                enc.set_defer_ln(defer)
                # FFNS=0,1: the fused deferred-LN FFN (rag_encoder_set_ffn_fused) off / on
                for ffn in [int(v) for v in os.environ.get("FFNS", "-1").split(",")]:
                    enc.set_ffn_fused(ffn)
                    stage_line(enc, name, prec, cfg, head, w, ids, tt, cu, B, reps, do_cpu,
                               defer, ffn)
            enc.close()


def stage_line(enc, name, prec, cfg, head, w, ids, tt, cu, B, reps, do_cpu, defer, ffn=-1):
    ms = run(enc, ids, tt, cu, reps)
    T = int(cu[-1])
    S = float(np.mean(np.diff(cu)))
    fl = T * flops_per_token(cfg, S)
    mult = 3 if prec == "fp16x3" else 1
    line = {"stage": name, "precision": prec, "sequences": B, "tokens": T,
            "ms": round(ms, 4), "tokens_per_s": round(T / ms * 1e3, 1),
            "algo_TFLOPs": round(fl / ms / 1e9, 1),
            "mfma_pipe_frac_of_2.5PF": round(fl * mult / (ms * 1e-3) / PEAK_F16, 4),
            "defer_ln": defer, "ffn_fused": ffn}
    save = os.environ.get("SAVE_OUT")         # digest of the forward's output bytes (A/B
    if save:                                  # builds / knobs must agree bit for bit)
        import hashlib
        o = enc.forward_packed(ids, tt, cu).cpu().numpy()
        line["out_sha1"] = hashlib.sha1(o.tobytes()).hexdigest()[:16]
    if do_cpu and prec == "fp16":
        cms, thr = cpu_torch_baseline(cfg, w, ids, tt, cu, head,
                                      budget=float(os.environ.get("CPU_BUDGET", "5")))
        line["cpu_torch_fp32_ms"] = round(cms, 1)
        line["cpu_threads"] = thr
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
