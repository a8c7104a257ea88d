"""Precision emulations for the rerank GEMMs: would a 2-product split
with W as ONE fp16 plane (a_hi w16 + a_lo w16 — exact activations, weights rounded to fp16;
2 MFMAs per product instead of fp16x3's 3, and half the W bytes) keep the cross-encoder logits
within the 1e-3 contract?

oracle/bert_ref.py's fp32 forward is run with the 2-D weight matrices rounded to fp16 — all
of them, then one GEMM kind at a time — on 24 pairs of ~288 tokens, for the benign and the
stress weight profiles (ragmi.synth). Rounding W is exactly what the
2-product split computes up to fp32 accumulation order. Prints max |logit - fp32 logit|
(and max |embedding - fp32| for bge-small). Result in DESIGN.md §R3: every variant fails the
CE bar on at least one profile, so fp16x3 stays.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bert_ref as R  # noqa: E402

PARTS = {"qkv": ("attention.self.query", "attention.self.key", "attention.self.value"),
         "o_proj": ("attention.output.dense",),
         "ffn1": ("intermediate.dense",),
         "ffn2": ("output.dense",)}


def rounded(w, which):
    out = {}
    for k, v in w.items():
        hit = v.ndim == 2 and "embeddings" not in k and k.startswith("encoder.layer.")
        if hit and which != "all":
            stem = k.split(".", 3)[3].rsplit(".", 1)[0]     # e.g. attention.self.query
            hit = stem in PARTS[which] and not (which == "ffn2" and stem.startswith("attention"))
        out[k] = v.astype(np.float16).astype(np.float32) if hit else v
    return out


def main():
    rng = np.random.default_rng(1)
    ids, tt, m = R.random_batch(rng, 24, 288, pair=True)
    for prof, seed in (("benign", 2), ("stress", 42)):
        w = R.make_weights(R.MINILM_CE, seed, profile=prof)
        ref = R.ce_logits(w, R.MINILM_CE, ids, tt, m)
        for which in ("all",) + tuple(PARTS):
            d = np.abs(R.ce_logits(rounded(w, which), R.MINILM_CE, ids, tt, m) - ref).max()
            print(f"{prof:6s} CE  W fp16 [{which:6s}]: max|d logit| {d:.2e} "
                  f"({'ok' if d <= 1e-3 else 'FAILS'} vs 1e-3)", flush=True)
        wb = R.make_weights(R.BGE_SMALL, seed, profile=prof)
        refb = R.bge_embed(wb, R.BGE_SMALL, ids, tt, m)
        d = np.abs(R.bge_embed(rounded(wb, "all"), R.BGE_SMALL, ids, tt, m) - refb).max()
        print(f"{prof:6s} bge W fp16 [all   ]: max|d emb| {d:.2e} "
              f"({'ok' if d <= 5e-5 else 'FAILS'} vs 5e-5)", flush=True)


if __name__ == "__main__":
    main()
