"""Precision emulation for VERDICT r3 item 1(c): fp16 main product + block-scaled fp8 correction
terms for the cross-encoder GEMMs. Would

    y = A_hi W_hi^T + [A_hi8 | A_lo8] [W_lo8 ; W_hi8]^T     (one fp16 MFMA + one fp8 MFMA over
                                                             concatenated K, v_mfma_scale_f32_*_f8f6f4)

keep the CE logits within the 1e-3 contract? A_hi = fp16(A), A_lo = A - A_hi (W likewise); X8 =
OCP e4m3 with one power-of-two scale per 32 consecutive K elements (MX block scaling; scale
2^(floor(log2 amax) - 7), so no element saturates). Activations are stored the same way
(hi fp16 + lo e4m3 block-scaled), modelled by rounding every GEMM input to hi + Q8(lo).
oracle/bert_ref.py's forward runs with its Linear layers of the 6 encoder layers replaced
(pooler / classifier exact), on 24 pairs of ~288 tokens, benign and stress weights; prints
max |logit - fp32 logit| against fp16x3's own (measured 2-3e-5 on the GPU).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bert_ref as R  # noqa: E402


def e4m3(v):
    """Round-to-nearest-even onto OCP e4m3 (|v| <= 448 assumed; subnormal step 2^-9)."""
    a = np.abs(v).astype(np.float64)
    e = np.floor(np.log2(np.where(a > 0, a, 1.0)))
    e = np.maximum(e, -6.0)
    step = np.exp2(e - 3.0)
    q = np.round(a / step) * step          # numpy rounds half to even
    return (np.sign(v) * np.minimum(q, 448.0)).astype(np.float64)


def q8(x, block=32):
    """MX-style block-scaled e4m3 along the last axis (blocks of 32)."""
    shp = x.shape
    K = shp[-1]
    xb = x.reshape(-1, K // block, block).astype(np.float64)
    amax = np.abs(xb).max(-1, keepdims=True)
    sc = np.exp2(np.floor(np.log2(np.where(amax > 0, amax, 1.0))) - 7.0)
    return (e4m3(xb / sc) * sc).reshape(shp)


def split(x):
    hi = x.astype(np.float16).astype(np.float64)
    return hi, x.astype(np.float64) - hi


def lin_fp8corr(x, w, b):
    xh, xl = split(x)
    xl = q8(xl)                            # stored activation: hi fp16 + lo e4m3 (scaled)
    wh, wl = split(w)
    y = xh @ wh.T + q8(xh) @ q8(wl).T + q8(xl) @ q8(wh).T
    return (y + b).astype(np.float32)


def lin_fp16x3(x, w, b):
    xh, xl = split(x)
    xl = xl.astype(np.float16).astype(np.float64)
    wh, wl = split(w)
    wl = wl.astype(np.float16).astype(np.float64)
    return (xh @ wh.T + xh @ wl.T + xl @ wh.T + b).astype(np.float32)


def ce(w, ids, tt, m, lin):
    orig = R._lin
    R._lin = lin
    try:
        cls = R.bert_forward(w, R.MINILM_CE, ids, tt, m)[:, 0]
    finally:
        R._lin = orig
    pooled = np.tanh(R._lin(cls, w["pooler.dense.weight"], w["pooler.dense.bias"]))
    return R._lin(pooled, w["classifier.weight"], w["classifier.bias"])[:, 0]


def main():
    rng = np.random.default_rng(1)
    ids, tt, m = R.random_batch(rng, 24, 288, pair=True)
    for prof, seed in (("benign", 2), ("stress", 42)):
        w = R.make_weights(R.MINILM_CE, seed, profile=prof)
        ref = R.ce_logits(w, R.MINILM_CE, ids, tt, m)
        for name, lin in (("fp16x3", lin_fp16x3), ("fp16 + fp8 corrections", lin_fp8corr)):
            d = np.abs(ce(w, ids, tt, m, lin) - ref).max()
            print(f"{prof:6s} CE {name:24s}: max|d logit| {d:.2e} "
                  f"({'ok' if d <= 1e-3 else 'FAILS'} vs 1e-3)", flush=True)


if __name__ == "__main__":
    main()
