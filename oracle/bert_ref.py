"""oracle/bert_ref.py — numpy fp32 restatement of the two encoders on the hot path.

TEST INFRASTRUCTURE ONLY (imported by tests/, __graft_entry__.smoke() and bench.py's checker
legs). The product encoders are the HIP kernels in financial-rag-system_amd/csrc.

Restates, for the reference's models:
  * bge-small-en-v1.5 via sentence-transformers `SentenceTransformer.encode` (reference
    main.py:80-84, 211-213; main2.py:88-96, 170-171): BertModel (12 layers) -> CLS pooling ->
    L2 normalise ([external] bge modules.json: Transformer -> Pooling(cls) -> Normalize).
  * cross-encoder/ms-marco-MiniLM-L-6-v2 via `CrossEncoder.predict` (main.py:86-90, 241-247):
    BertForSequenceClassification (6 layers, num_labels=1) -> pooler tanh(W h_CLS + b) ->
    Linear(384 -> 1), identity activation (raw logits; frontend.py:112-117 applies its own
    sigmoid to the returned scores).
BertModel arithmetic follows the installed transformers 5.15.0 modeling_bert.py:
  embeddings word+type+position -> LayerNorm (:96-107); per layer Q/K/V Linear (:164-175),
  eager attention softmax(QK^T * d^-0.5 + additive mask) V (:111-135), output dense + residual +
  LayerNorm (:282-293), intermediate dense + erf-GELU (:325-337), output dense + residual +
  LayerNorm (:340-351); pooler (:451-463); sequence-classification head (:1072-1118).
Pinned against transformers itself by tests/test_oracle_bert.py (live, CPU) and the committed
fixtures tests/golden/bert_golden.npz (tests/golden/make_golden_bert.py). The real checkpoints
are not on disk, so weights are seeded synthetic ones of the exact shapes.
"""
from __future__ import annotations

import numpy as np
from scipy.special import erf

# model shapes and seeded synthetic weights / batches: shared with the benches
# (financial-rag-system_amd/ragmi/synth.py; data generation, not the restated arithmetic)
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                  "financial-rag-system_amd"))
from ragmi.synth import BGE_LARGE, BGE_SMALL, MINILM_CE, make_weights, random_batch  # noqa: E402,F401


def _ln(x, g, b, eps):
    mu = x.mean(-1, keepdims=True, dtype=np.float32)
    var = ((x - mu) ** 2).mean(-1, keepdims=True, dtype=np.float32)
    return ((x - mu) / np.sqrt(var + eps) * g + b).astype(np.float32)


def _lin(x, w, b):
    return (x @ w.T + b).astype(np.float32)


def bert_forward(w: dict, cfg: dict, ids: np.ndarray, type_ids: np.ndarray,
                 mask: np.ndarray) -> np.ndarray:
    """Last hidden state [B, S, H] fp32 of BertModel with right padding (mask 1 = token)."""
    B, S = ids.shape
    H, nh = cfg["hidden"], cfg["heads"]
    hd = H // nh
    x = (w["embeddings.word_embeddings.weight"][ids]
         + w["embeddings.token_type_embeddings.weight"][type_ids]
         + w["embeddings.position_embeddings.weight"][np.arange(S)][None]).astype(np.float32)
    x = _ln(x, w["embeddings.LayerNorm.weight"], w["embeddings.LayerNorm.bias"], cfg["eps"])
    add_mask = np.where(mask[:, None, None, :] > 0, 0.0,
                        np.finfo(np.float32).min).astype(np.float32)
    for l in range(cfg["layers"]):
        p = f"encoder.layer.{l}."

        def heads(t):
            return t.reshape(B, S, nh, hd).transpose(0, 2, 1, 3)

        q = heads(_lin(x, w[p + "attention.self.query.weight"], w[p + "attention.self.query.bias"]))
        k = heads(_lin(x, w[p + "attention.self.key.weight"], w[p + "attention.self.key.bias"]))
        v = heads(_lin(x, w[p + "attention.self.value.weight"], w[p + "attention.self.value.bias"]))
        sc = (q @ k.transpose(0, 1, 3, 2)) * np.float32(hd ** -0.5) + add_mask
        sc = sc - sc.max(-1, keepdims=True)
        e = np.exp(sc).astype(np.float32)
        pr = e / e.sum(-1, keepdims=True)
        ctx = (pr @ v).transpose(0, 2, 1, 3).reshape(B, S, H).astype(np.float32)
        a = _lin(ctx, w[p + "attention.output.dense.weight"], w[p + "attention.output.dense.bias"])
        x = _ln(a + x, w[p + "attention.output.LayerNorm.weight"],
                w[p + "attention.output.LayerNorm.bias"], cfg["eps"])
        h = _lin(x, w[p + "intermediate.dense.weight"], w[p + "intermediate.dense.bias"])
        h = (0.5 * h * (1.0 + erf(h / np.sqrt(2.0)))).astype(np.float32)
        o = _lin(h, w[p + "output.dense.weight"], w[p + "output.dense.bias"])
        x = _ln(o + x, w[p + "output.LayerNorm.weight"], w[p + "output.LayerNorm.bias"],
                cfg["eps"])
    return x


def bge_embed(w, cfg, ids, type_ids, mask) -> np.ndarray:
    """sentence-transformers bge: CLS pooling + F.normalize(p=2, eps=1e-12) -> [B, H]."""
    cls = bert_forward(w, cfg, ids, type_ids, mask)[:, 0]
    nrm = np.maximum(np.linalg.norm(cls.astype(np.float64), axis=1, keepdims=True), 1e-12)
    return (cls / nrm).astype(np.float32)


def ce_logits(w, cfg, ids, type_ids, mask) -> np.ndarray:
    """CrossEncoder (num_labels=1, identity activation): tanh pooler -> classifier -> [B]."""
    cls = bert_forward(w, cfg, ids, type_ids, mask)[:, 0]
    pooled = np.tanh(_lin(cls, w["pooler.dense.weight"], w["pooler.dense.bias"]))
    return _lin(pooled, w["classifier.weight"], w["classifier.bias"])[:, 0]


def rerank_order(scores: np.ndarray, top_k: int) -> np.ndarray:
    """main.py:246 `np.argsort(scores)[::-1][:top_k]` exactly (default quicksort)."""
    return np.argsort(scores)[::-1][:top_k]
