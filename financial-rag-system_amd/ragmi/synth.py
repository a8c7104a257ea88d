"""ragmi.synth — synthetic benchmark inputs for the encoders: the three model shapes on the
path and seeded random weights / token batches of exactly those shapes (the real checkpoints
are not on disk: SURVEY §8c). Data generation only — no arithmetic of the path lives here;
oracle/bert_ref.py re-exports these so tests, fixtures and benches share one generator.

Shapes: bge-small-en-v1.5 (reference main.py:80-84, 211-213), bge-large-en-v1.5 (SURVEY §8f
row 4, config 5), cross-encoder/ms-marco-MiniLM-L-6-v2 (main.py:86-90).
"""
from __future__ import annotations

import numpy as np

BGE_SMALL = dict(vocab=30522, hidden=384, layers=12, heads=12, inter=1536, max_pos=512,
                 type_vocab=2, eps=1e-12, pooler=False)
# bge-large-en-v1.5 shape (1024-d vectors)
BGE_LARGE = dict(vocab=30522, hidden=1024, layers=24, heads=16, inter=4096, max_pos=512,
                 type_vocab=2, eps=1e-12, pooler=False)
MINILM_CE = dict(vocab=30522, hidden=384, layers=6, heads=12, inter=1536, max_pos=512,
                 type_vocab=2, eps=1e-12, pooler=True, num_labels=1)


def make_weights(cfg: dict, seed: int) -> dict:
    """Seeded synthetic weights with HF state-dict names (BertModel prefix 'bert.' omitted)."""
    rng = np.random.default_rng(seed)
    H, I = cfg["hidden"], cfg["inter"]

    def n(*shape, std=0.02):
        return (rng.standard_normal(shape) * std).astype(np.float32)

    w = {
        "embeddings.word_embeddings.weight": n(cfg["vocab"], H),
        "embeddings.position_embeddings.weight": n(cfg["max_pos"], H),
        "embeddings.token_type_embeddings.weight": n(cfg["type_vocab"], H),
        "embeddings.LayerNorm.weight": 1.0 + n(H, std=0.05),
        "embeddings.LayerNorm.bias": n(H),
    }
    for l in range(cfg["layers"]):
        p = f"encoder.layer.{l}."
        for name, (o, i) in {"attention.self.query": (H, H), "attention.self.key": (H, H),
                             "attention.self.value": (H, H), "attention.output.dense": (H, H),
                             "intermediate.dense": (I, H), "output.dense": (H, I)}.items():
            w[p + name + ".weight"] = n(o, i, std=0.05)
            w[p + name + ".bias"] = n(o)
        for ln in ("attention.output.LayerNorm", "output.LayerNorm"):
            w[p + ln + ".weight"] = 1.0 + n(H, std=0.05)
            w[p + ln + ".bias"] = n(H)
    if cfg.get("pooler"):
        w["pooler.dense.weight"] = n(H, H, std=0.05)
        w["pooler.dense.bias"] = n(H)
        w["classifier.weight"] = n(cfg.get("num_labels", 1), H, std=0.5)
        w["classifier.bias"] = n(cfg.get("num_labels", 1), std=0.5)
    return w


def random_batch(rng, B, max_len, pair=False, vocab=30522):
    """Token ids with [CLS]=101 ... [SEP]=102 (pairs: [CLS] a [SEP] b [SEP], type 0/1),
    right padding with 0, like a BERT tokenizer padded to the longest sequence."""
    lens = rng.integers(3, max_len + 1, B)
    lens[0] = max_len
    S = int(lens.max())
    ids = np.zeros((B, S), np.int64)
    tt = np.zeros((B, S), np.int64)
    mask = np.zeros((B, S), np.int64)
    for b, L in enumerate(lens):
        t = rng.integers(1000, vocab, L)
        t[0] = 101
        t[L - 1] = 102
        if pair and L >= 5:
            cut = int(rng.integers(2, L - 2))
            t[cut] = 102
            tt[b, cut + 1:L] = 1
        ids[b, :L] = t
        mask[b, :L] = 1
    return ids, tt, mask
