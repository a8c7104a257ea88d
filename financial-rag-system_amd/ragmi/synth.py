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


def make_weights(cfg: dict, seed: int, profile: str = "benign") -> dict:
    """Seeded synthetic weights with HF state-dict names (BertModel prefix 'bert.' omitted).

    profile "benign" (round 1/2 fixtures): Gaussian matrices std 0.05, LayerNorm gammas
    1 +- 0.05. profile "stress": the statistics real BERT checkpoints are known to carry and
    the benign ones lack, to exercise the fp16 hi/lo planes and the deferred-LayerNorm
    algebra where they are weakest:
      * heavy-tailed matrices and embeddings (Student-t, 3 degrees of freedom, scaled to the
        same std: occasional entries at 10-20 sigma);
      * a few OUTLIER hidden dimensions (3 per model, the same in every layer): LayerNorm
        gammas 8-20 and betas +-3 there, and output-projection biases of +-20-50 that drive
        the pre-LayerNorm residual of those dimensions to hundreds ("massive activations"),
        so post-LN hidden states reach |x| ~ 100-400;
      * the other gammas 1 +- 0.15 (|.|), betas std 0.1."""
    rng = np.random.default_rng(seed)
    H, I = cfg["hidden"], cfg["inter"]
    stress = profile == "stress"
    if profile not in ("benign", "stress"):
        raise ValueError(f"unknown weight profile {profile!r}")
    out_dims = rng.choice(H, 3, replace=False) if stress else np.zeros(0, np.int64)

    def n(*shape, std=0.02):
        if stress:
            return (rng.standard_t(3, shape) * (std / np.sqrt(3.0))).astype(np.float32)
        return (rng.standard_normal(shape) * std).astype(np.float32)

    def gamma():
        if not stress:
            return 1.0 + n(H, std=0.05)
        g = np.abs(1.0 + 0.15 * rng.standard_normal(H))
        g[out_dims] = rng.uniform(8.0, 20.0, len(out_dims))
        return g.astype(np.float32)

    def beta():
        if not stress:
            return n(H)
        b = (0.1 * rng.standard_normal(H))
        b[out_dims] = rng.choice([-3.0, 3.0], len(out_dims))
        return b.astype(np.float32)

    def out_bias():
        b = n(H)
        if stress:
            b[out_dims] = rng.choice([-1.0, 1.0], len(out_dims)) * rng.uniform(20, 50, len(out_dims))
        return b

    w = {
        "embeddings.word_embeddings.weight": n(cfg["vocab"], H),
        "embeddings.position_embeddings.weight": n(cfg["max_pos"], H),
        "embeddings.token_type_embeddings.weight": n(cfg["type_vocab"], H),
        "embeddings.LayerNorm.weight": gamma(),
        "embeddings.LayerNorm.bias": beta(),
    }
    for l in range(cfg["layers"]):
        p = f"encoder.layer.{l}."
        for name, (o, i) in {"attention.self.query": (H, H), "attention.self.key": (H, H),
                             "attention.self.value": (H, H), "attention.output.dense": (H, H),
                             "intermediate.dense": (I, H), "output.dense": (H, I)}.items():
            w[p + name + ".weight"] = n(o, i, std=0.05)
            w[p + name + ".bias"] = (out_bias() if name in ("attention.output.dense",
                                                            "output.dense") else n(o))
        for ln in ("attention.output.LayerNorm", "output.LayerNorm"):
            w[p + ln + ".weight"] = gamma()
            w[p + ln + ".bias"] = beta()
    if cfg.get("pooler"):
        # stress: a smaller pooler scale keeps tanh off saturation with |CLS| ~ 100s (the
        # logits then still separate pairs)
        w["pooler.dense.weight"] = n(H, H, std=0.005 if stress else 0.05)
        w["pooler.dense.bias"] = n(H)
        w["classifier.weight"] = n(cfg.get("num_labels", 1), H, std=0.5)
        w["classifier.bias"] = n(cfg.get("num_labels", 1), std=0.5)
    return w


def write_checkpoint(d: str, cfg: dict, w: dict, vocab: list[str], kind: str) -> str:
    """A local checkpoint directory in the layout of the real ones (the hub cannot be reached):
    config.json + model.safetensors + vocab.txt, plus for kind "bge" bge-small-en-v1.5's
    sentence-transformers stack (modules.json: Transformer -> Pooling(cls) -> Normalize) and
    for kind "ce" ms-marco-MiniLM-L-6-v2's one-label head with its configured Identity
    activation (raw logits)."""
    import json
    import os

    from safetensors.numpy import save_file
    os.makedirs(d, exist_ok=True)
    save_file(w, os.path.join(d, "model.safetensors"))
    hf = {"model_type": "bert", "vocab_size": cfg["vocab"], "hidden_size": cfg["hidden"],
          "num_hidden_layers": cfg["layers"], "num_attention_heads": cfg["heads"],
          "intermediate_size": cfg["inter"], "max_position_embeddings": cfg["max_pos"],
          "type_vocab_size": cfg["type_vocab"], "layer_norm_eps": cfg["eps"],
          "hidden_act": "gelu", "position_embedding_type": "absolute"}
    if kind == "ce":
        hf.update(id2label={"0": "LABEL_0"}, label2id={"LABEL_0": 0},
                  sbert_ce_default_activation_function="torch.nn.modules.linear.Identity")
    elif kind == "bge":
        mods = [{"idx": 0, "name": "0", "path": "", "type": "sentence_transformers.models.Transformer"},
                {"idx": 1, "name": "1", "path": "1_Pooling", "type": "sentence_transformers.models.Pooling"},
                {"idx": 2, "name": "2", "path": "2_Normalize", "type": "sentence_transformers.models.Normalize"}]
        with open(os.path.join(d, "modules.json"), "w") as f:
            json.dump(mods, f)
        os.makedirs(os.path.join(d, "1_Pooling"), exist_ok=True)
        with open(os.path.join(d, "1_Pooling", "config.json"), "w") as f:
            json.dump({"word_embedding_dimension": cfg["hidden"], "pooling_mode_cls_token": True,
                       "pooling_mode_mean_tokens": False, "pooling_mode_max_tokens": False,
                       "pooling_mode_mean_sqrt_len_tokens": False}, f)
    else:
        raise ValueError(kind)
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(hf, f)
    with open(os.path.join(d, "vocab.txt"), "w") as f:
        f.write("\n".join(vocab) + "\n")
    return d


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


# ------------------------------------------------------------------ synthetic text
_SYL = ("ka re to mi na lo su de pa ri ve no ta li mo ra se di ne po ba cu fi ga he "
        "ju ko lu ma ni ou pe qu ro si tu va wo xe yo ze an er in on ul st th ch sh").split()


def make_vocab(size: int = 30522, seed: int = 0) -> list[str]:
    """A BERT-layout WordPiece vocab of `size` entries (the real bge / MiniLM vocab.txt is not
    on disk): [PAD], [unused0-98], [UNK], [CLS], [SEP], [MASK] at ids 0 / 1-99 / 100-103,
    single characters and their ## continuations, then seeded syllable words and ## suffix
    pieces — so WordPiece sees whole words, split words and unknown characters."""
    rng = np.random.default_rng(seed)
    v = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    chars = [chr(c) for c in range(ord("a"), ord("z") + 1)] + list("0123456789") + list(".,?$%-'")
    v += chars + ["##" + c for c in chars if c.isalnum()]
    seen = set(v)
    while len(v) < size:
        w = "".join(rng.choice(_SYL, int(rng.integers(1, 4))))
        if rng.random() < 0.2:
            w = "##" + w
        if w not in seen:
            seen.add(w)
            v.append(w)
    return v[:size]


def query_texts(rng, vocab: list[str], n: int, min_words: int = 8, max_words: int = 18) -> list[str]:
    """n question-like strings: whole vocab words, some glued to a ## piece (split by WordPiece
    into two tokens), some digits and punctuation; ~16-32 WordPiece tokens each, the length of
    the reference's user questions (load_testing.py's AAPL queries)."""
    words = [w for w in vocab[104:] if not w.startswith("##") and len(w) > 1]
    pieces = [w[2:] for w in vocab[104:] if w.startswith("##") and len(w) > 3]
    out = []
    for _ in range(n):
        k = int(rng.integers(min_words, max_words + 1))
        ws = []
        for _ in range(k):
            w = words[int(rng.integers(len(words)))]
            r = rng.random()
            if r < 0.2:
                w = w + pieces[int(rng.integers(len(pieces)))]
            elif r < 0.25:
                w = str(int(rng.integers(1990, 2030)))
            ws.append(w)
        out.append(" ".join(ws).capitalize() + "?")
    return out
