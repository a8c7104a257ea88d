"""Generate tests/golden/bert_golden.npz (and bert_golden_stress.npz) with the installed `transformers` (5.15.0) BERT
classes — the library the reference's sentence-transformers stack runs on — built from a
LOCAL config with the seeded synthetic weights of oracle/bert_ref.make_weights (no hub
access; the real checkpoints are not on disk).

Stored: input ids / token types / masks and, per model, the CLS-normalised bge embeddings
[B,384] and the cross-encoder logits [B] computed by transformers in fp32 (eager attention).
bert_golden_stress.npz: the same for the "stress" weight profile (ragmi.synth.make_weights:
heavy-tailed matrices, outlier hidden dimensions with LayerNorm gammas 8-20 and massive
pre-LN activations, |hidden| ~ 100-400) — full 12-layer bge-small and 6-layer MiniLM shapes.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bert_ref as R  # noqa: E402

BGE_LARGE_2L = dict(R.BGE_LARGE, layers=2)


def hf_model(cfg, w, seq_cls):
    from transformers import BertConfig, BertForSequenceClassification, BertModel
    c = BertConfig(vocab_size=cfg["vocab"], hidden_size=cfg["hidden"],
                   num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"],
                   intermediate_size=cfg["inter"], max_position_embeddings=cfg["max_pos"],
                   type_vocab_size=cfg["type_vocab"], layer_norm_eps=cfg["eps"],
                   hidden_act="gelu", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                   num_labels=1, attn_implementation="eager")
    m = (BertForSequenceClassification(c) if seq_cls else BertModel(c, add_pooling_layer=False))
    sd = {}
    for k, v in w.items():
        if seq_cls:
            sd[k if k.startswith("classifier") else "bert." + k] = torch.from_numpy(v)
        else:
            sd[k] = torch.from_numpy(v)
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if "position_ids" not in k and "token_type_ids" not in k]
    assert not missing and not unexpected, (missing, unexpected)
    return m.eval()


def hf_bge(cfg, w, ids, tt, mask):
    m = hf_model(cfg, w, False)
    with torch.no_grad():
        h = m(input_ids=torch.from_numpy(ids), token_type_ids=torch.from_numpy(tt),
              attention_mask=torch.from_numpy(mask)).last_hidden_state[:, 0]
        return torch.nn.functional.normalize(h, p=2, dim=1).numpy()


def hf_ce(cfg, w, ids, tt, mask):
    m = hf_model(cfg, w, True)
    with torch.no_grad():
        return m(input_ids=torch.from_numpy(ids), token_type_ids=torch.from_numpy(tt),
                 attention_mask=torch.from_numpy(mask)).logits[:, 0].numpy()


def main():
    torch.manual_seed(0)
    rng = np.random.default_rng(2024)
    ids_q, tt_q, m_q = R.random_batch(rng, 6, 24)
    ids_p, tt_p, m_p = R.random_batch(rng, 6, 40, pair=True)
    wb = R.make_weights(R.BGE_SMALL, seed=11)
    wc = R.make_weights(R.MINILM_CE, seed=12)
    emb = hf_bge(R.BGE_SMALL, wb, ids_q, tt_q, m_q)
    logit = hf_ce(R.MINILM_CE, wc, ids_p, tt_p, m_p)
    # bge-large shape (hidden 1024, 16 heads of 64, FFN 4096), 2 of its 24 layers: the layer
    # arithmetic is the same per layer, the fixture stays small
    ids_l, tt_l, m_l = R.random_batch(rng, 5, 30)
    wl = R.make_weights(BGE_LARGE_2L, seed=13)
    emb_l = hf_bge(BGE_LARGE_2L, wl, ids_l, tt_l, m_l)
    np.savez_compressed(os.path.join(HERE, "bert_golden.npz"), ids_q=ids_q, tt_q=tt_q, m_q=m_q,
                        ids_p=ids_p, tt_p=tt_p, m_p=m_p, bge_emb=emb, ce_logits=logit,
                        bge_seed=11, ce_seed=12, ids_l=ids_l, tt_l=tt_l, m_l=m_l,
                        bgel_emb=emb_l, bgel_seed=13)
    print("bge", emb.shape, "ce", logit, "bge-large-2L", emb_l.shape)
    main_stress()


def main_stress():
    torch.manual_seed(0)
    rng = np.random.default_rng(4048)
    ids_q, tt_q, m_q = R.random_batch(rng, 8, 32)
    ids_p, tt_p, m_p = R.random_batch(rng, 8, 96, pair=True)
    wb = R.make_weights(R.BGE_SMALL, seed=41, profile="stress")
    wc = R.make_weights(R.MINILM_CE, seed=42, profile="stress")
    emb = hf_bge(R.BGE_SMALL, wb, ids_q, tt_q, m_q)
    logit = hf_ce(R.MINILM_CE, wc, ids_p, tt_p, m_p)
    np.savez_compressed(os.path.join(HERE, "bert_golden_stress.npz"), ids_q=ids_q, tt_q=tt_q,
                        m_q=m_q, ids_p=ids_p, tt_p=tt_p, m_p=m_p, bge_emb=emb,
                        ce_logits=logit, bge_seed=41, ce_seed=42)
    print("stress: bge", emb.shape, "ce", logit)


if __name__ == "__main__":
    if sys.argv[1:] == ["stress"]:
        main_stress()
    else:
        main()
