"""CPU tests pinning the encoder oracle (oracle/bert_ref.py) against transformers' BertModel /
BertForSequenceClassification (committed fixtures made by tests/golden/make_golden_bert.py,
plus a live re-check when transformers is importable)."""
import numpy as np
import pytest

import bert_ref as R


@pytest.fixture(scope="module")
def golden():
    import os
    from conftest import GOLDEN
    return dict(np.load(os.path.join(GOLDEN, "bert_golden.npz")))


def test_bge_oracle_matches_transformers_fixture(golden):
    g = golden
    w = R.make_weights(R.BGE_SMALL, int(g["bge_seed"]))
    emb = R.bge_embed(w, R.BGE_SMALL, g["ids_q"], g["tt_q"], g["m_q"])
    np.testing.assert_allclose(emb, g["bge_emb"], rtol=0, atol=2e-6)
    np.testing.assert_allclose(np.linalg.norm(emb, axis=1), 1.0, atol=1e-6)


def test_ce_oracle_matches_transformers_fixture(golden):
    g = golden
    w = R.make_weights(R.MINILM_CE, int(g["ce_seed"]))
    lg = R.ce_logits(w, R.MINILM_CE, g["ids_p"], g["tt_p"], g["m_p"])
    np.testing.assert_allclose(lg, g["ce_logits"], rtol=0, atol=2e-5)


def test_bge_large_shape_oracle_matches_transformers_fixture(golden):
    """bge-large shape (hidden 1024, 16 heads x 64, FFN 4096; 2 of 24 layers), config 5."""
    g = golden
    cfg = dict(R.BGE_LARGE, layers=2)
    w = R.make_weights(cfg, int(g["bgel_seed"]))
    emb = R.bge_embed(w, cfg, g["ids_l"], g["tt_l"], g["m_l"])
    np.testing.assert_allclose(emb, g["bgel_emb"], rtol=0, atol=2e-6)


def test_padding_does_not_change_valid_outputs(golden):
    """Right padding to a longer batch length leaves every sequence's output unchanged
    (what lets the HIP path pack sequences without padding)."""
    g = golden
    w = R.make_weights(R.MINILM_CE, int(g["ce_seed"]))
    ids, tt, m = g["ids_p"], g["tt_p"], g["m_p"]
    pad = lambda a: np.concatenate([a, np.zeros((a.shape[0], 7), a.dtype)], 1)
    a = R.ce_logits(w, R.MINILM_CE, ids, tt, m)
    b = R.ce_logits(w, R.MINILM_CE, pad(ids), pad(tt), pad(m))
    np.testing.assert_allclose(a, b, rtol=0, atol=1e-5)


def test_rerank_order_is_reference_argsort():
    s = np.array([0.3, -1.0, 2.5, 0.3, 7.0], np.float32)
    np.testing.assert_array_equal(R.rerank_order(s, 3), np.argsort(s)[::-1][:3])
    assert list(R.rerank_order(s, 10)) == [4, 2, 3, 0, 1]


def test_live_transformers_recheck():
    pytest.importorskip("transformers")
    import sys, os
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden_bert as M
    rng = np.random.default_rng(99)
    cfg = dict(R.MINILM_CE, layers=2)
    w = R.make_weights(cfg, 5)
    ids, tt, m = R.random_batch(rng, 3, 17, pair=True)
    np.testing.assert_allclose(R.ce_logits(w, cfg, ids, tt, m), M.hf_ce(cfg, w, ids, tt, m),
                               rtol=0, atol=2e-5)


def test_stress_oracle_matches_transformers_fixture():
    """The stress weight profile (outlier dimensions, |hidden| ~ 100-400): oracle vs the
    transformers 5.15 fixture (tests/golden/make_golden_bert.py main_stress)."""
    import os
    from conftest import GOLDEN
    g = dict(np.load(os.path.join(GOLDEN, "bert_golden_stress.npz")))
    wb = R.make_weights(R.BGE_SMALL, int(g["bge_seed"]), profile="stress")
    wc = R.make_weights(R.MINILM_CE, int(g["ce_seed"]), profile="stress")
    np.testing.assert_allclose(R.bge_embed(wb, R.BGE_SMALL, g["ids_q"], g["tt_q"], g["m_q"]),
                               g["bge_emb"], rtol=0, atol=3e-6)
    np.testing.assert_allclose(R.ce_logits(wc, R.MINILM_CE, g["ids_p"], g["tt_p"], g["m_p"]),
                               g["ce_logits"], rtol=0, atol=2e-5)
