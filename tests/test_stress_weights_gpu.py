"""Encoder parity on realistic weight statistics: the "stress" profile of
ragmi.synth.make_weights — heavy-tailed matrices, three outlier hidden dimensions with
LayerNorm gammas 8-20 and output biases of 20-50 that push post-LN hidden states to
|x| ~ 100-400 — where the benign Gaussian fixtures never take the fp16 hi/lo planes or the
deferred-LayerNorm algebra (un-normalised residual planes, rstd (z W'^T - mean c1) + c2).

Bars (north_star / VERDICT): CE logits within 1e-3 and bge embeddings within 5e-5 of the
transformers fixture (tests/golden/bert_golden_stress.npz, full 12-layer bge-small and 6-layer
MiniLM shapes) and of the oracle, fp16x3, in EVERY fusion x deferred-LN mode; plus the static
fp16 range guard: weights that could overflow an fp16 plane are refused at create, and the
deferred path is refused where only its un-normalised planes could overflow — no forward
returns inf."""
import os

import numpy as np
import pytest

import bert_ref as R

pytestmark = pytest.mark.gpu

TOL = {"bge": 5e-5, "ce": 1e-3}
MODES = [(f, d) for f in (-1, 0, 1) for d in (-1, 0, 1)]


@pytest.fixture(scope="module")
def sg():
    from conftest import GOLDEN
    return dict(np.load(os.path.join(GOLDEN, "bert_golden_stress.npz")))


@pytest.fixture(scope="module")
def encs(gpu, sg):
    from ragmi.encoders import HEAD_CLS_L2, HEAD_POOLER_CLS, BertEncoder
    wb = R.make_weights(R.BGE_SMALL, int(sg["bge_seed"]), profile="stress")
    wc = R.make_weights(R.MINILM_CE, int(sg["ce_seed"]), profile="stress")
    eb = BertEncoder(R.BGE_SMALL, wb, HEAD_CLS_L2, gpu, "fp16x3")
    ec = BertEncoder(R.MINILM_CE, wc, HEAD_POOLER_CLS, gpu, "fp16x3")
    yield (eb, wb), (ec, wc)
    eb.close()
    ec.close()


def _set(enc, fusion, defer):
    enc.set_fusion(fusion)
    enc.set_defer_ln(defer)


def _maxd(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


def test_stress_bounds_allow_every_path(encs):
    (eb, _), (ec, _) = encs
    for enc in (eb, ec):
        p, d = enc.range_bounds()
        assert 100 < p < 60000 and p <= d < 60000


@pytest.mark.parametrize("fusion,defer", MODES)
def test_stress_golden_every_mode(encs, sg, fusion, defer):
    (eb, _), (ec, _) = encs
    try:
        _set(eb, fusion, defer)
        _set(ec, fusion, defer)
        e = eb.forward_padded(sg["ids_q"], sg["tt_q"], sg["m_q"]).cpu().numpy()
        c = ec.forward_padded(sg["ids_p"], sg["tt_p"], sg["m_p"]).cpu().numpy()
    finally:
        _set(eb, -1, -1)
        _set(ec, -1, -1)
    de, dc = _maxd(e, sg["bge_emb"]), _maxd(c, sg["ce_logits"])
    print(f"stress fusion={fusion} defer={defer}: bge {de:.2e} ce {dc:.2e}")
    assert np.isfinite(e).all() and np.isfinite(c).all()
    assert de <= TOL["bge"] and dc <= TOL["ce"]


@pytest.fixture(scope="module")
def big_batches():
    """Token counts where AUTO takes the WS GEMMs and the deferred LayerNorm (>= ~11K tokens):
    48 rerank pairs of 200-260 tokens, 48 chunks of 200-260 tokens (ingest's /embed shape)."""
    rng = np.random.default_rng(77)

    def batch(n, pair):
        lens = rng.integers(200, 261, n)
        lens[0] = 260
        ids = np.zeros((n, 260), np.int64)
        tt, m = np.zeros_like(ids), np.zeros_like(ids)
        for b, L in enumerate(lens):
            t = rng.integers(1000, 30522, L)
            t[0], t[L - 1] = 101, 102
            if pair:
                cut = int(rng.integers(8, 40))              # [CLS] query [SEP] chunk [SEP]
                t[cut] = 102
                tt[b, cut + 1:L] = 1
            ids[b, :L] = t
            m[b, :L] = 1
        return ids, tt, m
    return batch(48, True), batch(48, False)


def test_stress_large_batches_vs_oracle_every_mode(encs, big_batches):
    (eb, wb), (ec, wc) = encs
    (pi, pt, pm), (ci, ct, cm) = big_batches
    ref_c = R.ce_logits(wc, R.MINILM_CE, pi, pt, pm)
    ref_e = R.bge_embed(wb, R.BGE_SMALL, ci, ct, cm)
    worst = {}
    try:
        for fusion, defer in MODES:
            _set(eb, fusion, defer)
            _set(ec, fusion, defer)
            c = ec.forward_padded(pi, pt, pm).cpu().numpy()
            e = eb.forward_padded(ci, ct, cm).cpu().numpy()
            assert np.isfinite(c).all() and np.isfinite(e).all()
            worst[(fusion, defer)] = (_maxd(c, ref_c), _maxd(e, ref_e))
    finally:
        _set(eb, -1, -1)
        _set(ec, -1, -1)
    for k, (dc, de) in worst.items():
        print(f"stress 48x~230 fusion={k[0]} defer={k[1]}: ce {dc:.2e} bge {de:.2e}")
    assert max(v[0] for v in worst.values()) <= TOL["ce"]
    assert max(v[1] for v in worst.values()) <= TOL["bge"]
    # the rerank order the reference returns (main.py:246) where the oracle separates scores
    c = ec.forward_padded(pi[:15], pt[:15], pm[:15]).cpu().numpy()
    srt = np.sort(ref_c[:15])[::-1]
    if np.min(np.abs(np.diff(srt[:6]))) > 2 * TOL["ce"]:
        np.testing.assert_array_equal(R.rerank_order(c, 5), R.rerank_order(ref_c[:15], 5))


def test_range_guard_refuses_overflowing_weights(gpu):
    """gamma 4000: an LN output can reach 4000 sqrt(383) ~ 78K > 65504 -> create refuses
    (RAG_ERANGE) instead of ever returning inf."""
    from ragmi._lib import RagmiError
    from ragmi.encoders import HEAD_CLS_L2, BertEncoder
    cfg = dict(R.BGE_SMALL, layers=2)
    w = R.make_weights(cfg, 3)
    w["encoder.layer.0.attention.output.LayerNorm.weight"][7] = 4000.0
    with pytest.raises(RagmiError) as e:
        BertEncoder(cfg, w, HEAD_CLS_L2, gpu, "fp16x3")
    assert e.value.code == -4 and "65504" in str(e.value)


def test_range_guard_keeps_deferred_ln_off(gpu):
    """An FFN2 bias of 1e5 only threatens the deferred path's un-normalised residual planes:
    AUTO never defers, forcing it fails, and the (plain) forward matches the oracle."""
    from ragmi._lib import RagmiError
    from ragmi.encoders import HEAD_POOLER_CLS, BertEncoder
    cfg = dict(R.MINILM_CE, layers=2)
    w = R.make_weights(cfg, 4)
    w["encoder.layer.0.output.dense.bias"][5] = 1e5
    enc = BertEncoder(cfg, w, HEAD_POOLER_CLS, gpu, "fp16x3")
    try:
        p, d = enc.range_bounds()
        assert p < 60000 < d
        with pytest.raises(RagmiError) as e:
            enc.set_defer_ln(1)
        assert e.value.code == -4
        rng = np.random.default_rng(8)
        ids, tt, m = R.random_batch(rng, 48, 260, pair=True)    # AUTO-defer size
        out = enc.forward_padded(ids, tt, m).cpu().numpy()
        ref = R.ce_logits(w, cfg, ids, tt, m)
        assert np.isfinite(out).all()
        assert _maxd(out, ref) <= TOL["ce"]
    finally:
        enc.close()
