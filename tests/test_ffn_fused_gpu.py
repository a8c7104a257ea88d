"""The fused deferred-LayerNorm FFN (round 6, VERDICT r5 item 1: bert_kernels.hip
ffn_fused_kernel, rag_encoder_set_ffn_fused): FFN1 + GELU + FFN2 + residual + LayerNorm
statistics in one launch per layer, the 1536-wide intermediate kept on the CU.

Bar: BITWISE. Every output element is computed with the MFMA sequence, epilogue arithmetic and
operand-to-lane mapping of the two-GEMM path (gemm_ws_kernel FFN1 / FFN2 at >= 64 row panels,
natural K order), so with the same weights and tokens the forward's outputs — cross-encoder
logits (modeling_bert.py BertForSequenceClassification head) and bge-small embeddings —
must equal the two-kernel forward's bit for bit, at token counts that leave a ragged last
128-row tile. Below 16,384 tokens the WS GEMMs rotate their K order, so there the fused
forward is held to the fp16x3 oracle bounds of test_config3_gpu.py instead (oracle/bert_ref.py:
logits 1e-4, embeddings 5e-6), on the benign and the stress weight profiles.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# the fused FFN is compiled into the diagnostic build only (measured slower):
# run with RAGMI_LIB_AB=<build with -DRAGMI_DIAG_BUILD> RAGMI_TEST_DIAG_BUILD=1
DIAG = os.environ.get("RAGMI_TEST_DIAG_BUILD") == "1"


def _packed(rng, n, lo, hi, pair=False):
    lens = rng.integers(lo, hi, n)
    ids = np.concatenate([np.r_[101, rng.integers(1000, 30000, L - 2), 102] for L in lens])
    types = np.zeros(len(ids), np.int32)
    if pair:
        cu = np.r_[0, np.cumsum(lens)]
        for a, b in zip(cu[:-1], cu[1:]):
            types[a + (b - a) // 2:b] = 1
    return ids.astype(np.int32), types, np.r_[0, np.cumsum(lens)].astype(np.int32)


def _enc(gpu, model, profile="benign", seed=7):
    import bert_ref as R
    from ragmi.encoders import HEAD_CLS_L2, HEAD_POOLER_CLS, BertEncoder
    cfg, head = (R.MINILM_CE, HEAD_POOLER_CLS) if model == "ce" else (R.BGE_SMALL, HEAD_CLS_L2)
    w = R.make_weights(cfg, seed, profile=profile)
    return BertEncoder(cfg, w, head, gpu, "fp16x3"), w, cfg


def _both(enc, ids, types, cu, modes=(0, 1, 2, 3, 4, 5)):
    """forward outputs with the fused FFN off (0), on with the 3-slot ring (1) and on with the
    5-slot ring (2, rag_encoder_set_ffn_fused's A/B shape)"""
    outs = {}
    try:
        for mode in modes:
            enc.set_ffn_fused(mode)
            outs[mode] = enc.forward_packed(ids, types, cu).cpu().numpy()
    finally:
        enc.set_ffn_fused(-1)
    return outs


if DIAG:
    @pytest.mark.parametrize("model,n,lo,hi,seed", [("ce", 80, 180, 289, 1), ("ce", 123, 150, 260, 2),
                                                    ("bge", 80, 200, 261, 3)])
    def test_fused_ffn_is_bitwise_the_two_kernel_forward(gpu, model, n, lo, hi, seed):
        """>= 16,384 tokens (deferred LayerNorm on by AUTO), ragged last tile: bit for bit."""
        rng = np.random.default_rng(100 + seed)
        ids, types, cu = _packed(rng, n, lo, hi, pair=model == "ce")
        assert cu[-1] >= 16384 and cu[-1] % 128
        enc, _, _ = _enc(gpu, model, seed=seed)
        try:
            enc.set_defer_ln(1)
            outs = _both(enc, ids, types, cu)
            for m in (1, 2, 3, 4, 5):
                d = np.abs(outs[m] - outs[0]).max()
                print(f"[{model} T={cu[-1]} ring {m}] max |fused - two-kernel| = {d:.3e}")
                assert np.array_equal(outs[m].view(np.uint32), outs[0].view(np.uint32))
        finally:
            enc.set_defer_ln(-1)
            enc.close()


    @pytest.mark.parametrize("model,profile", [("ce", "benign"), ("ce", "stress"), ("bge", "benign"),
                                               ("bge", "stress")])
    def test_fused_ffn_small_batches_vs_oracle(gpu, model, profile):
        """Small batches (deferred LayerNorm and the fused FFN forced on; one or two 128-row tiles
        per CU at most, a tile of fewer than 128 rows) against oracle/bert_ref.py."""
        import bert_ref as R
        from test_config3_gpu import _oracle
        rng = np.random.default_rng(7 if model == "ce" else 8)
        if model == "ce":
            ids, types, cu = _packed(rng, 24, 60, 300, pair=True)
            fn, tol = R.ce_logits, (1e-4 if profile == "benign" else 1e-3)
        else:
            ids, types, cu = _packed(rng, 20, 8, 260)
            fn, tol = R.bge_embed, 5e-6 if profile == "benign" else 5e-5
        enc, w, cfg = _enc(gpu, model, profile, seed=11)
        ref = _oracle(fn, w, cfg, ids, types, cu)
        try:
            enc.set_defer_ln(1)
            outs = _both(enc, ids, types, cu)
            for mode in (0, 1, 2):
                d = np.abs(outs[mode] - ref).max()
                print(f"[{model}/{profile} fused={mode}] max |d| vs oracle = {d:.3e}")
                assert d <= tol
            assert np.abs(outs[1] - outs[0]).max() <= tol
            assert np.array_equal(outs[1], outs[2])
        finally:
            enc.set_defer_ln(-1)
            enc.close()


def test_fused_ffn_modes(gpu):
    """The production library refuses the fused modes (diagnostic build only); -1 / 0 pass."""
    from ragmi._lib import RagmiError
    enc, _, _ = _enc(gpu, "ce")
    try:
        enc.set_ffn_fused(0)
        enc.set_ffn_fused(-1)
        with pytest.raises(RagmiError):
            enc.set_ffn_fused(6)
        if not DIAG:
            with pytest.raises(RagmiError, match="diagnostic build"):
                enc.set_ffn_fused(1)
    finally:
        enc.close()
