"""GPU parity of the deferred LayerNorm (fp16x3, hidden 384): csrc/bert_kernels.hip DlArgs /
ws_dl_epilogue, C entries rag_bert_gemm_dl and rag_encoder_set_defer_ln (ragmi_bert.h).

The token rows' residual stream stays un-normalised between sublayers (z as fp16 hi + lo
planes + per-row {mean, M2} of six 64-column blocks); consumers fold the pending LayerNorm
(modeling_bert.py BertSelfOutput / BertOutput: LayerNorm(dense(h) + x)) into their epilogue:
  LN_F16 / LN_GELU_F16:  [gelu](LN(z) W^T + b) = [gelu](rstd (z W'^T - mean c1) + c2)
  RES_LN:                z' = (a W^T + b) + LN(z), with z' and its block stats written back.
Reference: float64 torch of the same formulas from the un-folded weights (LN over the whole
row, biased variance, eps inside the sqrt). Bounds (outputs ~N(0, 1)-scaled, as in
test_gemm_gpu.py's fp16x3 bound): |out - ref| <= 3e-5 + 3e-6 |ref|; block stats: means within
2e-6 absolute, M2 within 1e-5 relative. Encoder level: the MiniLM cross-encoder and bge-small
forwards with the deferred path forced on at small batches, against oracle/bert_ref.py at the
fp16x3 bounds of test_config3_gpu.py (logits 1e-4, embeddings 5e-6) and against the
non-deferred forward.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H = 384


def _split(x32):
    h = x32.half()
    return h, (x32 - h.float()).half()


def _stats(z64):
    b = z64.view(z64.shape[0], H // 64, 64)
    m = b.mean(-1)
    return torch.stack([m, ((b - m[..., None]) ** 2).sum(-1)], -1)


def _ln(z64, gamma, beta, eps):
    mu = z64.mean(1, keepdim=True)
    var = ((z64 - mu) ** 2).mean(1, keepdim=True)
    return (z64 - mu) / torch.sqrt(var + eps) * gamma.double() + beta.double()


def _residual(M, g):
    """z ~ 2 N(0, 1) + a per-row offset (non-zero means exercise the mean c1 correction)."""
    z32 = 2 * torch.randn((M, H), generator=g, device="cuda") + \
        torch.randn((M, 1), generator=g, device="cuda")
    zh, zl = _split(z32)
    return zh, zl, zh.double() + zl.double()


def _close(out, ref, what):
    err = (out - ref).abs()
    bound = 3e-5 + 3e-6 * ref.abs()
    bad = err > bound
    print(f"{what}: max err {float(err.max()):.3g}")
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} out of bound, max {float(err.max()):.3g}"


@pytest.mark.parametrize("M", [777, 3000, 20001])
@pytest.mark.parametrize("N,gelu", [(1152, False), (1536, True), (1536, False)],
                         ids=["qkv", "ffn1", "ffn1-nogelu"])
def test_ln_consumer_matches_fp64(gpu, M, N, gelu):
    from ragmi.encoders import EPI_LN_F16, EPI_LN_GELU_F16, linear_dl
    g = torch.Generator(device="cuda")
    g.manual_seed(M + N + gelu)
    zh, zl, z64 = _residual(M, g)
    gamma = 1 + 0.2 * torch.randn((H,), generator=g, device="cuda")
    beta = 0.1 * torch.randn((H,), generator=g, device="cuda")
    w32 = torch.randn((N, H), generator=g, device="cuda") / math.sqrt(H)
    b = 0.1 * torch.randn((N,), generator=g, device="cuda")
    # the encoder's fold (bert_capi.hip fold_ln): W' = fp32(W gamma) as planes, c1 = their row
    # sums, c2 = b + W beta
    wfh, wfl = _split(w32 * gamma)
    c1 = (wfh.double() + wfl.double()).sum(1).float()
    c2 = (b.double() + w32.double() @ beta.double()).float()
    st = _stats(z64).float().contiguous()
    out_h = torch.empty((M, N), dtype=torch.float16, device="cuda")
    out_l = torch.empty_like(out_h)
    linear_dl(EPI_LN_GELU_F16 if gelu else EPI_LN_F16, zh, zl, wfh, wfl, c2, out_h, out_l,
              c1=c1, st_in=st, eps=1e-12)
    torch.cuda.synchronize()
    ref = _ln(z64, gamma, beta, 1e-12) @ w32.double().T + b.double()
    if gelu:
        ref = 0.5 * ref * (1.0 + torch.erf(ref / math.sqrt(2.0)))
    _close(out_h.double() + out_l.double(), ref, f"LN consumer M={M} N={N} gelu={gelu}")


@pytest.mark.parametrize("M", [777, 3000, 20001])
@pytest.mark.parametrize("K", [384, 1536], ids=["oproj", "ffn2"])
@pytest.mark.parametrize("pending", [True, False], ids=["ln-pending", "normalised"])
def test_residual_ln_matches_fp64(gpu, M, K, pending):
    from ragmi.encoders import EPI_RES_LN, linear_dl
    g = torch.Generator(device="cuda")
    g.manual_seed(M + K + pending)
    a32 = torch.randn((M, K), generator=g, device="cuda")
    ah, al = _split(a32)
    w32 = torch.randn((H, K), generator=g, device="cuda") / math.sqrt(K)
    wh, wl = _split(w32)
    b = 0.1 * torch.randn((H,), generator=g, device="cuda")
    zh, zl, z64 = _residual(M, g)
    gamma = 1 + 0.2 * torch.randn((H,), generator=g, device="cuda")
    beta = 0.1 * torch.randn((H,), generator=g, device="cuda")
    st_in = _stats(z64).float().contiguous() if pending else None
    st_out = torch.full((M, H // 64, 2), float("nan"), device="cuda")
    c, c_lo = zh.clone(), zl.clone()
    linear_dl(EPI_RES_LN, ah, al, wh, wl, b, c, c_lo, st_in=st_in,
              gamma=gamma if pending else None, beta=beta if pending else None, eps=1e-12,
              st_out=st_out)
    torch.cuda.synchronize()
    x = _ln(z64, gamma, beta, 1e-12) if pending else z64
    ref = (ah.double() + al.double()) @ (wh.double() + wl.double()).T + b.double() + x
    out = c.double() + c_lo.double()
    _close(out, ref, f"residual LN M={M} K={K} pending={pending}")
    want = _stats(ref)
    got = st_out.double()
    assert torch.isfinite(got).all()
    assert float((got[..., 0] - want[..., 0]).abs().max()) <= 2e-6
    rel = ((got[..., 1] - want[..., 1]).abs() / want[..., 1]).max()
    assert float(rel) <= 1e-5, float(rel)


def test_gemm_dl_rejects_bad_shapes(gpu):
    from ragmi.encoders import EPI_LN_F16, EPI_RES_LN, linear_dl
    z = torch.zeros((256, H), dtype=torch.float16, device="cuda")
    w = torch.zeros((256, H), dtype=torch.float16, device="cuda")
    v = torch.zeros((4096,), device="cuda")
    out = torch.zeros((256, 256), dtype=torch.float16, device="cuda")
    with pytest.raises(RuntimeError):          # RES_LN needs N == 384
        linear_dl(EPI_RES_LN, z, z, w, w, v, out, out.clone(), st_out=v)
    with pytest.raises(RuntimeError):          # LN consumers need c1 and st_in
        linear_dl(EPI_LN_F16, z, z, w, w, v, out, out.clone())
    wide = torch.zeros((2176, H), dtype=torch.float16, device="cuda")
    big = torch.zeros((256, 2176), dtype=torch.float16, device="cuda")
    with pytest.raises(RuntimeError):          # 2 N > the 4096-float staging area
        linear_dl(EPI_LN_F16, z, z, wide, wide, v, big, big.clone(), c1=v, st_in=v)


def _packed(rng, n, lo, hi, pair=False):
    lens = rng.integers(lo, hi, n)
    ids = np.concatenate([np.r_[101, rng.integers(1000, 30000, L - 2), 102] for L in lens])
    types = np.zeros(len(ids), np.int32)
    if pair:                                   # second half of every sequence: type 1
        cu = np.r_[0, np.cumsum(lens)]
        for a, b in zip(cu[:-1], cu[1:]):
            types[a + (b - a) // 2:b] = 1
    return ids.astype(np.int32), types, np.r_[0, np.cumsum(lens)].astype(np.int32)


@pytest.mark.parametrize("model", ["ce", "bge"])
def test_encoder_deferred_forced_vs_oracle(gpu, model):
    """Small batches (where AUTO leaves it off) with the deferred path forced on: every
    token-row GEMM runs on the WS kernel with the folded epilogues."""
    import bert_ref as R
    from ragmi.encoders import HEAD_CLS_L2, HEAD_POOLER_CLS, BertEncoder
    from test_config3_gpu import _oracle
    rng = np.random.default_rng(41 if model == "ce" else 42)
    if model == "ce":
        cfg, head, fn, tol = R.MINILM_CE, HEAD_POOLER_CLS, R.ce_logits, 1e-4
        ids, types, cu = _packed(rng, 24, 60, 300, pair=True)
    else:
        cfg, head, fn, tol = R.BGE_SMALL, HEAD_CLS_L2, R.bge_embed, 5e-6
        ids, types, cu = _packed(rng, 20, 8, 260)
    w = R.make_weights(cfg, 7)
    ref = _oracle(fn, w, cfg, ids, types, cu)
    enc = BertEncoder(cfg, w, head, gpu, "fp16x3")
    try:
        outs = {}
        for mode in (1, 0):
            enc.set_defer_ln(mode)
            outs[mode] = enc.forward_packed(ids, types, cu).cpu().numpy()
            d = np.abs(outs[mode] - ref)
            print(f"[{model} defer={mode}] max|d|={d.max():.3e}")
            assert d.max() <= tol
        assert np.abs(outs[1] - outs[0]).max() <= tol
    finally:
        enc.set_defer_ln(-1)
        enc.close()
