"""Bit-exact layout test of every encoder GEMM epilogue (rag_bert_gemm: TILE, PIPE, SMALL,
WIDE, SMALL-BK64, BIG, BIG128, WS, WS-NT; fp16 and fp16x3; fp32 and fp16 [+ lo plane] outputs).

Operands sit on a coarse dyadic grid (hi planes k/16, |k| <= 4; lo planes k/2048, |k| <= 2;
bias k/256) so every product and every partial sum is exactly representable in fp32: the
result does not depend on the MFMA accumulation order, and each output element — its fp32
value, its fp16 rounding and the fp16 lo plane fp16(v - fp16(v)) — is known exactly. A lane
or fragment stored to the wrong place (e.g. a v_permlane16_swap pairing that misroutes some
lanes of the 16-B fp16 stores, bert_kernels.hip store_f16_pair) shows up as a mismatch
regardless of any numerical tolerance.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(77, 1152, 384), (1000, 1536, 384), (3001, 384, 1536), (20000, 1152, 384),
          (9000, 384, 384), (130, 768, 768)]


def _grid(g, shape, den, kmax):
    return (torch.randint(-kmax, kmax + 1, shape, generator=g, device="cuda").float() / den)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("epi", [0, 2], ids=["f16", "f32"])
@pytest.mark.parametrize("split", [False, True], ids=["fp16", "fp16x3"])
@pytest.mark.parametrize("variant", [1, 5, 19], ids=["tile", "small", "ws"])
def test_gemm_epilogue_bit_exact(gpu, shape, epi, split, variant):
    from ragmi.encoders import linear
    M, N, K = shape
    g = torch.Generator(device="cuda")
    g.manual_seed(M * 7 + N + K)
    a = _grid(g, (M, K), 16, 4).half()
    w = _grid(g, (N, K), 16, 4).half()
    bias = _grid(g, (N,), 256, 64)
    al = wl = None
    if split:
        al = _grid(g, (M, K), 2048, 2).half()
        wl = _grid(g, (N, K), 2048, 2).half()
    out = linear(a, w, bias, epi, al, wl, variant)
    torch.cuda.synchronize()
    # exact reference: float64 sums of the fp16-exact products (each sum < 2^24 ulps)
    a64, w64 = a.double(), w.double()
    ref = a64 @ w64.T
    if split:
        ref = ref + al.double() @ w64.T + a64 @ wl.double().T
    ref = (ref + bias.double()).float()                 # exact in fp32 by construction
    assert torch.equal(ref.double(), (a64 @ w64.T + (al.double() @ w64.T + a64 @ wl.double().T
                                                      if split else 0) + bias.double()))
    if epi == 2:
        assert torch.equal(out, ref), "fp32 epilogue: misplaced or wrong elements"
        return
    hi_ref = ref.half()
    if isinstance(out, tuple):
        hi, lo = out
        lo_ref = (ref - hi_ref.float()).half()
        bad = (hi != hi_ref) | (lo != lo_ref)
    else:
        hi = out
        bad = hi != hi_ref
    if bool(bad.any()):
        rows, cols = torch.nonzero(bad, as_tuple=True)
        raise AssertionError(
            f"{int(bad.sum())} fp16 elements differ; first at rows {rows[:8].tolist()} "
            f"cols {cols[:8].tolist()} (row % 16: {(rows[:8] % 16).tolist()})")


@pytest.mark.parametrize("shape", [(20000, 1152, 384), (3001, 384, 1536), (777, 1536, 384)],
                         ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("variant", [1, 5, 19], ids=["tile", "small", "ws"])
def test_split_planes_match_fp32_epilogue(gpu, shape, variant):
    """Random (non-dyadic) fp16x3 operands: the fp16 epilogue's planes are exactly
    hi = fp16(v), lo = fp16(v - hi) of the fp32 value v the same kernel's fp32 epilogue stores
    (same MFMA chains, only the epilogue differs) — checks split16x2's v_fma_mix lo plane
    bit for bit where v - hi needs every fp16 rounding case."""
    from ragmi.encoders import linear
    M, N, K = shape
    g = torch.Generator(device="cuda")
    g.manual_seed(M + 3 * N + K)
    a32 = torch.randn((M, K), generator=g, device="cuda")
    w32 = torch.randn((N, K), generator=g, device="cuda") * 0.05
    bias = torch.randn((N,), generator=g, device="cuda") * 0.1
    a, w = a32.half(), w32.half()
    al, wl = (a32 - a.float()).half(), (w32 - w.float()).half()
    v = linear(a, w, bias, 2, al, wl, variant)
    hi, lo = linear(a, w, bias, 0, al, wl, variant)
    torch.cuda.synchronize()
    hi_ref = v.half()
    lo_ref = (v - hi_ref.float()).half()
    assert torch.equal(hi.view(torch.int16), hi_ref.view(torch.int16))
    assert torch.equal(lo.view(torch.int16), lo_ref.view(torch.int16))
