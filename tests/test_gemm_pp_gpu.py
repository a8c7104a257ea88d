"""The ping-pong encoder GEMM (csrc/bert_kernels.hip gemm_pp_kernel, rag_bert_gemm variant
RAG_GEMM_PP; round 5): fp16x3 256 x 192 tiles, two wave groups half a K step apart.

1. Dyadic operands (every product and partial sum exact in fp32, as in
   test_gemm_exact_gpu.py): every output element of the fp32 and fp16 hi + lo epilogues is
   known exactly, so a misplaced lane, fragment, ring slot or tile shows regardless of any
   tolerance. Shapes cover one tile row, ragged M, K = 1536, the panel-aligned XCD order
   (>= 64 row panels) and its split last round (half tiles: M = 40000 at N = 384), and grids
   where most workgroups get no tile at all (M = 1).
2. Random operands against float64 torch with test_gemm_gpu.py's bounds.
3. Bitwise agreement with the WS kernel where both run the same MFMA chains (>= 64 row panels:
   both take the K steps in order), f32 and f16 hi + lo outputs.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

PP, WS = 45, 19
SHAPES = [(1, 384, 384), (77, 1152, 384), (1000, 1536, 384), (3001, 384, 1536),
          (20000, 1152, 384), (40000, 384, 384), (40000, 384, 1536), (9000, 768, 384)]


def _grid(g, shape, den, kmax):
    return torch.randint(-kmax, kmax + 1, shape, generator=g, device="cuda").float() / den


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("epi", [0, 1, 2], ids=["f16", "gelu", "f32"])
def test_pp_epilogue_bit_exact(gpu, shape, epi):
    from ragmi.encoders import linear
    M, N, K = shape
    g = torch.Generator(device="cuda")
    g.manual_seed(M * 5 + N + 3 * K)
    a = _grid(g, (M, K), 16, 4).half()
    w = _grid(g, (N, K), 16, 4).half()
    bias = _grid(g, (N,), 256, 64)
    al = _grid(g, (M, K), 2048, 2).half()
    wl = _grid(g, (N, K), 2048, 2).half()
    out = linear(a, w, bias, epi, al, wl, PP)
    torch.cuda.synchronize()
    a64, w64 = a.double(), w.double()
    ref = (a64 @ w64.T + al.double() @ w64.T + a64 @ wl.double().T + bias.double()).float()
    if epi == 2:
        assert torch.equal(out, ref), "fp32 epilogue: misplaced or wrong elements"
        return
    if epi == 1:
        # GELU: compare with the WS kernel's GELU epilogue on the same exact sums instead of
        # re-deriving the polynomial (same gelu_erf4 arithmetic on identical inputs)
        hw, lw = linear(a, w, bias, epi, al, wl, WS)
        hi, lo = out
        assert torch.equal(hi.view(torch.int16), hw.view(torch.int16))
        assert torch.equal(lo.view(torch.int16), lw.view(torch.int16))
        return
    hi, lo = out
    hi_ref = ref.half()
    lo_ref = (ref - hi_ref.float()).half()
    bad = (hi != hi_ref) | (lo != lo_ref)
    if bool(bad.any()):
        rows, cols = torch.nonzero(bad, as_tuple=True)
        raise AssertionError(
            f"{int(bad.sum())} fp16 elements differ; first at rows {rows[:8].tolist()} "
            f"cols {cols[:8].tolist()}")


def _operands(M, N, K, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    a32 = torch.randn((M, K), generator=g, device="cuda")
    w32 = torch.randn((N, K), generator=g, device="cuda") / math.sqrt(K)
    bias = torch.randn((N,), generator=g, device="cuda") * 0.1
    a, w = a32.half(), w32.half()
    al, wl = (a32 - a.float()).half(), (w32 - w.float()).half()
    return a, al, w, wl, bias


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("epi", [0, 1, 2], ids=["f16", "gelu", "f32"])
def test_pp_matches_fp64(gpu, shape, epi):
    from ragmi.encoders import linear
    M, N, K = shape
    a, al, w, wl, bias = _operands(M, N, K, seed=M + 2 * N + K)
    out = linear(a, w, bias, epi, al, wl, PP)
    torch.cuda.synchronize()
    c = (a.double() + al.double()) @ (w.double() + wl.double()).T + bias.double()
    if epi == 1:
        c = 0.5 * c * (1.0 + torch.erf(c / math.sqrt(2.0)))
    v = (out[0].double() + out[1].double()) if isinstance(out, tuple) else out.double()
    err = (v - c).abs()
    bad = err > 2e-5 + 2e-6 * c.abs()
    assert not bool(bad.any()), f"{int(bad.sum())} out of bound, max err {float(err.max()):.3g}"


@pytest.mark.parametrize("shape", [(20000, 1152, 384), (40000, 384, 1536), (17000, 1536, 384)],
                         ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("epi", [0, 2], ids=["f16", "f32"])
def test_pp_bitwise_equals_ws(gpu, shape, epi):
    """From 64 row panels up both kernels run each output element's MFMA chain in the same
    order (K steps in order; per step W_lo A_hi, W_hi A_lo, W_hi A_hi), so random operands
    give identical bits."""
    from ragmi.encoders import linear
    M, N, K = shape
    a, al, w, wl, bias = _operands(M, N, K, seed=7 * M + N)
    p = linear(a, w, bias, epi, al, wl, PP)
    q = linear(a, w, bias, epi, al, wl, WS)
    torch.cuda.synchronize()
    if epi == 2:
        assert torch.equal(p.view(torch.int32), q.view(torch.int32))
    else:
        assert torch.equal(p[0].view(torch.int16), q[0].view(torch.int16))
        assert torch.equal(p[1].view(torch.int16), q[1].view(torch.int16))


def test_pp_rejects_bad_shapes(gpu):
    from ragmi._lib import RagmiError
    from ragmi.encoders import linear
    a, al, w, wl, bias = _operands(300, 512, 384, seed=1)     # N % 192 != 0
    with pytest.raises(RagmiError):
        linear(a, w, bias, 2, al, wl, PP)
    a, _, w, _, bias = _operands(300, 384, 384, seed=2)       # fp16 (no lo planes)
    with pytest.raises(RagmiError):
        linear(a, w, bias, 2, None, None, PP)
