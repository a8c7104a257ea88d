"""GPU tests of the encoder GEMM kernels (csrc/bert_kernels.hip: gemm_kernel = TILE,
gemm_pipe_kernel<PipeSmall> = SMALL, gemm_ws_kernel = WS) through the C ABI diagnostic entry rag_bert_gemm, against a float64
torch reference of the same nn.Linear (modeling_bert.py BertSelfAttention.query/key/value,
BertSelfOutput.dense, BertIntermediate.dense + erf-GELU, BertOutput.dense).

Tolerances (C ~ N(0, 1): A ~ N(0, 1), W ~ N(0, 1/K)):
  fp16 operands, fp32 out:   |C - ref| <= 2e-5 + 2e-6 |ref|   (fp32 accumulation of exact products)
  fp16 out:                  |C - fp64 ref| <= 2^-10 |ref| + 2e-5  (one fp16 rounding)
  fp16x3 (hi + lo planes):   |C - fp64 ref((Ah+Al)(Wh+Wl))| <= 2e-5 + 2e-6 |ref|
  erf-GELU epilogue: the same bounds against 0.5 x (1 + erf(x / sqrt 2)) in fp64.
TILE, SMALL and WS must agree to the same bounds (they differ only in accumulation
association).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, N, K): query batch, chunk batch, rerank batch tails, FFN2 K = 1536
    (1, 384, 384), (77, 1152, 384), (1000, 1536, 384), (3001, 384, 1536),
    (20000, 1152, 384), (9000, 384, 384),
]


def _operands(M, N, K, split, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    a32 = torch.randn((M, K), generator=g, device="cuda")
    w32 = torch.randn((N, K), generator=g, device="cuda") / math.sqrt(K)
    bias = torch.randn((N,), generator=g, device="cuda") * 0.1
    a, w = a32.half(), w32.half()
    if not split:
        return a, None, w, None, bias, a.double(), w.double()
    al = (a32 - a.float()).half()
    wl = (w32 - w.float()).half()
    return a, al, w, wl, bias, a.double() + al.double(), w.double() + wl.double()


def _ref(a64, w64, bias, epi):
    from ragmi.encoders import EPI_GELU_F16
    c = a64 @ w64.T + bias.double()
    if epi == EPI_GELU_F16:
        c = 0.5 * c * (1.0 + torch.erf(c / math.sqrt(2.0)))
    return c


def _check(c, ref, epi, split):
    from ragmi.encoders import EPI_F32
    c = c.double()
    err = (c - ref).abs()
    if epi == EPI_F32:
        bound = 2e-5 + 2e-6 * ref.abs()
    else:
        bound = 2e-5 + ref.abs() * 2.0 ** -10
    bad = err > bound
    assert not bool(bad.any()), (f"{int(bad.sum())} elements out of bound; max err "
                                 f"{float(err.max()):.3g}")


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("epi", [0, 1, 2], ids=["f16", "gelu", "f32"])
@pytest.mark.parametrize("split", [False, True], ids=["fp16", "fp16x3"])
@pytest.mark.parametrize("variant", [1, 5, 19], ids=["tile", "small", "ws"])
def test_gemm_matches_fp64(gpu, shape, epi, split, variant):
    from ragmi.encoders import linear
    M, N, K = shape
    a, al, w, wl, bias, a64, w64 = _operands(M, N, K, split, seed=M + N + K)
    out = linear(a, w, bias, epi, al, wl, variant)
    torch.cuda.synchronize()
    ref = _ref(a64, w64, bias, epi)
    if isinstance(out, tuple):          # fp16x3 fp16 output: hi + lo reconstructs fp32
        hi, lo = out
        _check(hi.double() + lo.double(), ref, 2, split)
        _check(hi, ref, epi, split)
    else:
        _check(out, ref, epi, split)


@pytest.mark.parametrize("split", [False, True], ids=["fp16", "fp16x3"])
def test_ws_equals_tile(gpu, split):
    """The persistent kernel computes the same tile products as the per-tile kernel (many
    tiles per workgroup, a partial last M tile)."""
    from ragmi.encoders import EPI_F32, GEMM_TILE, GEMM_WS, linear
    M, N, K = 70001, 1536, 384
    a, al, w, wl, bias, _, _ = _operands(M, N, K, split, seed=7)
    c_t = linear(a, w, bias, EPI_F32, al, wl, GEMM_TILE)
    c_p = linear(a, w, bias, EPI_F32, al, wl, GEMM_WS)
    torch.cuda.synchronize()
    err = (c_t - c_p).abs()
    assert float(err.max()) <= 2e-5 + 2e-6 * float(c_t.abs().max()), float(err.max())


def test_gemm_rejects_bad_shapes(gpu):
    from ragmi._lib import RagmiError
    from ragmi.encoders import EPI_F32, GEMM_WS, linear
    a = torch.zeros((16, 96), dtype=torch.float16, device="cuda")     # K % 64 != 0
    w = torch.zeros((128, 96), dtype=torch.float16, device="cuda")
    b = torch.zeros((128,), dtype=torch.float32, device="cuda")
    with pytest.raises(RagmiError):
        linear(a, w, b, EPI_F32, variant=GEMM_WS)
    # variant ids of the A/B forms removed in round 5 are refused, not silently mapped
    a = torch.zeros((16, 128), dtype=torch.float16, device="cuda")
    w = torch.zeros((128, 128), dtype=torch.float16, device="cuda")
    for v in (2, 8, 10, 34, 35, 45):
        with pytest.raises(RagmiError):
            linear(a, w, b, EPI_F32, variant=v)


@pytest.mark.parametrize("shape", [(1, 384), (3001, 1536), (20000, 384), (70001, 1536)],
                         ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("split", [False, True], ids=["fp16", "fp16x3"])
def test_gemm_add_ln_matches_fp64(gpu, shape, split):
    """rag_bert_gemm_add_ln: x <- LN(x + a.w^T + bias) * gamma + beta (BertSelfOutput /
    BertOutput), whole 384-wide rows per tile, against fp64. The pre-LN sum carries the GEMM
    bound above; normalising by its std (~1.4) keeps it: |x - ref| <= 5e-5 + 5e-6 |ref|.
    xh must be exactly the fp16 rounding of the returned fp32 x, xl its residual."""
    from ragmi.encoders import linear_add_ln
    M, K = shape
    N = 384
    a, al, w, wl, bias, a64, w64 = _operands(M, N, K, split, seed=M + K + 1)
    g = torch.Generator(device="cuda")
    g.manual_seed(M + 3)
    # x is the head of a larger buffer: the 130 rows after it must come through untouched
    # (the last tile's rows past M are dropped by the bounded buffer stores)
    x_full = torch.randn((M + 130, N), generator=g, device="cuda")
    tail = x_full[M:].clone()
    x = x_full[:M]
    gamma = 1.0 + 0.2 * torch.randn((N,), generator=g, device="cuda")
    beta = 0.1 * torch.randn((N,), generator=g, device="cuda")
    eps = 1e-12
    v = x.double() + a64 @ w64.T + bias.double()
    mu = v.mean(1, keepdim=True)
    var = ((v - mu) ** 2).mean(1, keepdim=True)
    ref = (v - mu) / torch.sqrt(var + eps) * gamma.double() + beta.double()
    out = linear_add_ln(a, w, bias, gamma, beta, eps, x, al, wl)
    torch.cuda.synchronize()
    xo, xh = out[0], out[1]
    assert xo.data_ptr() == x.data_ptr()
    assert torch.equal(x_full[M:], tail)
    assert bool(torch.isfinite(xo).all())
    err = (xo.double() - ref).abs()
    bad = err > 5e-5 + 5e-6 * ref.abs()
    assert not bool(bad.any()), f"{int(bad.sum())} out of bound; max err {float(err.max()):.3g}"
    assert torch.equal(xh, xo.half())
    if split:   # xl: x - xh to fp16 precision (the kernel may round it once, from x - xh
        #         in one mixed-precision op, where torch rounds twice: 1 fp16 ulp apart, rarely)
        xl = out[2].double()
        assert float(((xh.double() + xl) - xo.double()).abs().sub(
            xl.abs() * 2.0 ** -10 + 2.0 ** -24).max()) <= 0


def test_gemm_add_ln_rejects_bad_shapes(gpu):
    from ragmi._lib import RagmiError
    from ragmi.encoders import linear_add_ln
    a = torch.zeros((16, 384), dtype=torch.float16, device="cuda")
    w = torch.zeros((768, 384), dtype=torch.float16, device="cuda")     # N != 384
    v = torch.zeros((768,), dtype=torch.float32, device="cuda")
    x = torch.zeros((16, 768), dtype=torch.float32, device="cuda")
    with pytest.raises(RagmiError):
        linear_add_ln(a, w, v, v, v, 1e-12, x)


@pytest.mark.parametrize("shape", [(117000, 384, 1536), (117000, 1152, 384), (70001, 1536, 384),
                                   (20000, 384, 384)], ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("epi", [0, 2], ids=["f16", "f32"])
@pytest.mark.parametrize("split", [False, True], ids=["fp16", "fp16x3"])
def test_ws_split_last_round_matches_fp64(gpu, shape, epi, split):
    """The WS kernel at the forward's large shapes, where its split last round runs the XCD's
    last r <= 16 tiles as 128-row halves on two workgroups each: every row (half tiles and the
    partial last panel included) within the fp64 bound."""
    from ragmi.encoders import GEMM_WS, linear
    M, N, K = shape
    a, al, w, wl, bias, a64, w64 = _operands(M, N, K, split, seed=M + 3 * N)
    out = linear(a, w, bias, epi, al, wl, GEMM_WS)
    torch.cuda.synchronize()
    ref = _ref(a64, w64, bias, epi)
    if isinstance(out, tuple):
        _check(out[0].double() + out[1].double(), ref, 2, split)
    else:
        _check(out, ref, epi, split)


@pytest.mark.parametrize("shape", [(1, 384, 384), (782, 384, 384), (782, 384, 1536),
                                   (33, 1024, 4096), (3001, 384, 1536)],
                         ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("split", [False, True], ids=["fp16", "fp16x3"])
@pytest.mark.parametrize("variant", [0, 5], ids=["auto", "small"])
def test_gemm_splitk_parts_sum_to_fp64(gpu, shape, split, variant):
    """Split-K of the small-batch fp32-output GEMMs (rag_bert_gemm_splitk: the parts the
    forward sums in its residual + LayerNorm pass): sum of parts vs fp64 at the fp32-output
    bound, part 0 alone carries the bias, and the part count depends on K only (batch
    independence)."""
    import ctypes

    from ragmi import _lib
    M, N, K = shape
    a, al, w, wl, bias, a64, w64 = _operands(M, N, K, split, seed=3 * M + K)
    c = torch.full((4, M, N), float("nan"), device="cuda")
    parts = ctypes.c_int()
    _lib.check(_lib.load().rag_bert_gemm_splitk(
        variant, a.data_ptr(), al.data_ptr() if split else None, w.data_ptr(),
        wl.data_ptr() if split else None, bias.data_ptr(), M, N, K, c.data_ptr(), 4,
        ctypes.byref(parts), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    p = parts.value
    assert 1 <= p <= 4
    tot = c[:p].double().sum(0)
    _check(tot, _ref(a64, w64, bias, 2), 2, split)
    if p > 1:
        # parts 1.. are bias-free partial products (no part is left unwritten)
        assert not bool(torch.isnan(c[:p]).any())
    if M > 1 and variant != 0:
        one = torch.full((4, 1, N), float("nan"), device="cuda")
        p1 = ctypes.c_int()
        _lib.check(_lib.load().rag_bert_gemm_splitk(
            variant, a[:1].contiguous().data_ptr(), al[:1].contiguous().data_ptr() if split else None,
            w.data_ptr(), wl.data_ptr() if split else None, bias.data_ptr(), 1, N, K,
            one.data_ptr(), 4, ctypes.byref(p1), torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        assert p1.value == p
        assert torch.equal(one[:p].sum(0)[0], c[:p, 0].sum(0))
