"""GPU tests of the encoder GEMM kernels (csrc/bert_kernels.hip: gemm_kernel = TILE,
gemm_pipe_kernel = PIPE) through the C ABI diagnostic entry rag_bert_gemm, against a float64
torch reference of the same nn.Linear (modeling_bert.py BertSelfAttention.query/key/value,
BertSelfOutput.dense, BertIntermediate.dense + erf-GELU, BertOutput.dense).

Tolerances (C ~ N(0, 1): A ~ N(0, 1), W ~ N(0, 1/K)):
  fp16 operands, fp32 out:   |C - ref| <= 2e-5 + 2e-6 |ref|   (fp32 accumulation of exact products)
  fp16 out:                  |C - fp64 ref| <= 2^-10 |ref| + 2e-5  (one fp16 rounding)
  fp16x3 (hi + lo planes):   |C - fp64 ref((Ah+Al)(Wh+Wl))| <= 2e-5 + 2e-6 |ref|
  erf-GELU epilogue: the same bounds against 0.5 x (1 + erf(x / sqrt 2)) in fp64.
TILE, PIPE and SMALL must agree to the same bounds (they differ only in accumulation
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
@pytest.mark.parametrize("variant", [1, 2, 5, 8], ids=["tile", "pipe", "small", "wide"])
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
def test_pipe_equals_tile(gpu, split):
    """The persistent kernel computes the same tile products as the per-tile kernel (many
    tiles per workgroup, a partial last M tile)."""
    from ragmi.encoders import EPI_F32, GEMM_PIPE, GEMM_TILE, linear
    M, N, K = 70001, 1536, 384
    a, al, w, wl, bias, _, _ = _operands(M, N, K, split, seed=7)
    c_t = linear(a, w, bias, EPI_F32, al, wl, GEMM_TILE)
    c_p = linear(a, w, bias, EPI_F32, al, wl, GEMM_PIPE)
    torch.cuda.synchronize()
    err = (c_t - c_p).abs()
    assert float(err.max()) <= 2e-5 + 2e-6 * float(c_t.abs().max()), float(err.max())


def test_gemm_rejects_bad_shapes(gpu):
    from ragmi._lib import RagmiError
    from ragmi.encoders import EPI_F32, GEMM_PIPE, linear
    a = torch.zeros((16, 96), dtype=torch.float16, device="cuda")     # K % 64 != 0
    w = torch.zeros((128, 96), dtype=torch.float16, device="cuda")
    b = torch.zeros((128,), dtype=torch.float32, device="cuda")
    with pytest.raises(RagmiError):
        linear(a, w, b, EPI_F32, variant=GEMM_PIPE)
