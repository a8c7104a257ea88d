import sys, math, torch
sys.path.insert(0, "financial-rag-system_amd"); sys.path.insert(0, "tests")
from ragmi.encoders import linear_add_ln
from test_gemm_gpu import _operands
for M, K, split in ((3001, 1536, True), (300, 384, True), (129, 384, True)):
    N = 384
    a, al, w, wl, bias, a64, w64 = _operands(M, N, K, split, seed=M + K + 1)
    g = torch.Generator(device="cuda"); g.manual_seed(M + 3)
    x = torch.randn((M, N), generator=g, device="cuda")
    gamma = 1.0 + 0.2 * torch.randn((N,), generator=g, device="cuda")
    beta = 0.1 * torch.randn((N,), generator=g, device="cuda")
    out = linear_add_ln(a, w, bias, gamma, beta, 1e-12, x, al, wl)
    torch.cuda.synchronize()
    xo, xh, xl = out
    bad = (xh != xo.half())
    idx = bad.nonzero()
    print(M, K, "bad xh:", int(bad.sum()), "rows", sorted(set((idx[:, 0] % 128).tolist()))[:20], "cols", sorted(set(idx[:, 1].tolist()))[:40])
    for r, c in idx[:5].tolist():
        print("  ", r, c, float(xh[r, c]), float(xo[r, c]), float(xl[r, c]))
    badl = ((xh.double() + xl.double() - xo.double()).abs() > xl.double().abs() * 2**-10 + 2**-24)
    print("  bad xl:", int(badl.sum()))
