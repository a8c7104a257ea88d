"""Diagnostic: per-element dump of the attention kernel's worst fp16x3 outputs vs a float64
reference (sequence lengths with and without a masked tail block)."""
import numpy as np, torch, sys
sys.path.insert(0, "financial-rag-system_amd")
from ragmi.encoders import attention
def ref(x, cu):
    x = x.double(); out = torch.empty((x.shape[0], 384), dtype=torch.float64, device=x.device)
    for b in range(len(cu)-1):
        a, e = cu[b], cu[b+1]
        for h in range(12):
            sl = slice(32*h, 32*h+32)
            s = (x[a:e, sl] @ x[a:e, 384+32*h:384+32*h+32].T) / np.sqrt(32.0)
            out[a:e, sl] = torch.softmax(s, 1) @ x[a:e, 768+32*h:768+32*h+32]
    return out
for L in (240, 288):
    g = torch.Generator(device="cuda"); g.manual_seed(5)
    cu = np.array([0, L], np.int32)
    x = torch.randn((L, 1152), generator=g, device="cuda") * 2.0
    x[:, 768:] = torch.rand((L, 384), generator=g, device="cuda") * 2 - 1
    hi = x.half(); lo = (x - hi.float()).half()
    xs = hi.float() + lo.float()
    o, ol = attention(hi, torch.from_numpy(cu).cuda(), L, lo, 2)
    r = ref(xs, cu)
    got = o.double() + ol.double()
    d = (got - r).abs()
    idx = torch.nonzero(d > 1e-5)
    for t, c in idx.tolist():
        print(f"L {L} q {t} head {c//32} d {c%32} (dt {c%32//16} g {(c%16)//4} r {c%4}): hi {o[t,c].item():.8f} lo {ol[t,c].item():.3e} "
              f"ref {r[t,c].item():.8f} fp16(ref) {r[t,c].half().item():.8f} err {(got[t,c]-r[t,c]).item():.3e}", flush=True)
    # same query, neighbouring d: all fine?
