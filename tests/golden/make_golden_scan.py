"""Generate tests/golden/scan_golden.npz from the CPU restatement (oracle/scan_ref.c).

The reference (pythonmailer/financial-rag-system) holds no golden vectors or numeric tests
for this path (tests.py runs TESTING stubs, main.py:216), and its search engine (Qdrant
server) is not available here, so these fixtures are produced by the oracle and pinned
independently by tests/test_oracle_scan.py (numpy float64 formulation). Inputs are stored,
not regenerated, so the fixture is independent of numpy's RNG stream.

Contents (D = 384, the bge-small width, database.py:31 VECTOR_SIZE):
  x        [N,D] f32  raw vectors as handed to upsert (N = 400: 25 tiles, ragged last wave)
  tags     [N]   u32  ticker code | doctype code << 16
  enc16    [N,D] u16  stored fp16 rows (canonical normalise, RNE)
  q        [B,D] f32  32 planted (corpus row + 0.05 noise) + 8 pure random queries
  filt     [B,2] u32  per-query (mask, value)
  ids15/s15    unfiltered top-15 (limit=15, main.py:215)
  idsf/sf      filtered top-15
  ids5/s5      top-5 (QueryRequest.top_k default, main.py:118)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle_scan as O  # noqa: E402


def main():
    rng = np.random.default_rng(20260515)
    N, D = 400, 384
    x = rng.standard_normal((N, D), dtype=np.float32)
    x[7] *= 1e-3            # tiny-norm row
    x[11] = 0.0             # zero vector: stays zero
    x[42] = x[41]           # exact duplicate (tie broken by row id)
    tickers = rng.integers(1, 5, N).astype(np.uint32)
    doct = rng.integers(1, 3, N).astype(np.uint32)
    tags = tickers | (doct << 16)
    enc16 = O.encode_rows(x)
    picks = rng.choice(N, 32, replace=False)
    picks[0] = 41
    q_pl = x[picks] + 0.05 * rng.standard_normal((32, D), dtype=np.float32)
    q = np.concatenate([q_pl, rng.standard_normal((8, D), dtype=np.float32)]).astype(np.float32)
    B = q.shape[0]
    filt = np.zeros((B, 2), dtype=np.uint32)
    for b in range(B):
        if b % 3 == 0:
            filt[b] = (0xFFFF, rng.integers(1, 5))                       # ticker == T
        elif b % 3 == 1:
            filt[b] = (0xFFFFFFFF, rng.integers(1, 5) | (rng.integers(1, 3) << 16))  # + doctype
    s15, ids15 = O.search(enc16, q, 15)
    s5, ids5 = O.search(enc16, q, 5)
    sf = np.empty((B, 15), np.float32)
    idsf = np.empty((B, 15), np.int64)
    for b in range(B):
        a, i = O.search(enc16, q[b:b + 1], 15, tags=tags, mask=int(filt[b, 0]),
                        value=int(filt[b, 1]), use_filter=True)
        sf[b], idsf[b] = a[0], i[0]
    np.savez_compressed(os.path.join(HERE, "scan_golden.npz"), x=x, tags=tags, enc16=enc16,
                        q=q, filt=filt, ids15=ids15, s15=s15, ids5=ids5, s5=s5, idsf=idsf,
                        sf=sf)
    print("wrote scan_golden.npz", {k: v.shape for k, v in
                                     dict(x=x, q=q, ids15=ids15, idsf=idsf).items()})


if __name__ == "__main__":
    main()
