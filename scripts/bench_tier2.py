"""Latency of the certificate's tier 2 (the rescan pass, csrc/scan_kernels.hip rescan_kernel)
on a duplicate-heavy corpus (measure it at 1.25M and 10M rows).

Corpus: torch randn rows (GPU generator), every `every`-th row replaced by base + 1e-5 noise
(near-duplicates of one vector: each scan wave's list overflows inside the MFMA error band,
so tier 1 cannot certify). Batch of 32: M queries near `base` (tier 2; M = 4 by default, and
16 / 32 with --marked) + 32 - M random (tier 0). Round 4: all marked queries of a pass share
one rescan launch (csrc/scan_kernels.hip rescan_kernel).
Reports the device time of one search call with and without the tier-2 queries, the tiers,
and the ids of the tier-2 queries checked against an fp64 exact top-15 of the duplicate rows
(the duplicates dominate every tier-2 query's top-15)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
from ragmi.index import FlatIndex  # noqa: E402

D, B, K = 384, 32, 15


def run(n, every, reps=5, marked=4):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    idx = FlatIndex(dim=D, capacity=n, device=dev, diagnostic=True)
    base = torch.randn((1, D), generator=g, device=dev)
    chunk = 1 << 20
    dup_rows = []
    for r0 in range(0, n, chunk):
        m = min(chunk, n - r0)
        x = torch.randn((m, D), generator=g, device=dev)
        rows = torch.arange(r0, r0 + m, device=dev)
        sel = (rows % every) == 0
        x[sel] = base + 1e-5 * torch.randn((int(sel.sum()), D), generator=g, device=dev)
        dup_rows.append(rows[sel])
        idx.upsert(x, rows, new_count=r0 + m)
    dup_rows = torch.cat(dup_rows)
    q_dup = base + 0.02 * torch.randn((marked, D), generator=g, device=dev)
    q_rnd = torch.randn((B - marked, D), generator=g, device=dev)
    q_mix = torch.cat([q_dup, q_rnd])
    q_all_rnd = torch.randn((B, D), generator=g, device=dev)

    def timed(q):
        idx.search(q, K)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            out = idx.search(q, K)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps, out
    t_rnd, _ = timed(q_all_rnd)
    t1a, t2a, _ = idx.exactness_stats()
    t_mix, (s, i) = timed(q_mix)
    t1b, t2b, tiers = idx.exactness_stats(B)
    # exact check of the tier-2 queries over the duplicate rows (they fill each top-15):
    # fp64 scores of the STORED rows, ranked (score desc, row asc)
    # canonical scores: the oracle's normalised fp32 query, fp64 dot with the
    # stored fp16 row, rounded to fp32; ties by row asc
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_scan as O
    rows = dup_rows.cpu().numpy()
    stored = idx.export_rows(0, n).view(np.float16)[rows].astype(np.float64)
    qn = O.normalize(q_mix[:marked].cpu().numpy())
    ok = 0
    for j in range(marked):
        sc = (stored @ qn[j].astype(np.float64)).astype(np.float32)
        order = np.lexsort((rows, -sc.astype(np.float64)))[:K]
        ok += int(np.array_equal(rows[order], i[j].cpu().numpy()) and
                  np.array_equal(sc[order], s[j].cpu().numpy()))
    idx.close()
    return {"rows": n, "duplicates": int(dup_rows.numel()), "dup_every": every,
            "search_ms_all_random": round(t_rnd, 4),
            "marked": marked,
            "search_ms_with_tier2_queries": round(t_mix, 4),
            "tier2_added_ms": round(t_mix - t_rnd, 4),
            "rescan_wg_knob": os.environ.get("RAGMI_RESCAN_WG"),
            "tier2_queries_per_call": int((t2b - t2a) / (reps + 1)),
            "tiers_first_8": tiers[:8].tolist(),
            "tier2_ids_match_fp64_exact": f"{ok}/{marked}"}


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--marked", type=int, nargs="+", default=[4])
    ap.add_argument("--rows", type=int, nargs="+", default=[1_250_000, 10_000_000])
    a = ap.parse_args()
    every = {1_250_000: 12, 10_000_000: 50}
    for n in a.rows:
        for m in a.marked:
            print(json.dumps(run(n, every.get(n, 12), marked=m)), flush=True)
