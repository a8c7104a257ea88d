"""Per-GEMM HBM traffic of the rerank forward as it runs (deferred-LN WS kernels), from a
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE pass over scripts/bench_stages.py (STAGES=rerank):
each WS dispatch is named by its place in the layer (QKV, O-proj, FFN1, FFN2) and its
FETCH_SIZE x 1024 x 2 (gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md §HBM)
is set against the algorithmic reads of that GEMM at T tokens (fp16x3 operand planes: 4 B
per element of A and W; the residual planes and row statistics the epilogues read).
Usage: python scripts/fwd_pmc_summary.py <pmc_dir> <T> [counter]"""
import collections
import csv
import glob
import json
import os
import sys

H, FF, NL = 384, 1536, 6


def mfma_busy(d, T):
    """MFMA-busy pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE): per forward
    GEMM, the busy cycles against (a) the MFMA count the GEMM issues x 16 cycles per
    16x16x32 MFMA (MI355X_MICROARCH.md price list: the counter's own scale) and (b) the
    dispatch's cycles x 1024 SIMDs (GRBM_GUI_ACTIVE / 8 XCDs = the dispatch's clock cycles)."""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"name": r["Kernel_Name"]})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    shapes = {"qkv": (3 * H, H), "o_proj": (H, H), "ffn1": (FF, H), "ffn2": (H, FF)}
    res = collections.defaultdict(list)
    n6 = 0
    for e in disp.values():
        name = e["name"]
        if "gemm_ws_kernel" not in name:
            continue
        epi = name.split("gemm_ws_kernelILi")[1].split("E")[0]
        key = {"0": "qkv", "4": "qkv", "5": "ffn1"}.get(epi)
        if epi == "6":
            key = "o_proj" if n6 % 2 == 0 else "ffn2"
            n6 += 1
        if key is None:
            continue
        res[key].append(e)
    out = {"counter": "SQ_VALU_MFMA_BUSY_CYCLES", "tokens": T,
           "note": "per GEMM (median launch): busy / (MFMAs issued x 16) is the counter's scale "
                   "check; busy / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) the MFMA-busy fraction"}
    for key, es in res.items():
        N, K = shapes[key]
        n_mfma = 3 * T * N * K / (16 * 16 * 32)          # fp16x3: three MFMAs per product
        es = sorted(es, key=lambda e: e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0))
        e = es[len(es) // 2]
        busy = e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        cyc = e.get("GRBM_GUI_ACTIVE", 0.0) / 8
        out[key] = {"launches": len(es), "mfma_busy_cycles": busy,
                    "sq_busy_cycles": e.get("SQ_BUSY_CYCLES"), "dispatch_cycles": cyc,
                    "busy_per_mfma": round(busy / n_mfma, 3) if n_mfma else None,
                    "mfma_busy_frac": round(busy / (cyc * 1024), 4) if cyc else None}
    print(json.dumps(out))


def main():
    d, T = sys.argv[1], int(sys.argv[2])
    ctr = sys.argv[3] if len(sys.argv) > 3 else "FETCH_SIZE"
    if ctr == "MFMA":
        return mfma_busy(d, T)
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != ctr:
            continue
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, [r["Kernel_Name"], 0.0])
        e[1] += float(r["Counter_Value"])
    stats = T * (H // 64) * 8
    algo = {"qkv": T * H * 4 + 3 * H * H * 4 + stats,
            "o_proj": T * H * 4 + H * H * 4 + T * H * 4 + stats,
            "ffn1": T * H * 4 + FF * H * 4 + stats,
            "ffn2": T * FF * 4 + H * FF * 4 + T * H * 4 + stats}
    seq = []
    for k, (name, v) in disp.items():
        if "gemm_ws_kernel" not in name:
            continue
        epi = name.split("gemm_ws_kernelILi")[1].split("E")[0]
        seq.append((epi, v))
    # per forward: [QKV plain (EPI 0) or Ln (4)], ResLn O (6), LnGelu (5), ResLn FFN2 (6), ...
    res = collections.defaultdict(list)
    n6 = 0
    for epi, v in seq:
        if epi in ("0", "4"):
            key = "qkv"
        elif epi == "5":
            key = "ffn1"
        elif epi == "6":
            key = "o_proj" if n6 % 2 == 0 else "ffn2"
            n6 += 1
        else:
            continue
        b = v * 1024 * (2 if ctr == "FETCH_SIZE" else 1)
        res[key].append(b)
    out = {"counter": ctr, "tokens": T, "note": "FETCH_SIZE kB x 1024 x 2 (gfx950 correction); "
           "algorithmic = operand planes + residual planes + row statistics read once"}
    for key, vals in res.items():
        m = sorted(vals)[len(vals) // 2]
        out[key] = {"launches": len(vals), "median_bytes": m,
                    "algorithmic_read_bytes": algo[key] if ctr == "FETCH_SIZE" else None,
                    "ratio": round(m / algo[key], 3) if ctr == "FETCH_SIZE" else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
