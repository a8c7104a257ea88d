"""HBM traffic of one encoder forward: the config-3 rerank forward
(MiniLM-L6 CE, 480 pairs) and the config-2 query forward (bge-small, 32 queries), from
rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes over scripts/bench_stages.py
(scripts/gpu_encoder_pmc.sh). Per forward (dispatches split at each embed_ln_kernel):
  read  = sum of FETCH_SIZE x 1024 x 2 (gfx950 reports half of wide streaming reads,
          MI355X_MICROARCH.md §HBM; the encoder's loads are 16-B-per-lane streams)
  write = sum of WRITE_SIZE x 1024
against the forward's ALGORITHMIC bytes: every weight plane read once, and per layer every
activation plane read and written once by an unsplit, unfused data flow — Q|K|V, context,
LayerNorm output, FFN intermediate, residual (fp16x3: hi + lo planes, 4 B per element) —
so the ratio measures what the implementation adds: split-K partial slabs, the fp32 residual
copy, deferred-LN row statistics, operand re-reads beyond L2.
Usage: python scripts/encoder_traffic.py <stage> <fetch_dir> <write_dir> <stage_log> [out.json]
"""
import collections
import csv
import glob
import json
import os
import sys

CFG = {"rerank": dict(H=384, FF=1536, L=6, cls_last=True, model="MiniLM-L6 cross-encoder"),
       "encode_q": dict(H=384, FF=1536, L=12, cls_last=True, model="bge-small-en-v1.5")}
P = 4          # fp16x3: hi + lo planes, 2 B each


def algorithmic(stage: str, T: int) -> tuple[int, int]:
    c = CFG[stage]
    H, FF, L = c["H"], c["FF"], c["L"]
    w_layer = (4 * H * H + 2 * H * FF) * P
    reads = L * w_layer + 2 * T * H * 4                 # weights; word + position rows (fp32)
    writes = T * H * P                                  # embedding LayerNorm output
    full = L - 1 if c["cls_last"] else L
    reads += full * T * (H + 3 * H + H + H + H + FF + H) * P
    writes += full * T * (3 * H + H + H + FF + H) * P
    if c["cls_last"]:                                   # last layer: K|V for every token,
        reads += T * (H + 2 * H) * P                    # the rest on the CLS rows only
        writes += T * 2 * H * P
    return reads, writes


def per_dispatch(d: str, counter: str):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, [r["Kernel_Name"], 0.0])
        e[1] += float(r["Counter_Value"])
    return [(disp[k][0], disp[k][1]) for k in sorted(disp)]


def forwards(seq):
    """Split a dispatch sequence into whole forwards (each starts at embed_ln_kernel); the
    harness's first forward (warm-up) is included, partial ones are dropped."""
    out, cur = [], None
    for name, v in seq:
        if "embed_ln_kernel" in name:
            if cur:
                out.append(cur)
            cur = []
        if cur is not None and "ragmi" in name:
            cur.append((name, v))
    if cur:
        out.append(cur)
    return out


def classify(name: str) -> str:
    for key in ("gemm_ws_kernel", "gemm_pipe_kernel", "attn_cls_kernel", "attn_kernel",
                "add_ln", "embed_ln", "gather_cls", "ce_head", "cls_normalize"):
        if key in name:
            return key
    return "other"


def main():
    stage, fdir, wdir, log = sys.argv[1:5]
    out_path = sys.argv[5] if len(sys.argv) > 5 else None
    line = next(json.loads(x) for x in open(log) if x.startswith("{") and stage in x)
    T, B = int(line["tokens"]), int(line["sequences"])
    res = {"stage": stage, "model": CFG[stage]["model"], "tokens": T, "sequences": B,
           "precision": line.get("precision")}
    for counter, d, scale in (("FETCH_SIZE", fdir, 2048), ("WRITE_SIZE", wdir, 1024)):
        fw = forwards(per_dispatch(d, counter))
        # the last complete forward's kernels (every forward of the harness is identical)
        totals = [sum(v for _, v in f) * scale for f in fw]
        f = fw[-1]
        by = collections.defaultdict(float)
        for name, v in f:
            by[classify(name)] += v * scale
        key = "read" if counter == "FETCH_SIZE" else "write"
        res[f"{key}_bytes_per_forward"] = round(totals[-1])
        res[f"{key}_forwards_seen"] = len(fw)
        res[f"{key}_spread"] = round((max(totals) - min(totals)) / max(totals), 4) if totals else None
        res[f"{key}_by_kernel"] = {k: round(v) for k, v in sorted(by.items(), key=lambda x: -x[1])}
    ar, aw = algorithmic(stage, T)
    res["algorithmic_read_bytes"] = ar
    res["algorithmic_write_bytes"] = aw
    res["read_ratio"] = round(res["read_bytes_per_forward"] / ar, 3)
    res["write_ratio"] = round(res["write_bytes_per_forward"] / aw, 3)
    res["note"] = ("read = FETCH_SIZE x 1024 x 2 (gfx950 correction), write = WRITE_SIZE x "
                   "1024, summed over one forward's dispatches; algorithmic = weights once + "
                   "every activation plane (fp16x3 hi + lo) read and written once per layer")
    print(json.dumps(res))
    if out_path:
        table = {}
        if os.path.exists(out_path):
            table = json.load(open(out_path))
        table[stage] = res
        json.dump(table, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
