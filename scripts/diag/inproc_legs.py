"""why the config-2 leg loses ~21% inside the headline's process (62K vs
79K qps, profiles/r06c_legs.jsonl) while config 3 does not. One process, config-2 legs
(scripts/bench_modes.run_pipeline, 20 warm-up + 200 timed batches) after each of:
  fresh            nothing before it
  streams+N        N extra torch streams created and used (one kernel each), kept alive
  streams+N_freed  the same, then the stream objects dropped
  headline         a 10M x 384 index built, searched on 2 streams (the headline's shape), freed
One JSON line per case: qps, ms per batch, host enqueue ms per batch."""
import argparse
import gc
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench_modes  # noqa: E402


def leg(tag, extra=None, partition="auto"):
    a = argparse.Namespace(config="2", steps=200, warmup=20, rows=0, streams=0, partition=partition,
                           precision="fp16x3", no_recall=True, no_cpu=True, cpu_budget=1.0,
                           diagnostic=False, gpus=1)
    line = bench_modes.run_pipeline(a, 2, emit=False)
    out = {"case": tag, "qps": round(line["value"], 1), "ms_per_step": line["ms_per_step"],
           "host_enqueue_ms_per_step": line.get("host_enqueue_ms_per_step")}
    out.update(extra or {})
    print(json.dumps(out), flush=True)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    x = torch.zeros(1, device=dev)
    cases = os.environ.get("CASES", "fresh,streams1,streams1+whole,headline,headline+whole,"
                                    "fresh,fresh+whole").split(",")
    keep = []
    for c in cases:
        part = "whole" if c.endswith("+whole") else "auto"
        base = c.split("+")[0]
        if base.startswith("streams") and c.endswith("+whole"):
            leg(c, {"live_extra_streams": len(keep)}, part)     # the state as it is, whole streams
        elif base == "headline" and c.endswith("+whole"):
            leg(c, {"live_extra_streams": len(keep)}, part)
        elif c.startswith("streams"):
            n = int(c[7:].split("_")[0])
            ss = [torch.cuda.Stream(dev) for _ in range(n)]
            for s in ss:
                with torch.cuda.stream(s):
                    x.add_(1)
            torch.cuda.synchronize()
            if c.endswith("_freed"):
                del ss
                gc.collect()
            else:
                keep += ss
            leg(c, {"live_extra_streams": len(keep)})
        elif c == "headline":
            from ragmi.dist import ShardedIndex
            import bench
            sh = ShardedIndex(10_000_000, dim=384, device=dev)
            bench.build_shard(sh.local, sh.lo, sh.hi, 10_000_000, dev)
            qs, _ = bench.make_queries(10, 10_000_000, dev)
            s2 = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
            for i, q in enumerate(qs):
                with torch.cuda.stream(s2[i % 2]):
                    sh.search(q, 15)
            torch.cuda.synchronize()
            sh.local.close()
            del sh, qs
            torch.cuda.empty_cache()
            keep.append(s2[1])
            leg(c, {"live_extra_streams": len(keep)})
        else:
            leg(c, {"live_extra_streams": len(keep)}, part)


if __name__ == "__main__":
    main()
