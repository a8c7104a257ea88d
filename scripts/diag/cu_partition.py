"""Spatial partitioning of the batches in flight (VERDICT r4 item 3 probe): at the 8-GPU shard
size (1.25M x 384 rows) with 4 batches in flight, each batch's stream gets its own quarter of
the CUs (hipExtStreamCreateWithCUMask) and the scan a grid sized for it, so the four scans run
side by side on disjoint CUs instead of all four interleaving over every CU; the scan's
launch ramp and tail then amortise over a 4x longer launch. Prints one JSON line: qps over
the timed batches, and whether every timed batch's ids and scores equal the unpartitioned
run's (the exact top-k does not depend on the grid).
Usage (GPU box): RAGMI_SCAN_WGS=<wgs> python scripts/diag/cu_partition.py <parts> [rows]"""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

import bench  # noqa: E402
from ragmi.index import FlatIndex  # noqa: E402


def _hip():
    """the HIP runtime torch loaded (a second copy would own different streams)"""
    for ln in open("/proc/self/maps"):
        p = ln.split()[-1]
        if "libamdhip64.so" in p:
            return ctypes.CDLL(p)
    raise RuntimeError("libamdhip64 not loaded")


def masked_streams(parts, n_cu, dev):
    hip = _hip()
    words = (n_cu + 31) // 32
    out = []
    per = n_cu // parts
    for p in range(parts):
        bits = [0] * words
        for cu in range(p * per, (p + 1) * per):
            bits[cu // 32] |= 1 << (cu % 32)
        arr = (ctypes.c_uint32 * words)(*bits)
        s = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), arr)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
        out.append(torch.cuda.ExternalStream(s.value, device=dev))
    return out


def main():
    parts = int(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_250_000
    steps, warm = 200, 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    idx = FlatIndex(bench.D, n, dev, diagnostic=True)
    bench.build_shard(idx, 0, n, n, dev)
    qs, _ = bench.make_queries(steps + warm, n, dev)
    if parts > 1:
        streams = masked_streams(parts, n_cu, dev)
    else:
        streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(3)]
    cur = torch.cuda.current_stream(dev)
    for s in streams:
        s.wait_stream(cur)

    def run(i):
        s = streams[i % len(streams)]
        with torch.cuda.stream(s):
            return idx.search(qs[i], bench.K_TOP)

    for i in range(warm):
        run(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = [run(warm + k) for k in range(steps)]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # reference: the same batches one at a time on the default stream, full grid
    same = True
    for k in range(0, steps, 20):
        s_ref, i_ref = idx.search(qs[warm + k], bench.K_TOP)
        torch.cuda.synchronize()
        same &= bool(torch.equal(i_ref, outs[k][1]) and torch.equal(s_ref, outs[k][0]))
    print(json.dumps({"parts": parts, "rows": n, "streams": len(streams),
                      "scan_wgs_env": os.environ.get("RAGMI_SCAN_WGS"),
                      "qps": round(bench.B * steps / el, 1), "ms_per_batch": round(el / steps * 1e3, 4),
                      "same_as_reference": same, "n_cu": n_cu}), flush=True)
    idx.close()


if __name__ == "__main__":
    main()
