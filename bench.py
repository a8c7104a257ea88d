"""bench.py — queries/sec + recall@5 of batched cosine top-k over a 10M x 384 fp16 corpus.

Metric (BASELINE.json): "queries/sec + recall@5, batch=32 over 10M x 384 corpus at 1/2/4/8
MI355X". One step = one batch of 32 queries through the hot path that replaces
`retrieve_from_qdrant` (reference main.py:215-239; batched as main2.py:281-295 would):
query normalisation -> HIP MFMA scan of the local shard with per-wave top-k -> exact
rescoring merge -> (N > 1) RCCL all-gather of the per-shard top-15 over xGMI + GPU merge.
The corpus is fixed at 10M rows and sharded over the N ranks (strong scaling), contiguous
row ranges, identical data for every N (1M-row chunks, each from its own seed).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       N > 1 either under a launcher that sets WORLD_SIZE / RANK / LOCAL_RANK
       (python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...), or
       plain `python bench.py --gpus N`: the process then starts N rank processes itself
       (launch_ranks) before anything touches the GPU, and exits with their status.
       WORLD_SIZE set but != N is an error (exit 2): the line's n_gpus is what ran.
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

D = 384
K_TOP = 15          # limit=15, main.py:215
B = 32              # MAX_BATCH_SIZE, main2.py:51
CHUNK = 1_000_000
HBM_PEAK = 8.0e12   # B/s, MI355X_MICROARCH.md chip table (spec)
# scan-kernel HIP events on every PROF_EVERY-th step of the timed region (an event record
# idles the queue for a few us; sampling keeps the timed steps unperturbed)
PROF_EVERY = 4


def gen_chunk(c: int, dev, rows: int = CHUNK) -> torch.Tensor:
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + c)
    return torch.randn((rows, D), generator=g, device=dev, dtype=torch.float32)


def chunk_rows(c, n_total):
    return min(CHUNK, n_total - c * CHUNK)


def build_shard(idx, lo, hi, n_total, dev):
    """Upsert global rows [lo, hi) into the local index as local rows [0, hi-lo)."""
    c0, c1 = lo // CHUNK, (hi - 1) // CHUNK
    for c in range(c0, c1 + 1):
        x = gen_chunk(c, dev, chunk_rows(c, n_total))
        a, b = max(lo, c * CHUNK), min(hi, c * CHUNK + x.shape[0])
        rows = torch.arange(a - lo, b - lo, device=dev, dtype=torch.int64)
        idx.upsert(x[a - c * CHUNK:b - c * CHUNK], rows, new_count=max(idx.count, b - lo))
        del x
    torch.cuda.synchronize()


def make_queries(n_batches, n_total, dev):
    """Planted queries: a corpus row + 0.05 N(0,1) noise; every 4th batch is
    pure random (the non-planted case)."""
    rng = np.random.default_rng(1)
    picks = rng.integers(0, n_total, (n_batches, B))
    need = sorted(set((picks // CHUNK).ravel().tolist()))
    rows = {}
    for c in need:
        x = gen_chunk(c, dev, chunk_rows(c, n_total))
        sel = picks[(picks // CHUNK) == c]
        for r in np.unique(sel):
            rows[int(r)] = x[int(r) - c * CHUNK].clone()
        del x
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    qs = []
    for i in range(n_batches):
        base = torch.stack([rows[int(r)] for r in picks[i]])
        noise = torch.randn((B, D), generator=g, device=dev)
        q = base + 0.05 * noise if i % 4 != 3 else noise
        qs.append(q.contiguous())
    return qs, picks


def cpu_baseline(corpus16_sample: np.ndarray, q: np.ndarray, n_total: int, budget_s=10.0):
    """Reference CPU path restated: numpy fp32 Q @ C^T + argpartition top-15 on
    the host cores, over a bounded sample of the corpus; scaled to the full corpus."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_scan as O
    try:
        from threadpoolctl import threadpool_info
        cores = max([p.get("num_threads", 1) for p in threadpool_info()
                     if p.get("user_api") == "blas"] or [os.cpu_count()])
    except Exception:
        cores = os.cpu_count()
    c32 = corpus16_sample.view(np.float16).astype(np.float32)
    qn = O.normalize(q)
    t0 = time.perf_counter()
    reps = 0
    while True:
        s = qn @ c32.T
        part = np.argpartition(-s, K_TOP - 1, axis=1)[:, :K_TOP]
        top = np.take_along_axis(s, part, axis=1)
        _ = np.take_along_axis(part, np.argsort(-top, axis=1), axis=1)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    t_batch_full = el / reps * (n_total / c32.shape[0])
    return {"value": round(B / t_batch_full, 3), "unit": "queries/s", "cores": int(cores),
            "kind": "port",
            "sample": f"{c32.shape[0]} of {n_total} rows x {B} queries, {reps} reps "
                      f"({el:.1f} s), numpy fp32 matmul + argpartition top-{K_TOP}, "
                      f"scaled linearly to {n_total} rows"}


def scan_traffic(rows_per_gpu: int, storage: str = "fp16", path: str | None = None,
                 kind: str = "scan_384"):
    """HBM bytes per scan launch from the committed rocprofv3 --pmc FETCH_SIZE passes
    (profiles/scan_pmc.json, written by scripts/profile.sh; x2 gfx950 correction), keyed by
    the rows one launch scans: a rank's shard of R rows runs the same launch as a 1-GPU run
    of `bench.py --rows R`. Returns (bytes, source) or (None, None) when no pass matches."""
    path = path or os.path.join(ROOT, "profiles", "scan_pmc.json")
    try:
        with open(path) as f:
            p = json.load(f)
    except (OSError, ValueError):
        return None, None
    if kind == "scan_384":
        table = dict(p.get("by_rows_per_gpu", {}))
        if "hbm_bytes_per_launch" in p:             # the headline pass (10M rows per GPU)
            table.setdefault(str(p.get("rows_per_gpu", 10_000_000)), p)
    else:                                           # wide_1024 (config 5), filtered_384
        table = dict(p.get(f"by_rows_{kind}", {}))
    e = table.get(str(int(rows_per_gpu)))
    if storage != "fp16" or not e or e.get("hbm_bytes_per_launch") is None:
        return None, None
    return e["hbm_bytes_per_launch"], (
        "not measured in this run: rocprofv3 --pmc FETCH_SIZE pass (x2 gfx950 correction) "
        f"of a scan launch over {int(rows_per_gpu)} rows, " + str(e.get("source")) + ", " +
        str(e.get("commit", "")))


def recall_fp32(q, gpu_ids, lo, hi, n_total, rank, world, dev, qchunk=512):
    """recall@5 against the UNROUNDED corpus ("also report recall vs the unrounded
    fp32 corpus") for every query of q [n, D]: each rank regenerates its rows in fp32, scores
    them against the fp32 queries (both L2-normalised, as Qdrant COSINE does at insert) with a
    torch fp32 matmul, keeps a running top-15; rank 0 merges the shards. Measurement only,
    outside the timed region. Returns per-query recall (rank 0) or None."""
    qn = torch.nn.functional.normalize(q.float(), dim=1)
    nq = q.shape[0]
    best_s = torch.full((nq, 0), float("-inf"), device=dev)
    best_i = torch.zeros((nq, 0), dtype=torch.int64, device=dev)
    for c in range(lo // CHUNK, (hi - 1) // CHUNK + 1):
        x = gen_chunk(c, dev, chunk_rows(c, n_total))
        a, b = max(lo, c * CHUNK), min(hi, c * CHUNK + x.shape[0])
        xs = torch.nn.functional.normalize(x[a - c * CHUNK:b - c * CHUNK], dim=1)
        ts, ti = [], []
        for q0 in range(0, nq, qchunk):
            sc = qn[q0:q0 + qchunk] @ xs.T
            s_, i_ = torch.topk(sc, K_TOP, dim=1)
            ts.append(s_)
            ti.append(i_ + a)
            del sc
        best_s = torch.cat([best_s, torch.cat(ts)], 1)
        best_i = torch.cat([best_i, torch.cat(ti)], 1)
        best_s, o = torch.topk(best_s, K_TOP, dim=1)
        best_i = torch.gather(best_i, 1, o)
        del x, xs
    mine = (best_s.cpu().numpy(), best_i.cpu().numpy())
    parts = [mine]
    if world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, mine)
    if rank != 0:
        return None
    S = np.concatenate([p[0] for p in parts], axis=1)
    I = np.concatenate([p[1] for p in parts], axis=1)
    top5 = np.take_along_axis(I, np.argsort(-S, axis=1, kind="stable")[:, :5], axis=1)
    return np.array([len(set(gpu_ids[b, :5]) & set(top5[b])) / 5 for b in range(nq)])


def verify_exact(idx, q, gpu_s, gpu_ids, lo, rank, world, dev):
    """Certified check of EVERY timed batch against the oracle (oracle/oracle_scan.py,
    canonical arithmetic of scan_ref.c), after the timed region:
      1. each returned row is rescored exactly on the rank that holds it; floor_q = the
         worst of the 15 (a lower bound of the true 15th-best score);
      2. every rank collects its rows with exact score >= floor_q (BLAS superset + exact
         rescoring: oracle_scan.candidates_above), rank 0 merges them by (score desc, row
         asc) = the exact top-15 of the whole corpus.
    Returns (per-query recall@5, per-query exact-match flags) on rank 0, else None."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_scan as O
    enc = idx.export_rows32() if getattr(idx, "storage", "fp16") == "fp32" else idx.export_rows()
    qn = O.normalize(q)
    own = (gpu_ids >= lo) & (gpu_ids < lo + enc.shape[0])
    e_gpu = O.rescore(enc, qn, np.where(own, gpu_ids - lo, -1))
    if world > 1:
        t = torch.from_numpy(e_gpu).to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        e_gpu = t.cpu().numpy()
    floor = e_gpu.min(axis=1)
    mine = O.candidates_above(enc, qn, floor, row_offset=lo)
    parts = [mine]
    if world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, mine)
    if rank != 0:
        return None
    r5 = np.zeros(len(q))
    ok = np.zeros(len(q), bool)
    for j in range(len(q)):
        ids = np.concatenate([p[j][0] for p in parts])
        sc = np.concatenate([p[j][1] for p in parts])
        order = np.lexsort((ids, -sc.astype(np.float64)))[:K_TOP]
        ref_i, ref_s = ids[order], sc[order]
        r5[j] = len(set(gpu_ids[j, :5].tolist()) & set(ref_i[:5].tolist())) / 5
        ok[j] = np.array_equal(ref_i, gpu_ids[j]) and np.array_equal(ref_s, gpu_s[j])
    return r5, ok


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str], cmd: list[str] | None = None,
                 env: dict | None = None, poll_s: float = 0.05) -> int:
    """Start `n` rank processes of this script (or of `cmd`) on this node with the env
    contract of torch.distributed.run — RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE
    = n, MASTER_ADDR 127.0.0.1, a free MASTER_PORT — and wait for them. The parent never
    initialises the GPU (it only imports torch) and never execs: children are plain
    subprocesses. If a rank fails, the others are terminated and its exit status returned
    (a signal death -s as 128 + s); 0 when every rank exits 0."""
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", GROUP_WORLD_SIZE="1",
                HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + list(argv)
    procs = [subprocess.Popen(cmd, env=dict(base, RANK=str(r), LOCAL_RANK=str(r),
                                            ROLE_RANK=str(r)))
             for r in range(n)]

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    rc = 0
    try:
        live = set(range(n))
        while live:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    stop()
            if live:
                time.sleep(poll_s)
    finally:
        stop()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        signal.signal(signal.SIGTERM, old)
    return rc


def check_world(gpus: int, environ=None) -> int:
    """World size the run will have: WORLD_SIZE when a launcher set it (it must equal --gpus),
    else --gpus (launch_ranks starts the ranks when > 1). Raises SystemExit(2) on mismatch."""
    environ = os.environ if environ is None else environ
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" in environ:
        w = int(environ["WORLD_SIZE"])
        if w != gpus:
            print(f"bench.py: WORLD_SIZE={w} from the launcher but --gpus {gpus}; refusing "
                  "to report a line whose n_gpus differs from the request", file=sys.stderr)
            raise SystemExit(2)
        return w
    return gpus


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 50; --config 2 / 3: 200)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps (default 20 — 30 vs 5 measured +0.2-0.3%% on the headline, "
                         "profiles/r06k_warmup_ab.jsonl; --config 2 / 3: 20 — the encoder's "
                         "hipGraphs are captured per padded shape and per stream, so the "
                         "pipelines need a few batches per stream to reach steady state)")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--no-recall", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--streams", type=int, default=0,
                    help="batches in flight (0 = by shard size: 4 below 4M rows per GPU, "
                         "else 2)")
    ap.add_argument("--scan-order", choices=["auto", "serial", "free", "stream"], default="auto",
                    help="serial: each batch's scan waits for the previous batch's scan "
                         "(rag_index_set_scan_order); free: scans on different streams overlap")
    ap.add_argument("--prof-every", type=int, default=0,
                    help="time every n-th scan launch (0 = auto: every launch when scans of "
                         "several streams overlap, else every %d-th)" % PROF_EVERY)
    ap.add_argument("--storage", choices=["fp16", "fp32"], default="fp16",
                    help="vector storage (rag_index_create_ex): fp16 (the metric's fp16 corpus) "
                         "or fp32 (Qdrant's default Float32 datatype: exact scores on the fp32 "
                         "rows, the scan on their fp16 copy)")
    ap.add_argument("--config", choices=["4", "2", "3", "5", "filtered"], default="4",
                    help="4 (default): the headline 10M x 384 line (BASELINE configs[3] at N "
                         "GPUs); 2 / 3: encode + search (+ rerank) pipeline over 1M x 384; "
                         "5: 50M x 1024 at batch 128; filtered: 10M x 384 with per-query "
                         "ticker filters (scripts/bench_modes.py)")
    ap.add_argument("--diagnostic", action="store_true",
                    help="create the index with RAG_CREATE_DIAGNOSTIC, so the RAGMI_* kernel "
                         "A/B knobs are honoured (never for a reported line)")
    ap.add_argument("--precision", choices=["fp16x3", "fp16"], default="fp16x3",
                    help="encoder precision for --config 2/3 (fp16x3 = the 1e-3 contract)")
    ap.add_argument("--partition", choices=["auto", "on", "off", "whole"], default="auto",
                    help="batches in flight on CU-partitioned streams (rag_stream_create_cu_"
                         "partition): auto = with free scan order and several in flight "
                         "(shards below 4M rows per GPU)")
    ap.add_argument("--no-configs", action="store_true",
                    help="default line without the config-2 / config-3 legs (profiling runs: "
                         "their 1M-row scans share the headline scan kernel's name)")
    ap.add_argument("--certify", action="store_true",
                    help="--config 5: certify EVERY timed batch exact after the timed region "
                         "(oracle rescoring + an fp32 GEMM superset; scripts/bench_modes.py "
                         "_certify_all) instead of recall on two batches")
    ap.add_argument("--legs", choices=["child", "inproc"], default="inproc",
                    help="where the default line's config-2 / config-3 legs run: inside this "
                         "process after the headline's index is freed (default: the serving "
                         "shape, one process holding the index and both encoders; VERDICT r5 "
                         "item 4), or a fresh child process each. With the pipelines' batch "
                         "streams on dedicated hardware queues the two agree within 1%% "
                         "(profiles/r06_legs/)")
    ap.add_argument("--config-steps", type=int, default=200,
                    help="timed batches of each config-2 / config-3 leg (warmup 20)")
    args = ap.parse_args()
    pipeline = args.config in ("2", "3")
    if args.steps is None:
        args.steps = 200 if pipeline else 50
    if args.warmup is None:
        args.warmup = 20
    world = check_world(args.gpus)
    if world > 1 and "WORLD_SIZE" not in os.environ:
        # plain `python bench.py --gpus N`: one rank process per GPU, started before this
        # process touches the GPU; rank 0 prints the line
        sys.exit(launch_ranks(world, sys.argv[1:]))
    if args.config != "4":
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import bench_modes
        if args.rows == 10_000_000:
            args.rows = 0            # each mode's own default size
        return bench_modes.run(args)

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    backend, ranks_seen = None, 1
    # RAGMI_DIST_REHEARSAL=1 (one GPU, diagnostic): a world-1 process group whose packed
    # all-gather + GPU merge still run every batch (ShardedIndex force_exchange), so the RCCL
    # stream's interplay with the batches in flight can be measured on a one-GPU box
    rehearsal = world == 1 and os.environ.get("RAGMI_DIST_REHEARSAL") == "1"
    if world > 1 or rehearsal:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        backend = os.environ.get("RAGMI_DIST_BACKEND", "nccl")   # nccl = RCCL over xGMI
        if rehearsal:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # RCCL's communicator is created lazily (no device_id: at the first collective, after
        # the shard is built). Created eagerly here, before the corpus allocation, its buffers
        # left the 960 MB shard with a placement that scans ~8% slower: 1.25M rows, 4 in flight,
        # plain search 184K vs 201K qps, the same with the communicator created after the
        # shard 201K (scripts/rccl_exchange_probe.py, profiles/r03w_rccl_probe.jsonl)
        dist.init_process_group(backend)
        backend = dist.get_backend()
        ranks_seen = dist.get_world_size()
        if ranks_seen != world:
            raise SystemExit(f"bench.py: process group has {ranks_seen} ranks, expected {world}")

    from ragmi.dist import ShardedIndex
    from ragmi.index import busy_union_ms

    n_total = args.rows
    sh = ShardedIndex(n_total, dim=D, device=dev, storage=args.storage, force_exchange=rehearsal,
                      diagnostic=args.diagnostic)
    idx, lo, hi = sh.local, sh.lo, sh.hi
    build_shard(idx, lo, hi, n_total, dev)
    nb = args.warmup + args.steps
    qs, _ = make_queries(nb, n_total, dev)

    # Consecutive batches alternate over `--streams` HIP streams (a serving loop keeps more
    # than one batch in flight): batch i+1's query prep / seed sampling / scan start run beside
    # batch i's scan tail and select. Each stream owns its own search workspace
    # (rag_index_search), so no cross-stream synchronisation is needed; the timed region still
    # ends with a device-wide synchronize.
    # Default depth by shard size: a scan launch has a fixed ramp/tail (~30 us) and a batch
    # ~35 us of latency-bound work around it (query prep, seed sampling, select, exchange) —
    # 3% of a 10M-row step but ~20% of a 1.25M-row one (8-GPU shard). Measured on one MI355X
    # (profiles/r01c_streams.txt), qps by batches in flight 1/2/3/4: 1.25M rows 146K / 177K /
    # 185K / 196K; 2.5M 89K / 99K / - / 103K; 5M 49.8K / 54.1K / - / 53.4K; 10M 26.5K / 27.9K /
    # - / 27.7K. Shards below 4M rows keep 4 in flight, larger ones 2. Not more than 4: a
    # process gets 4 hardware queues (GPU_MAX_HW_QUEUES), and 6 or 8 streams sharing them
    # measured 149K against 210K qps at 1.25M rows (profiles/r01f_small_shard_streams.jsonl).
    # Scan order (rag_index_set_scan_order): at >= 4M rows per GPU the scans are chained
    # (serial) so only the ~40 us of per-batch prep / seeding / select overlaps another batch's
    # scan and every scan launch runs alone on HBM — 10M rows, 2 in flight: 27.4K qps with the
    # scan at 83.2% of the roofline (free order 27.5K but each scan 3% longer; 1 in flight
    # 26.8K); small shards keep free order, where overlapping scan ramps/tails is the gain
    # (1.25M rows, 4 in flight: 195K free vs 193K serial) — profiles/r01h_scan_order.jsonl.
    rows_local = hi - lo
    n_streams = args.streams or (4 if rows_local < 4_000_000 else 2)
    serial = args.scan_order == "serial" or (args.scan_order == "auto"
                                             and rows_local >= 4_000_000)
    if args.scan_order == "stream":
        serial = True
        idx.set_scan_order(2)
    else:
        idx.set_scan_order(serial)
    # Spatial partition (round 5): with free order and several batches in
    # flight, each batch's stream owns 1/n of the CUs and its scan one workgroup per CU of
    # them, so the scans run side by side instead of interleaving over every CU — 1.25M rows,
    # 4 in flight: 222-223K qps vs 206-208K (scripts/diag/cu_partition.py,
    # profiles/r05c_cu_partition.jsonl)
    partition = whole = None
    use_part = args.partition == "on" or (args.partition == "auto" and not serial
                                          and n_streams > 1)
    if use_part:
        from ragmi.index import PartitionStreams
        partition = PartitionStreams(dev, n_streams)
        streams = list(partition.streams)
        for s in streams:
            s.wait_stream(torch.cuda.current_stream(dev))   # the queries were made there
    elif args.partition == "whole":
        # every batch stream on a dedicated hardware queue (full-CU-mask streams)
        from ragmi.index import PartitionStreams
        whole = PartitionStreams(dev, n_streams, whole=True)
        streams = list(whole.streams)
        for s in streams:
            s.wait_stream(torch.cuda.current_stream(dev))
    else:
        streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev)
                                                      for _ in range(n_streams - 1)]
    n_step = [0]

    def step(q):
        s = streams[n_step[0] % len(streams)]
        n_step[0] += 1
        if s is not streams[0] and n_step[0] <= len(streams):
            s.wait_stream(streams[0])      # first use: the queries were made on stream 0
        with torch.cuda.stream(s):
            return sh.search(q, K_TOP)

    for w in range(args.warmup):
        step(qs[w])
    torch.cuda.synchronize()
    tier1_0, tier2_0, _ = idx.exactness_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # free scan order with several batches in flight: the scans of different streams overlap
    # in time, so every launch is timed and the kernel's device time is the union of their
    # event intervals (overlap counted once); otherwise launches never overlap and a sample of
    # every PROF_EVERY-th one gives the same per-launch time
    overlapped = len(streams) > 1 and not serial
    prof_every = args.prof_every or (1 if overlapped else PROF_EVERY)
    overlapped = overlapped and prof_every == 1      # a sample of one stream never overlaps
    idx.profile(prof_every)
    outs = []
    t0 = time.perf_counter()
    for k in range(args.steps):
        outs.append(step(qs[args.warmup + k]))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    idx.profile(False)
    tier1, tier2, _ = idx.exactness_stats()
    tier1, tier2 = tier1 - tier1_0, tier2 - tier2_0
    t_a, t_b = idx.profile_scan_intervals()
    launches = len(t_a)
    scan_avg_ms = float((t_b - t_a).sum()) / max(launches, 1)     # per-launch event duration
    busy_ms = busy_union_ms(t_a, t_b) / max(launches, 1)           # device time per launch
    # With several batches in flight a scan launch shares HBM with the other batches' scans,
    # so its duration over the timed region is not the kernel's own rate: time the same
    # workload once more on ONE stream (after the timed region, not part of `value`). Serial
    # scan order already keeps every scan launch alone.
    alone_ms = scan_avg_ms
    if partition is not None:
        alone_ms = None        # a partition's scan alone runs on 1/n of the CUs: not comparable
    elif len(streams) > 1 and not serial:
        torch.cuda.synchronize()
        idx.profile(True)
        for k in range(min(args.steps, 20)):
            sh.search(qs[args.warmup + k], K_TOP)
        torch.cuda.synchronize()
        idx.profile(False)
        a_ms, a_n = idx.profile_scan_ms()
        alone_ms = a_ms / max(a_n, 1)
    if world > 1:
        t = torch.tensor([elapsed, scan_avg_ms, alone_ms or 0.0, busy_ms], device=dev,
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, scan_avg_ms, alone_ms, busy_ms = (float(v) for v in t.tolist())
        alone_ms = alone_ms if partition is None else None

    check = None
    if not args.no_recall:
        # every timed batch (planted and pure-random), after the timed region
        q_all = torch.cat(qs[args.warmup:args.warmup + args.steps])
        g_s = torch.cat([o[0] for o in outs]).cpu().numpy()
        g_i = torch.cat([o[1] for o in outs]).cpu().numpy()
        res = verify_exact(idx, q_all.cpu().numpy(), g_s, g_i, lo, rank, world, dev)
        r32 = recall_fp32(q_all, g_i, lo, hi, n_total, rank, world, dev)
        if rank == 0:
            r5, ok = res
            per_b = r5.reshape(args.steps, B).mean(1)
            ok_b = ok.reshape(args.steps, B).all(1)
            f32_b = r32.reshape(args.steps, B).mean(1)
            check = {"recall_at_5": round(float(r5.mean()), 6),
                     "recall_at_5_min": round(float(per_b.min()), 6),
                     "exact_batches": f"{int(ok_b.sum())}/{args.steps}",
                     "recall_at_5_vs_fp32_corpus": round(float(r32.mean()), 6),
                     "recall_at_5_vs_fp32_corpus_min": round(float(f32_b.min()), 6)}

    cpu = None
    if rank == 0 and not args.no_cpu:
        # at every N (north_star: the CPU path "in the same run"), rank 0, after the timed
        # region: the whole-corpus CPU rate, from a sample of rank 0's shard
        sample = idx.export_rows(0, min(CHUNK, hi - lo))
        cpu = cpu_baseline(sample, qs[args.warmup].cpu().numpy(), n_total, args.cpu_budget)
    if world > 1:
        dist.barrier()

    if rank == 0:
        local_rows = hi - lo
        algo_bytes = local_rows * D * 2                      # (N/G)*D*2 per batch
        # achieved = algorithmic bytes per launch / device time per launch, where launches that
        # overlap in time (free order, several batches in flight) count their common time once
        # (the union of the launches' HIP-event intervals over the timed region, / launches);
        # without overlap this IS the average launch duration (avg_ms)
        achieved = algo_bytes / (busy_ms * 1e-3)
        traffic, traffic_source = scan_traffic(local_rows, args.storage)
        if partition is not None:
            # the PMC FETCH_SIZE of a CU-partitioned scan launch reads 0.50x its algorithmic
            # bytes after the x2 correction (profiles/scan_pmc.json partitioned_by_rows_per_gpu)
            # — below what the launch must read, so not a traffic measurement
            traffic, traffic_source = None, ("not reported: PMC FETCH_SIZE under-counts the "
                                             "CU-partitioned scan launch (DESIGN R5.3)")
        qps = B * args.steps / elapsed
        line = {
            "metric": "queries/sec + recall@5, batch=32 over 10Mx384 corpus",
            "value": round(qps, 2),
            "unit": "queries/s",
            "n_gpus": world,
            "backend": backend,            # torch.distributed backend ("nccl" = RCCL); None at N=1
            "ranks_seen": ranks_seen,      # dist.get_world_size() of the process group
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp16",
            "data": "synthetic (torch randn corpus, 1M-row chunks seeded 1000+c; planted "
                    "queries = corpus row + 0.05 N(0,1), every 4th batch pure random)",
            "config": {"workload": f"cosine top-{K_TOP} over {n_total}x{D} fp16 corpus, "
                                   f"batch={B}, {world} shard(s)" +
                                   (" + RCCL all-gather merge" if world > 1 else
                                    " + world-1 exchange rehearsal" if rehearsal else ""),
                       "corpus_rows": n_total, "dim": D, "batch": B, "k": K_TOP,
                       "rows_per_gpu": local_rows, "parallelism": f"corpus-shard{world}",
                       "batches_in_flight": n_streams, "storage": args.storage,
                       "scan_order": args.scan_order if args.scan_order == "stream" else
                                     "serial" if serial else "free",
                       "cu_partition": len(streams) if partition is not None else None,
                       "stream_queues": ("CU partitions" if partition is not None else
                                         "dedicated (whole-CU-mask streams)" if whole is not None
                                         else "torch streams")},
            "recall_at_5": check and check["recall_at_5"],
            "recall_at_5_min": check and check["recall_at_5_min"],
            "exact_batches": check and check["exact_batches"],
            "top15_exact_vs_oracle": check and check["exact_batches"] == f"{args.steps}/{args.steps}",
            "recall_at_5_vs_fp32_corpus": check and check["recall_at_5_vs_fp32_corpus"],
            "recall_at_5_vs_fp32_corpus_min": check and check["recall_at_5_vs_fp32_corpus_min"],
            "exactness_fallbacks": {"queries": B * args.steps, "tier1_list_rescoring": tier1,
                                    "tier2_second_pass": tier2},
            # a diagnostic run (--diagnostic: the RAGMI_* kernel A/B knobs honoured) says which
            # knobs it ran with; production lines carry null
            "diagnostic_knobs": ({k: v for k, v in os.environ.items() if k.startswith("RAGMI_")}
                                 if args.diagnostic else None),
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 1),
                         "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK, 4),
                         "traffic": traffic, "traffic_source": traffic_source,
                         "kernel": "scan_kernel<384,false>",
                         "time_basis": ("union of the scan launches' HIP-event intervals "
                                        "over the timed region / launches" if overlapped else
                                        "average scan launch duration (HIP events)"),
                         "busy_ms_per_launch": round(busy_ms, 4),
                         "avg_ms": round(scan_avg_ms, 4),
                         # avg_ms counts overlapping launches' shared time once per launch
                         "frac_of_avg_launch": round(algo_bytes / (scan_avg_ms * 1e-3) / HBM_PEAK, 4),
                         "algorithmic_bytes_per_launch": algo_bytes,
                         # whole-step view: the shard's bytes per batch over the step time
                         "step_frac": round(algo_bytes / (elapsed / args.steps) / HBM_PEAK, 4),
                         # the same launch timed alone (differs from avg_ms only when several
                         # batches are in flight and their scans overlap)
                         "standalone_avg_ms": round(alone_ms, 4) if alone_ms else None,
                         "standalone_frac": (round(algo_bytes / (alone_ms * 1e-3) / HBM_PEAK, 4)
                                             if alone_ms else None)},
            "cpu_baseline": cpu,
        }
    idx.close()
    for ps in (partition, whole):
        if ps is not None:
            ps.close()
    if world > 1 or rehearsal:
        dist.destroy_process_group()
    if rank == 0:
        # the default run also measures the end-to-end configs 2 and 3
        # (BASELINE configs[1] / [2]: encode + search (+ CE rerank) of 32 query strings over
        # 1M x 384) after the headline's timed region, each with its own parity legs,
        # rooflines and CPU baseline, as extra keys; value / ms_per_step stay the headline's.
        # N = 1 only (at N > 1 every rank would run its own replica of them).
        legs_on = world == 1 and not rehearsal and not args.no_configs
        leg_fn = _config_leg_inproc if args.legs == "inproc" else _config_leg
        for cfg in ("2", "3"):
            line[f"config{cfg}"] = (leg_fn(args, cfg) if legs_on else
                                    {"skipped": "--no-configs" if args.no_configs else
                                     "N > 1 (measured by the N = 1 run)"})
        print(json.dumps(line), flush=True)


LEG_KEYS = ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "dtype", "config",
            "search_top15_exact_queries", "encode_max_abs_diff_vs_oracle",
            "rerank_max_abs_diff_vs_oracle", "rerank_checked_queries",
            "rerank_top5_order_matches", "checked_timed_batches", "roofline", "roofline_search",
            "cpu_baseline", "id_input_qps", "text_vs_id_input", "host_enqueue_ms_per_step")


def _config_leg_inproc(args, cfg: str) -> dict:
    """The same leg inside this process (--legs inproc): bench_modes.run_pipeline builds the
    1M-row index, bge-small and the cross-encoder here, after the headline's index was freed."""
    import copy
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench_modes
    a = copy.copy(args)
    a.config, a.steps, a.warmup, a.rows, a.streams, a.partition = cfg, args.config_steps, 20, 0, 0, "auto"
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    try:
        full = bench_modes.run_pipeline(a, int(cfg), emit=False)
    except Exception as e:                              # the headline line still prints
        return {"error": f"config {cfg} leg (in process): {type(e).__name__}: {e}"}
    leg = {k: full[k] for k in LEG_KEYS if k in full}
    leg["wall_s"] = round(time.perf_counter() - t0, 1)
    leg["process"] = "in-process (after the headline)"
    return leg


def _config_leg(args, cfg: str) -> dict:
    """One config-2 / config-3 measurement (`bench.py --config 2|3`, scripts/bench_modes.py) as
    a dict of the keys a reader compares: qps, ms per batch, the certified parity legs,
    rooflines, the CPU baseline — in a child process (--legs child). Round 5 ran the legs this
    way because config 2 lost ~21% inside the headline's process; round 6 traced that to the
    batch streams sharing hardware queues and gave them dedicated queues, so
    the default is now in process (_config_leg_inproc)."""
    torch.cuda.empty_cache()
    cmd = [sys.executable, "-u", os.path.abspath(__file__), "--config", cfg,
           "--steps", str(args.config_steps), "--warmup", "20", "--precision", args.precision,
           "--cpu-budget", str(args.cpu_budget)]
    cmd += [f for f, on in (("--no-cpu", args.no_cpu), ("--no-recall", args.no_recall),
                            ("--diagnostic", args.diagnostic)) if on]
    print(f"bench.py: headline done; config {cfg} leg ({args.config_steps} batches)",
          file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True, timeout=900)
    except (subprocess.TimeoutExpired, OSError) as e:
        # the headline is already measured: a hung or unstartable leg must not lose its line
        return {"error": f"config {cfg} leg: {type(e).__name__}: {e}"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"config {cfg} leg exited {r.returncode}"}
    full = json.loads(lines[-1])
    leg = {k: full[k] for k in LEG_KEYS if k in full}
    leg["wall_s"] = round(time.perf_counter() - t0, 1)
    leg["process"] = "child"
    return leg

if __name__ == "__main__":
    main()
