#!/bin/bash
# the per-rank workloads of the driver's N = 2 / 4 / 8 runs on one GPU, through the RCCL
# exchange (RAGMI_DIST_REHEARSAL=1: world-1 nccl group, packed all-gather + merge per batch):
# 10M / N rows per rank; plus config 5's per-rank shard at N = 8 (6.25M x 1024, batch 128)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; out=gpurun_out/per_rank.jsonl; : > $out
for rows in 5000000 2500000 1250000; do
  RAGMI_DIST_REHEARSAL=1 timeout -k 10 300 python3 -u bench.py --rows $rows --steps 200 --warmup 10 2> gpurun_out/pr.err | grep '^{' >> $out || { tail -20 gpurun_out/pr.err; exit 1; }
done
timeout -k 10 400 python3 -u bench.py --config 5 --rows 6250000 --no-cpu 2> gpurun_out/pr5.err | grep '^{' >> $out || { tail -20 gpurun_out/pr5.err; exit 1; }
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); r=d.get('roofline') or {}; c=d['config']
    print(c.get('rows_per_gpu'), d['value'], d.get('backend'), r.get('frac'), d.get('exact_batches'), d.get('recall_at_5_vs_fp32'))"
