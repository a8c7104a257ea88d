#!/bin/bash
# one-GPU rehearsal of the N > 1 per-rank step over RCCL (RAGMI_DIST_REHEARSAL=1: world-1 nccl
# group, packed all-gather + GPU merge every batch) at the 8-GPU shard size: batches in flight
# 3 vs 4 (the collective's stream shares the 4 hardware queues), against the plain 1-GPU step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/rccl_rehearsal.jsonl; : > $out
A="--rows 1250000 --steps 300 --warmup 10 --no-cpu --no-recall"
RAGMI_DIST_REHEARSAL=1 timeout -k 10 300 python3 -u bench.py --rows 1250000 --steps 50 --warmup 5 --no-cpu 2> gpurun_out/rr.err | grep '^{' | sed 's/^{/{"label": "rehearsal_checked", /' >> $out || { tail -20 gpurun_out/rr.err; exit 1; }
for rep in 1 2; do
  for s in 3 4; do
    RAGMI_DIST_REHEARSAL=1 timeout -k 10 300 python3 -u bench.py $A --streams $s 2> gpurun_out/rr.err | grep '^{' | sed "s/^{/{\"label\": \"rccl_s$s\", /" >> $out || { tail -20 gpurun_out/rr.err; exit 1; }
  done
  timeout -k 10 300 python3 -u bench.py $A 2> gpurun_out/rr.err | grep '^{' | sed "s/^{/{\"label\": \"plain_s4\", /" >> $out || { tail -20 gpurun_out/rr.err; exit 1; }
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); r=d['roofline']
    print(d['label'], d['value'], d['backend'], d['config']['batches_in_flight'], r['frac'], d.get('exact_batches'))"
