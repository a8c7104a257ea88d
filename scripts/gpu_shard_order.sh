#!/bin/bash
# scan order / batches in flight at the N = 4 and N = 8 per-rank shard sizes (2.5M, 1.25M rows)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; out=gpurun_out/shard_order.jsonl; : > $out
for rows in 2500000 1250000; do for rep in 1 2; do for a in "--scan-order free --streams 4" "--scan-order serial --streams 4" "--scan-order serial --streams 2" "--scan-order serial --streams 3"; do
  timeout -k 10 300 python3 -u bench.py --rows $rows --steps 300 --warmup 10 --no-cpu --no-recall $a 2> gpurun_out/so.err | grep '^{' | sed "s/^{/{\"args\": \"$a\", \"rep\": $rep, /" >> $out || { tail -20 gpurun_out/so.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); r=d['roofline']
print($rows, d['args'], d['rep'], d['value'], r['frac'], d['ms_per_step'])"
done; done; done
