#!/bin/bash
# headline scan order on the current grid: serial (default at >= 4M rows) vs free, 2 / 3 in flight
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; out=gpurun_out/order.jsonl; : > $out
for rep in 1 2; do for a in "--scan-order serial" "--scan-order free" "--scan-order free --streams 3" "--scan-order serial --streams 3"; do
  timeout -k 10 300 python3 -u bench.py --steps 50 --warmup 5 --no-cpu --no-recall $a 2> gpurun_out/order.err | grep '^{' | sed "s/^{/{\"args\": \"$a\", \"rep\": $rep, /" >> $out || { tail -20 gpurun_out/order.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); r=d['roofline']
print(d['args'], d['rep'], d['value'], r['frac'], r['avg_ms'], r.get('busy_ms_per_launch'), d['ms_per_step'])"
done; done
