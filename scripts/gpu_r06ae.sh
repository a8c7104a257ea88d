#!/bin/bash
# round 6: headline scan order — serial event chain (mode 1, default) vs the handle's own scan
# stream (mode 2: consecutive scans on one queue, no cross-queue wait between them)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r06ae_scan_order.jsonl
rm -f $out
for o in ${SPECS:-auto stream auto stream auto stream}; do
  timeout -k 10 300 python -u bench.py --no-configs --no-cpu --scan-order $o > gpurun_out/r06ae_b.json 2> gpurun_out/r06ae.err \
    || { rc=$?; tail -5 gpurun_out/r06ae.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06ae_b.json').read().strip().splitlines()[-1])
print(json.dumps({'order': '$o', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'frac': d['roofline']['frac'], 'avg_ms': d['roofline']['avg_ms'], 'exact': d['exact_batches'], 'scan_order': d['config']['scan_order']}))" | tee -a $out
done
