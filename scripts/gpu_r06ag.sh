#!/bin/bash
# round 6: rescan grid default 64 (free CUs) vs 256: tier-2 latency and the 1.25M-row line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r06ag_rescan.jsonl
rm -f $out
for g in 64 256; do
  RAGMI_RESCAN_WG=$g timeout -k 10 300 python -u scripts/bench_tier2.py > gpurun_out/r06ag_t2.jsonl 2> gpurun_out/r06ag.err \
    || { rc=$?; tail -5 gpurun_out/r06ag.err; exit $rc; }
  sed "s/^{/{\"rescan_wg\": $g, /" gpurun_out/r06ag_t2.jsonl | grep '^{' | tee -a $out
done
for g in 64 256 64 256; do
  RAGMI_RESCAN_WG=$g timeout -k 10 300 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu --no-configs --diagnostic > gpurun_out/r06ag_b.json 2> gpurun_out/r06ag.err \
    || { rc=$?; tail -5 gpurun_out/r06ag.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06ag_b.json').read().strip().splitlines()[-1])
print(json.dumps({'rescan_wg': $g, 'rows': 1250000, 'value': d['value'], 'frac': d['roofline']['frac'], 'exact': d['exact_batches']}))" | tee -a $out
done
