#!/bin/bash
# round 6: first-run headline penalty on a fresh box: warm-up 5 vs 30, alternating, first run first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/r06k_warm.jsonl
for w in 30 5 30 5; do
  timeout -k 10 240 python -u bench.py --no-configs --no-cpu --warmup $w > gpurun_out/r06k_w$w.json 2> gpurun_out/r06k.err \
      || { rc=$?; tail -5 gpurun_out/r06k.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06k_w$w.json').read().strip().splitlines()[-1])
print(json.dumps({'warmup':$w,'value':d['value'],'frac':d['roofline']['frac'],'avg_ms':d['roofline']['avg_ms'],'exact':d['exact_batches']}))" | tee -a gpurun_out/r06k_warm.jsonl
done
