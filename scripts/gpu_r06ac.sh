#!/bin/bash
# round 6: run-to-run spread of the default bench line on the final build (3 runs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r06ac_default_spread.jsonl
rm -f $out
for r in 1 2 3; do
  timeout -k 10 400 python -u bench.py > gpurun_out/r06ac_b.json 2> gpurun_out/r06ac.err \
    || { rc=$?; tail -5 gpurun_out/r06ac.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06ac_b.json').read().strip().splitlines()[-1])
print(json.dumps({'run': $r, 'value': d['value'], 'frac': d['roofline']['frac'], 'exact': d['exact_batches'], 'config2': d['config2']['value'], 'config3': d['config3']['value'], 'cpu_qps': d['cpu_baseline']['value']}))" | tee -a $out
done
