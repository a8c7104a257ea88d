#!/bin/bash
# round 6: config 2 batches in flight 3 / 4 / 5 on the 40 KB small-GEMM ring build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r06v_c2_streams.jsonl
rm -f $out
for s in ${SPECS:-4 5 3 4 5 3}; do
  timeout -k 10 240 python -u bench.py --config 2 --streams $s --no-cpu > gpurun_out/r06v_c2.json 2> gpurun_out/r06v.err \
    || { rc=$?; tail -5 gpurun_out/r06v.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06v_c2.json').read().strip().splitlines()[-1])
print(json.dumps({'streams': $s, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'exact': d.get('search_top15_exact_queries')}))" | tee -a $out
done
