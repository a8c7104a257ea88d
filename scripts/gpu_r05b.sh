#!/bin/bash
# ring-depth A/B of the query-batch GEMMs (builds in ab/), then the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_ns_ab.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { rc=$?; tail -20 gpurun_out/bench_default.log; exit $rc; }
tail -1 gpurun_out/bench_default.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('headline', d['value'], 'c2', d['config2'].get('value'), d['config2'].get('id_input_qps'), 'c3', d['config3'].get('value'))"
