#!/bin/bash
# round 4, first box: new tier-2 rescan (one launch for all marked queries) — parity, worst
# case latency, idle cost at the headline and at the N = 8 shard size
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_exactness_gpu.py tests/test_storage32_gpu.py tests/test_scan_gpu.py \
  tests/test_encoder_graph_gpu.py tests/test_attention_gpu.py > $O/t_exact.log 2>&1 \
  || { tail -40 $O/t_exact.log; exit 1; }
tail -3 $O/t_exact.log
timeout -k 10 300 python3 -u scripts/bench_tier2.py --marked 4 16 32 > $O/tier2.jsonl 2> $O/tier2.err \
  || { tail -20 $O/tier2.err; exit 1; }
cat $O/tier2.jsonl
: > $O/lines.jsonl
for rows in 1250000 10000000; do
  timeout -k 10 300 python3 -u bench.py --rows $rows --steps 200 --warmup 10 --no-cpu --no-recall 2> $O/b.err | grep '^{' >> $O/lines.jsonl || { tail -20 $O/b.err; exit 1; }
  RAGMI_RESCAN_WG=0 timeout -k 10 300 python3 -u bench.py --diagnostic --rows $rows --steps 200 --warmup 10 --no-cpu --no-recall 2> $O/b.err | grep '^{' >> $O/lines.jsonl || { tail -20 $O/b.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/lines.jsonl'):
    d=json.loads(l); r=d.get('roofline') or {}
    print(d['config'].get('rows_per_gpu'), d['value'], r.get('frac'), d.get('exact_batches'), d.get('ms_per_step'))"
