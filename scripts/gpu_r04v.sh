#!/bin/bash
# round 4: config 3 (and 2) — 3 vs 4 batches in flight (default hardware queues)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out; out=$O/c3_streams.jsonl; : > $out
run() { timeout -k 10 300 python3 -u bench.py --no-cpu "$@" 2>> $O/c3s.err | grep '^{' | python3 -c "
import json,sys,os
d=json.loads(sys.stdin.read())
print(json.dumps({'args':'$*','value':d['value'],'ms':d['ms_per_step']}))" >> $out; }
for rep in 1 2; do
  for S in 3 4; do run --config 3 --streams $S || exit 1; done
  for S in 3 4; do run --config 2 --streams $S || exit 1; done
done
cat $out
