#!/bin/bash
# round 4: config 2 — batches in flight x hardware queues per process (diagnostic sweep)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out; out=$O/c2_streams.jsonl; : > $out
run() { timeout -k 10 300 python3 -u bench.py --config 2 --no-cpu "$@" 2>> $O/c2s.err | grep '^{' | python3 -c "
import json,sys,os
d=json.loads(sys.stdin.read())
print(json.dumps({'args':'$*','hwq':os.environ.get('GPU_MAX_HW_QUEUES'),'value':d['value'],'ms':d['ms_per_step']}))" >> $out; }
for rep in 1 2; do
  for S in 3 4; do run --streams $S || exit 1; done
  for S in 4 5 6; do GPU_MAX_HW_QUEUES=8 run --streams $S || exit 1; done
done
cat $out
