#!/bin/bash
# round 4: 1.25M rows with an 8-slot workspace ring: batches in flight x hardware queues per
# process (GPU_MAX_HW_QUEUES) (diagnostic sweep)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out; out=$O/hwq125.jsonl; : > $out
run() { timeout -k 10 200 python3 -u bench.py --rows 1250000 --steps 400 --warmup 20 --no-cpu --no-recall "$@" 2>> $O/hwq125.err | grep '^{' | python3 -c "
import json,sys,os
d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}
print(json.dumps({'args':'$*','hwq':os.environ.get('GPU_MAX_HW_QUEUES'),'value':d['value'],'ms':d['ms_per_step'],'frac':r.get('frac'),'exact':d.get('exact_batches')}))" >> $out; }
for rep in 1 2; do
  for S in 4 5 6; do run --streams $S || exit 1; done
  for S in 5 6 8; do GPU_MAX_HW_QUEUES=8 run --streams $S || exit 1; done
  for S in 6 8; do GPU_MAX_HW_QUEUES=16 run --streams $S || exit 1; done
done
cat $out
