#!/bin/bash
# round 4: 1.25M rows — scan grid x batches in flight sweep on the current build (diagnostic)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out; out=$O/sweep125.jsonl; : > $out
run() { timeout -k 10 200 python3 -u bench.py --rows 1250000 --steps 400 --warmup 20 --no-cpu --no-recall "$@" 2>> $O/sweep125.err | grep '^{' | python3 -c "
import json,sys,os
d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}
print(json.dumps({'args':'$*','scan_wgs':os.environ.get('RAGMI_SCAN_WGS'),'value':d['value'],'ms':d['ms_per_step'],'frac':r.get('frac')}))" >> $out; }
for rep in 1 2; do
  for S in 4 5 6; do
    for W in 192 224 256; do RAGMI_SCAN_WGS=$W run --diagnostic --streams $S || exit 1; done
  done
done
cat $out
