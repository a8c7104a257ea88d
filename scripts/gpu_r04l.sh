#!/bin/bash
# round 4: 1.25M rows, 4 in flight: timing events around every scan vs sampled, idle rescan on/off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out; out=$O/ab125.jsonl; : > $out
run() { timeout -k 10 200 python3 -u bench.py --rows 1250000 --steps 400 --warmup 20 --no-cpu --no-recall "$@" 2>> $O/ab125.err | grep '^{' | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}
d2={'args':'$*','value':d['value'],'ms':d['ms_per_step'],'frac':r.get('frac'),'union_frac':r.get('union_frac'),'exact':d.get('exact_batches')}
print(json.dumps(d2))" >> $out; }
for rep in 1 2; do
  run || exit 1
  run --prof-every 1000000 || exit 1
  RAGMI_RESCAN_WG=0 run --diagnostic --prof-every 1000000 || exit 1
done
cat $out
