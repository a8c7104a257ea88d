#!/bin/bash
# round 4: 1.25M rows, 4 in flight with the scan timed by its own dispatch (hipExtLaunchKernel
# events); tier-2 grid sweep (idle cost vs 4-marked latency)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out; out=$O/ab125m.jsonl; : > $out
run() { timeout -k 10 200 python3 -u bench.py --rows 1250000 --steps 400 --warmup 20 --no-cpu --no-recall "$@" 2>> $O/ab125.err | grep '^{' | python3 -c "
import json,sys,os
d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}
d2={'args':'$*','rescan_wg':os.environ.get('RAGMI_RESCAN_WG'),'value':d['value'],'ms':d['ms_per_step'],'frac':r.get('frac'),'roof':{k:v for k,v in r.items() if k not in ('note',)}}
print(json.dumps(d2))" >> $out; }
for rep in 1 2; do
  run || exit 1
  run --prof-every 1000000 || exit 1
  for R in 64 128 256; do RAGMI_RESCAN_WG=$R run --diagnostic --prof-every 1000000 || exit 1; done
done
cut -c1-250 $out
for R in 128 256 512; do RAGMI_RESCAN_WG=$R timeout -k 10 300 python3 -u scripts/bench_tier2.py --marked 4 --rows 1250000 10000000 >> $O/t2grid.jsonl 2>> $O/t2.err || { tail $O/t2.err; exit 1; }; done
cut -c1-300 $O/t2grid.jsonl
