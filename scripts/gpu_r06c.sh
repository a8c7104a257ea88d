#!/bin/bash
# round 6 item 4: config legs in the serving shape (in process) vs child processes, twice each,
# interleaved on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/r06c_legs.jsonl
for rep in 1 2; do
  for legs in child inproc; do
    timeout -k 10 420 python -u bench.py --legs $legs --no-cpu > gpurun_out/r06c_$legs$rep.json 2> gpurun_out/r06c_$legs$rep.err \
        || { rc=$?; tail -5 gpurun_out/r06c_$legs$rep.err; exit $rc; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r06c_$legs$rep.json').read().strip().splitlines()[-1])
out={'legs':'$legs','rep':$rep,'headline':d['value'],'config2':d['config2'].get('value'),'config3':d['config3'].get('value'),
     'c2_ms':d['config2'].get('ms_per_step'),'c3_ms':d['config3'].get('ms_per_step'),
     'c3_ce_ms':(d['config3'].get('roofline') or {}).get('avg_ms'),'c2_enc_ms':(d['config2'].get('roofline') or {}).get('avg_ms'),
     'c2_traffic':(d['config2'].get('roofline') or {}).get('traffic'),'c3_traffic':(d['config3'].get('roofline') or {}).get('traffic')}
print(json.dumps(out))" | tee -a gpurun_out/r06c_legs.jsonl
  done
done
