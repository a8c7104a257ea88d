#!/bin/bash
# A/B of an environment knob on a bench.py line, interleaved processes:
# ENVS="RAGMI_RESCAN_WG=0 RAGMI_RESCAN_WG=512" ARGS="--rows 1250000 --steps 300" bash scripts/gpu_ab_bench.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_bench.jsonl
: > $out
for rep in $(seq ${REPS:-2}); do
  for e in $ENVS; do
    env $e timeout -k 10 300 python3 bench.py $ARGS --no-cpu --no-recall 2> gpurun_out/ab_bench.err \
      | python3 -c "import json,sys; [print(json.dumps({'env': '$e', 'rep': $rep, 'qps': d['value'], 'ms': d['ms_per_step'], 'frac': (d.get('roofline') or {}).get('frac'), 'standalone_frac': (d.get('roofline') or {}).get('standalone_frac')})) for d in map(json.loads, (l for l in sys.stdin if l.startswith('{')))]" >> $out || { tail -20 gpurun_out/ab_bench.err; exit 1; }
  done
done
cat $out
