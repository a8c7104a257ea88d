#!/bin/bash
# Sweep one environment knob over a bench.py command, interleaved processes, REPS rounds:
#   VAR=RAGMI_WIDE_WGS VALS="256 192" ARGS="--config 5 --rows 25000000 --steps 20 --warmup 3 --no-cpu" \
#   OUT=gpurun_out/sweep.jsonl bash scripts/gpu_env_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=${OUT:-gpurun_out/sweep.jsonl}
: > $out
for rep in $(seq 1 ${REPS:-2}); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 ${TMO:-300} python3 -u bench.py --diagnostic $ARGS > gpurun_out/sweep_one.log 2> gpurun_out/sweep.err \
      || { rc=$?; tail -20 gpurun_out/sweep.err; exit $rc; }
    grep '^{' gpurun_out/sweep_one.log | sed "s/^{/{\"$VAR\": \"$v\", \"rep\": $rep, /" >> $out
    python3 -c "
import json,sys
d=json.loads(open('$out').read().strip().splitlines()[-1]); r=d.get('roofline') or {}
print('$VAR=$v rep $rep', d['value'], r.get('frac'), r.get('avg_ms'), d.get('exact_batches'))"
  done
done
