#!/bin/bash
# config 2 line by batches in flight (STREAMS) and env knobs (ENVS), one process each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/c2_streams.jsonl
: > $out
for e in $ENVS; do
  for s in ${STREAMS:-2 3 4}; do
    env $e timeout -k 10 300 python3 bench.py --config 2 --steps ${STEPS:-100} --warmup 10 --streams $s --no-cpu --no-recall 2> gpurun_out/c2s.err \
      | python3 -c "import json,sys; [print(json.dumps({'env': '$e', 'streams': $s, 'qps': d['value'], 'id_qps': d.get('id_input_qps'), 'ms': d['ms_per_step']})) for d in map(json.loads, (l for l in sys.stdin if l.startswith('{')))]" >> $out || { tail -20 gpurun_out/c2s.err; exit 1; }
  done
done
cat $out
