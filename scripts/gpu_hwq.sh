#!/bin/bash
# Batches in flight vs hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4 on the
# box): the 1.25M-row shard line and the config-2 line, interleaved processes.
#   REPS=2 bash scripts/gpu_hwq.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/hwq.jsonl
: > $out
run() {   # label env args...
  local label=$1 envv=$2
  shift 2
  env $envv timeout -k 10 300 python3 bench.py "$@" --no-cpu 2> gpurun_out/hwq.err \
    | python3 -c "import json,sys; [print(json.dumps({'case': '$label', 'env': '$envv', 'qps': d['value'], 'ms': d['ms_per_step'], 'frac': (d.get('roofline') or {}).get('frac'), 'union_frac': (d.get('roofline') or {}).get('frac'), 'in_flight': d['config'].get('batches_in_flight')})) for d in map(json.loads, (l for l in sys.stdin if l.startswith('{')))]" >> $out \
    || { tail -20 gpurun_out/hwq.err; exit 1; }
}
for rep in $(seq ${REPS:-1}); do
  for q in 4 8; do
    for s in 4 6 8; do
      [ $q = 4 ] && [ $s != 4 ] && continue
      run "shard1.25M q$q s$s" "GPU_MAX_HW_QUEUES=$q" --rows 1250000 --steps 300 --warmup 10 --no-recall --streams $s
    done
    for s in 3 5 7; do
      [ $q = 4 ] && [ $s != 3 ] && continue
      run "config2 q$q s$s" "GPU_MAX_HW_QUEUES=$q" --config 2 --steps 100 --warmup 10 --streams $s
    done
  done
done
cat $out
