#!/bin/bash
# quick knob sweeps on the current build: config-2 batches in flight, 1.25M-row shard knobs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/knobs.jsonl; : > $out
run() {  # label, env..., -- bench args
  local label=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 -u bench.py "$@" 2> gpurun_out/knob.err | grep '^{' | sed "s/^{/{\"label\": \"$label\", /" >> $out || { tail -20 gpurun_out/knob.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); r=d.get('roofline') or {}
print(d['label'], d['value'], r.get('frac'), d.get('id_input_qps'))"
}
for rep in 1 2; do
  for s in 3 4 2; do run c2_s$s X=1 -- --config 2 --no-cpu --streams $s; done
  run sh_base X=1 -- --rows 1250000 --steps 300 --warmup 10 --no-cpu --no-recall
  run sh_norescan RAGMI_RESCAN_WG=0 -- --rows 1250000 --steps 300 --warmup 10 --no-cpu --no-recall
  run sh_s3 X=1 -- --rows 1250000 --steps 300 --warmup 10 --no-cpu --no-recall --streams 3
  run sh_div64 RAGMI_SAMPLE_DIV=64 -- --rows 1250000 --steps 300 --warmup 10 --no-cpu --no-recall
done
