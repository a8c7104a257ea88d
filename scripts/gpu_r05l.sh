#!/bin/bash
# config lines at the pipeline defaults (200 timed batches, 20 warmup)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; out=gpurun_out/c23_defaults.jsonl; : > $out
for c in 2 2 2 3; do
  timeout -k 10 400 python3 -u bench.py --config $c --no-cpu 2> gpurun_out/cd.err | grep '^{' >> $out || { tail -20 gpurun_out/cd.err; exit 1; }
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['metric'][-10:], d['value'], d['steps'], d['warmup'], d.get('id_input_qps'), d.get('text_vs_id_input'), d.get('host_enqueue_ms_per_step'), d.get('search_top15_exact_queries'), d['roofline'].get('avg_ms'))"
