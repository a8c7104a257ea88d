#!/bin/bash
# config 2 / 3 lines with inline tokenisation (3 reps each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; out=gpurun_out/inline_tok.jsonl; : > $out
for rep in 1 2 3; do for c in 2 3; do
  timeout -k 10 300 python3 -u bench.py --config $c --no-cpu 2> gpurun_out/it.err | grep '^{' >> $out || { tail -20 gpurun_out/it.err; exit 1; }
done; done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['metric'][-10:], d['value'], d.get('id_input_qps'), d.get('text_vs_id_input'), d.get('host_enqueue_ms_per_step'), d.get('search_top15_exact_queries'))"
