#!/bin/bash
# config 2 / 3 lines with the batches in flight on CU-partitioned streams vs plain streams
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/part_c23.jsonl; : > $out
for rep in 1 2; do
  for a in "--config 2 --partition off" "--config 2 --partition on" "--config 3 --partition off" "--config 3 --partition on"; do
    timeout -k 10 300 python3 -u bench.py $a --no-cpu 2> gpurun_out/pc.err | grep '^{' | sed "s/^{/{\"args\": \"$a\", /" >> $out || { tail -20 gpurun_out/pc.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['args'], d['value'], d.get('id_input_qps'), d.get('search_top15_exact_queries'), d.get('rerank_max_abs_diff_vs_oracle'), d.get('host_enqueue_ms_per_step'))"
