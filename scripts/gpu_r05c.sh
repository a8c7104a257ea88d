#!/bin/bash
# CU-partition probe at 1.25M rows, then the config-2 line twice (host enqueue time per batch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_cu_part.sh || exit $?
: > gpurun_out/c2_host.jsonl
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --config 2 --no-cpu 2> gpurun_out/c2h.err | grep '^{' >> gpurun_out/c2_host.jsonl || { tail -20 gpurun_out/c2h.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/c2_host.jsonl'):
    d=json.loads(l); print(d['value'], d['id_input_qps'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
