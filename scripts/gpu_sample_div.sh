#!/bin/bash
# Seed-sample fraction A/B at small shards (the N = 4 / N = 8 shard sizes), 4 batches in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/sample_div.jsonl; : > $out
for rows in 1250000 2500000; do
  for div in 128 64 32 16; do
    echo "# rows=$rows RAGMI_SAMPLE_DIV=$div" >> $out
    RAGMI_SAMPLE_DIV=$div timeout -k 10 200 python -u bench.py --rows $rows --steps 200 --warmup 10 --no-cpu \
        >> $out 2> gpurun_out/sample_div_err.log || { rc=$?; tail -20 gpurun_out/sample_div_err.log; exit $rc; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/sample_div.jsonl"):
    if l.startswith("#"): print(l.strip(), end="  ")
    elif l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(d["value"], d["ms_per_step"], r["step_frac"], r["standalone_frac"], d["recall_at_5"], d["top15_exact_vs_oracle"])
PY
