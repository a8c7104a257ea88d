#!/bin/bash
# Scan oversubscription A/B (RAGMI_SCAN_OVERSUB 1 / 2) at the 8-GPU shard size and at 10M,
# after the scan parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RAGMI_SCAN_OVERSUB=2 timeout -k 10 400 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/oversub_tests.log 2>&1 \
    || { rc=$?; tail -30 gpurun_out/oversub_tests.log; exit $rc; }
tail -2 gpurun_out/oversub_tests.log
out=gpurun_out/oversub.jsonl; : > $out
for cfg in "1250000 4 free" "1250000 4 serial" "10000000 2 serial"; do
  set -- $cfg
  for ov in 1 2; do
    echo "# rows=$1 streams=$2 order=$3 RAGMI_SCAN_OVERSUB=$ov" >> $out
    RAGMI_SCAN_OVERSUB=$ov timeout -k 10 240 python -u bench.py --rows $1 --streams $2 --scan-order $3 \
        --steps 200 --warmup 10 --no-cpu >> $out 2> gpurun_out/oversub_err.log \
        || { rc=$?; tail -20 gpurun_out/oversub_err.log; exit $rc; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/oversub.jsonl"):
    if l.startswith("#"): print(l.strip(), end="  ")
    elif l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(d["value"], r["frac"], r["avg_ms"], r["step_frac"], r["standalone_frac"], d["recall_at_5"], d["top15_exact_vs_oracle"])
PY
