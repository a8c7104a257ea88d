#!/bin/bash
# Wide scan (config 5) ring-load cache policy A/B: RAGMI_WIDE_NT 0/1 x RAGMI_WIDE_MODE 0/2,
# after the D=1024 parity tests pass with nt loads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RAGMI_WIDE_NT=1 timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "1024" > gpurun_out/wide_nt_tests.log 2>&1 \
    || { rc=$?; tail -20 gpurun_out/wide_nt_tests.log; exit $rc; }
tail -2 gpurun_out/wide_nt_tests.log
out=gpurun_out/wide_nt.jsonl; : > $out
for rows in 12500000 50000000; do
  for mode in 0 2; do
    for nt in 0 1; do
      echo "# rows=$rows RAGMI_WIDE_MODE=$mode RAGMI_WIDE_NT=$nt" >> $out
      RAGMI_WIDE_MODE=$mode RAGMI_WIDE_NT=$nt timeout -k 10 240 python -u scripts/bench_config5.py \
          --rows $rows --no-recall >> $out 2> gpurun_out/wide_nt_err.log \
          || { rc=$?; tail -20 gpurun_out/wide_nt_err.log; exit $rc; }
    done
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/wide_nt.jsonl"):
    if l.startswith("#"): print(l.strip(), end="  ")
    elif l.startswith("{"):
        d = json.loads(l); print(d["roofline"]["frac"], d["roofline"]["avg_ms"], d["value"])
PY
