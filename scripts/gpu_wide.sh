#!/bin/bash
# Wide scan (config 5) check: D=1024 parity tests, then bench_config5 at the 8-GPU shard
# (12.5M rows) and the 1-GPU size (50M rows) for each RAGMI_WIDE_MODE in $MODES (default "0 1").
# Usage: gpurun -- 'OUT=r01h_wide_pre bash scripts/gpu_wide.sh'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "1024" > gpurun_out/wide_tests.log 2>&1 \
    || { rc=$?; tail -30 gpurun_out/wide_tests.log; exit $rc; }
tail -2 gpurun_out/wide_tests.log
out=gpurun_out/${OUT:-wide}.jsonl; : > $out
for rows in 12500000 50000000; do
  for mode in ${MODES:-0 1}; do
    echo "# rows=$rows RAGMI_WIDE_MODE=$mode" >> $out
    RAGMI_WIDE_MODE=$mode timeout -k 10 240 python -u scripts/bench_config5.py --rows $rows \
        $( [ "$mode" = 0 ] && [ "$rows" = 50000000 ] || echo --no-recall ) >> $out 2> gpurun_out/wide_err.log \
        || { rc=$?; tail -20 gpurun_out/wide_err.log; exit $rc; }
  done
done
python - "$out" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("#"): print(l.strip(), end="  ")
    elif l.startswith("{"):
        d = json.loads(l); print(d["roofline"]["frac"], d["roofline"]["avg_ms"], d["value"], d.get("recall_at_5_vs_fp32"))
PY
