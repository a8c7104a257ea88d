#!/bin/bash
# Config-5 seed sample size A/B: 16384-tile cap (default now) vs the old 4096 cap, emulated
# with RAGMI_SAMPLE_DIV (n_tiles / DIV = 4096), interleaved, after the D=1024 parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "1024" > gpurun_out/wide_tests.log 2>&1 \
    || { rc=$?; tail -30 gpurun_out/wide_tests.log; exit $rc; }
tail -2 gpurun_out/wide_tests.log
out=gpurun_out/wide_sample.jsonl; : > $out
for rep in 1 2; do
  for cfg in "50000000 128" "50000000 763" "12500000 128" "12500000 191"; do
    set -- $cfg
    echo "# rows=$1 RAGMI_SAMPLE_DIV=$2 rep=$rep" >> $out
    RAGMI_SAMPLE_DIV=$2 timeout -k 10 240 python -u scripts/bench_config5.py --rows $1 \
        $( [ "$rep" = 1 ] && [ "$2" = 128 ] || echo --no-recall ) >> $out 2> gpurun_out/wide_err.log \
        || { rc=$?; tail -20 gpurun_out/wide_err.log; exit $rc; }
  done
done
python - "$out" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("#"): print(l.strip(), end="  ")
    elif l.startswith("{"):
        d = json.loads(l); print(d["roofline"]["frac"], d["roofline"]["avg_ms"], d["ms_per_step"], d["value"], d.get("recall_at_5_vs_fp32"))
PY
