#!/bin/bash
# Scan-order A/B: batches in flight x serial/free scan order at the 1-GPU (10M) and 8-GPU
# shard (1.25M) sizes; wide-scan no-top-k mode with nt ring loads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "serial_scan_order or d1024" > gpurun_out/order_tests.log 2>&1 \
    || { rc=$?; tail -30 gpurun_out/order_tests.log; exit $rc; }
tail -2 gpurun_out/order_tests.log
out=gpurun_out/order.jsonl; : > $out
run() {  # rows streams order
  echo "# rows=$1 streams=$2 scan_order=$3" >> $out
  timeout -k 10 240 python -u bench.py --rows $1 --streams $2 --scan-order $3 --no-cpu --no-recall \
      >> $out 2> gpurun_out/order_err.log || { rc=$?; tail -20 gpurun_out/order_err.log; exit $rc; }
}
run 10000000 1 free && run 10000000 2 serial && run 10000000 3 serial && run 10000000 2 free \
 && run 1250000 4 free && run 1250000 4 serial && run 1250000 2 serial && run 1250000 3 serial || exit $?
echo "# rows=12500000 wide MODE=1 NT=1" >> $out
RAGMI_WIDE_MODE=1 timeout -k 10 240 python -u scripts/bench_config5.py --rows 12500000 --no-recall \
    >> $out 2> gpurun_out/order_err.log || { rc=$?; tail -20 gpurun_out/order_err.log; exit $rc; }
python - <<'PY'
import json
for l in open("gpurun_out/order.jsonl"):
    if l.startswith("#"): print(l.strip(), end="  ")
    elif l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(d["value"], d["ms_per_step"], r["frac"], r["avg_ms"], r.get("step_frac"))
PY
