#!/bin/bash
# rocprof kernel traces of the 1.25M-row bench (4 batches in flight) by scan order: the scans'
# true dispatch durations and overlap vs the bench's event-timed avg_ms; then plain bench runs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/order2.jsonl
: > $out
for order in ${ORDERS:-serial stream}; do
  rm -rf gpurun_out/prof_o_$order
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_o_$order" -o tr \
      -- python3 "$R/bench.py" --rows ${ROWS:-1250000} --steps 200 --warmup 10 --no-cpu --no-recall \
      --scan-order $order > gpurun_out/order2_$order.log 2>&1 || { rc=$?; tail -20 gpurun_out/order2_$order.log; exit $rc; }
  tail -1 gpurun_out/order2_$order.log >> $out
  python3 scripts/scan_overlap.py gpurun_out/prof_o_$order "${ROWS:-1250000} 4 in flight $order" >> $out
done
for order in ${ORDERS:-serial stream} free; do
  timeout -k 10 300 python3 bench.py --rows ${ROWS:-1250000} --steps 300 --warmup 10 --no-cpu --no-recall \
      --scan-order $order >> $out 2> gpurun_out/order2_b.err || { rc=$?; tail -20 gpurun_out/order2_b.err; exit $rc; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/order2.jsonl"):
    d = json.loads(l)
    if "metric" in d:
        r = d["roofline"]
        print(d["config"]["rows_per_gpu"], d["config"]["scan_order"], d["value"], r["avg_ms"], r["frac"], r["step_frac"], r["standalone_frac"])
    else:
        print(d)
PY
