#!/bin/bash
# the driver-parsable config lines on the current code: 3, 2, filtered, 5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/lines.jsonl
: > $out
for c in ${CONFIGS:-3 2 filtered 5}; do
  timeout -k 10 600 python -u bench.py --config $c >> $out 2> gpurun_out/lines_$c.err || { rc=$?; tail -20 gpurun_out/lines_$c.err; exit $rc; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/lines.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); r = d.get("roofline") or {}
        print(d["metric"][:60], d["value"], d["ms_per_step"], r.get("frac"), r.get("avg_ms"))
PY
