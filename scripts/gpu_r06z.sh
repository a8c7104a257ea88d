#!/bin/bash
# round 6: kernel dispatches per config-2 batch (rocprofv3 kernel trace of a short run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/c2trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c2trace" -o t \
  -- python3 "$R/bench.py" --config 2 --no-cpu --steps 40 --warmup 20 > gpurun_out/c2trace.log 2>&1 \
  || { rc=$?; tail -5 gpurun_out/c2trace.log; exit $rc; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/c2trace/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(int(r["Calls"]) for r in rows)
print("total dispatches", tot)
for r in sorted(rows, key=lambda r: -int(r["Calls"]))[:40]:
    print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), r["Name"][:110])
PY
