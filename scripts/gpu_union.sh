#!/bin/bash
# small-shard (8-GPU shard size) bench with every scan launch event-timed: the union-of-
# intervals device time per launch vs the rocprofv3 kernel trace's own union; qps with every
# launch timed vs every 4th (same process order: A, B, A, B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/union.jsonl
: > $out
rm -rf gpurun_out/prof_union
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_union" -o tr \
    -- python3 "$R/bench.py" --rows 1250000 --steps 300 --warmup 10 --no-cpu --no-recall \
    > gpurun_out/union_prof.log 2>&1 || { rc=$?; tail -20 gpurun_out/union_prof.log; exit $rc; }
grep '^{' gpurun_out/union_prof.log >> $out
python3 scripts/scan_overlap.py gpurun_out/prof_union "1.25M 4 in flight free (rocprof trace)" >> $out
for pe in 1 4 1 4; do
  timeout -k 10 300 python3 bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu --no-recall \
      --prof-every $pe >> $out 2> gpurun_out/union_b.err || { rc=$?; tail -20 gpurun_out/union_b.err; exit $rc; }
done
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --no-cpu >> $out 2>> gpurun_out/union_b.err || { rc=$?; tail -20 gpurun_out/union_b.err; exit $rc; }
python3 - <<'PY'
import json
for l in open("gpurun_out/union.jsonl"):
    d = json.loads(l)
    if "metric" in d:
        r = d["roofline"]
        print(d["config"]["rows_per_gpu"], d["value"], r.get("time_basis"), r.get("busy_ms_per_launch"), r["avg_ms"], r["frac"], r.get("frac_of_avg_launch"), r["step_frac"], r["standalone_frac"])
    else:
        print(d)
PY
