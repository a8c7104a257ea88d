#!/bin/bash
# rerank (480 pairs) stage time + per-kernel rocprof breakdown; PRECS overrides precisions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES=rerank PRECS=${PRECS:-fp16x3,fp16} CPU=0 timeout -k 10 200 python scripts/bench_stages.py > gpurun_out/rr_stages.log 2>&1 || { rc=$?; tail -20 gpurun_out/rr_stages.log; exit $rc; }
grep '^{' gpurun_out/rr_stages.log
rm -rf gpurun_out/prof_rr
STAGES=rerank PRECS=${PRECS:-fp16x3,fp16} REPS=5 CPU=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_rr" -o st \
    -- python3 "$R/scripts/bench_stages.py" > gpurun_out/prof_rr.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof_rr.log; exit $rc; }
python3 scripts/stage_breakdown.py gpurun_out/prof_rr
