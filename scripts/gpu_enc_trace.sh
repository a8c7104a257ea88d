#!/bin/bash
# Stage bench + per-kernel trace of one stage (STAGE_ONLY) for the encoder breakdown.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
CPU=0 timeout -k 10 300 python scripts/bench_stages.py > gpurun_out/stages.log 2>&1 || { rc=$?; tail -20 gpurun_out/stages.log; exit $rc; }
grep '^{' gpurun_out/stages.log
rm -rf gpurun_out/prof_enc
REPS=5 CPU=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_enc" -o st \
    -- python3 "$R/scripts/bench_stages.py" > gpurun_out/prof_enc.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof_enc.log; exit $rc; }
python3 scripts/stage_breakdown.py gpurun_out/prof_enc
