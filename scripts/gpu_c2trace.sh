#!/bin/bash
# config 2 (encode + search, 2 in flight): is the GPU busy, or is the host the limit?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_c2" -o tr \
    -- python3 "$R/bench.py" --config 2 --no-cpu > gpurun_out/c2_prof.log 2>&1 || { rc=$?; tail -20 gpurun_out/c2_prof.log; exit $rc; }
grep '^{' gpurun_out/c2_prof.log | cut -c1-200
python3 scripts/trace_busy.py gpurun_out/prof_c2 0.3
