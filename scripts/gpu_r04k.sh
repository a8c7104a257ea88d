#!/bin/bash
# round 4: kernel trace of the 1.25M-row, 4-in-flight line (the N = 8 per-rank step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr125 -o tr -- python3 -u bench.py --rows 1250000 --steps 200 --warmup 10 --no-cpu --no-recall > $O/tr125.log 2>&1 || { tail -30 $O/tr125.log; exit 1; }
grep '^{' $O/tr125.log | tail -1 | cut -c1-400
find $O/tr125 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -20
