#!/bin/bash
# kernel trace of the config-3 rerank forward (480 pairs, fp16x3): per-kernel totals of one
# forward (scripts/trace_forward.py) -> gpurun_out/rerank_forward.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
rm -rf gpurun_out/prof_rr
STAGES=rerank PRECS=fp16x3 CPU=0 REPS=5 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
  -d "$R/gpurun_out/prof_rr" -o rr -- python3 "$R/scripts/bench_stages.py" > gpurun_out/prof_rr.log 2>&1 || { tail -20 gpurun_out/prof_rr.log; exit 1; }
grep '^{' gpurun_out/prof_rr.log | cut -c1-250
python3 scripts/trace_forward.py gpurun_out/prof_rr ${NK:-40} > gpurun_out/rerank_forward.txt && tail -16 gpurun_out/rerank_forward.txt
