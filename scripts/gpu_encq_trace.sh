#!/bin/bash
# kernel trace of the 32-query bge-small forward (config 2's encoder) on the current code:
# per-kernel durations of one forward (scripts/trace_forward.py) -> gpurun_out/encq_forward.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_encq
STAGES=encode_q PRECS=fp16x3 CPU=0 REPS=30 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
  -d "$R/gpurun_out/prof_encq" -o encq -- python3 "$R/scripts/bench_stages.py" > gpurun_out/prof_encq.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof_encq.log; exit $rc; }
grep '^{' gpurun_out/prof_encq.log | cut -c1-300
python3 scripts/trace_forward.py gpurun_out/prof_encq ${NK:-87} > gpurun_out/encq_forward.txt && tail -14 gpurun_out/encq_forward.txt
