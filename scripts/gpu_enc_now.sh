#!/bin/bash
# Encoder state on the current code: all stages (device time), the rerank forward's per-kernel
# rocprof breakdown, then the driver-parsable config-3 and config-2 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
CPU=0 timeout -k 10 300 python -u scripts/bench_stages.py > gpurun_out/stages_now.log 2>&1 || { rc=$?; tail -20 gpurun_out/stages_now.log; exit $rc; }
grep '^{' gpurun_out/stages_now.log > gpurun_out/stages_now.jsonl
cat gpurun_out/stages_now.jsonl | cut -c1-200
bash scripts/gpu_rerank_trace.sh || exit $?
timeout -k 10 400 python -u bench.py --config 3 > gpurun_out/config3_now.log 2> gpurun_out/config3_now.err || { rc=$?; tail -20 gpurun_out/config3_now.err; exit $rc; }
tail -1 gpurun_out/config3_now.log | cut -c1-900
timeout -k 10 400 python -u bench.py --config 2 > gpurun_out/config2_now.log 2> gpurun_out/config2_now.err || { rc=$?; tail -20 gpurun_out/config2_now.err; exit $rc; }
tail -1 gpurun_out/config2_now.log | cut -c1-600
