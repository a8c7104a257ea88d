#!/bin/bash
# end-of-session check: smoke + full GPU suite, headline bench + rocprof evidence (TAG), the
# 8-GPU-shard-size line and the config-3 line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r02t} PROFILE=1 bash scripts/gpu_verify.sh || exit $?
out=gpurun_out/extra_lines.jsonl
: > $out
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu >> $out 2> gpurun_out/extra.err || { rc=$?; tail -20 gpurun_out/extra.err; exit $rc; }
cut -c1-300 $out
CONFIGS=3 bash scripts/gpu_lines.sh
