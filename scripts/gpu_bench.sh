#!/bin/bash
# headline bench (default flags) with wall-clock; ARGS overrides the flags
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T0=$(date +%s)
timeout -k 10 600 python -u bench.py ${ARGS} > gpurun_out/bench_${TAG:-x}.log 2> gpurun_out/bench_${TAG:-x}.err \
    || { rc=$?; tail -20 gpurun_out/bench_${TAG:-x}.err; exit $rc; }
echo "wall $(( $(date +%s) - T0 )) s"
tail -1 gpurun_out/bench_${TAG:-x}.log
