#!/bin/bash
# GPU-box check: parity tests, a short bench, and a rocprofv3 kernel-trace of the bench.
# Stops at the first crash/timeout (exit codes other than 0/1 from pytest).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
STEPS=${STEPS:-20}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps $STEPS --warmup 3 > gpurun_out/bench.log 2>&1 || { rc=$?; tail -20 gpurun_out/bench.log; exit $rc; }
tail -2 gpurun_out/bench.log
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run \
      -- python3 "$R/bench.py" --steps $STEPS --warmup 3 --no-recall --no-cpu \
      > gpurun_out/prof.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof.log; exit $rc; }
  tail -1 gpurun_out/prof.log
fi
exit 0
