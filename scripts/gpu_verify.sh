#!/bin/bash
# Full round check on the GPU box: smoke, parity tests, then bench + rocprof evidence.
# Usage: gpurun --timeout 1200 -- 'TAG=r01b bash scripts/gpu_verify.sh'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { rc=$?; tail -20 gpurun_out/smoke.log; exit $rc; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then TAG=${TAG:-r01} bash scripts/profile.sh; fi
