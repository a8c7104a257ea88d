#!/bin/bash
# smoke + the whole GPU suite (one process), log per-test durations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { rc=$?; tail -20 gpurun_out/smoke.log; exit $rc; }
tail -1 gpurun_out/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread --durations=15 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -22 gpurun_out/pytest_gpu.log
exit $rc
