#!/bin/bash
# parity tests, then bench + rocprof evidence (profile.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
TAG=${TAG:-r01} bash scripts/profile.sh
