#!/bin/bash
# quick GPU iteration: parity tests + scan variant A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python scripts/scan_variants.py > gpurun_out/variants.log 2>&1 || { rc=$?; tail -20 gpurun_out/variants.log; exit $rc; }
cat gpurun_out/variants.log
