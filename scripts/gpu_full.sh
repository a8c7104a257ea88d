#!/bin/bash
# Full GPU parity suite, then the config-5 scan bench and the end-to-end pipeline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 300 python -u scripts/bench_config5.py > gpurun_out/config5.log 2>&1 || { rc=$?; tail -20 gpurun_out/config5.log; exit $rc; }
grep '^{' gpurun_out/config5.log
timeout -k 10 300 python -u scripts/bench_pipeline.py > gpurun_out/pipeline.log 2>&1 || { rc=$?; tail -20 gpurun_out/pipeline.log; exit $rc; }
grep '^{' gpurun_out/pipeline.log
