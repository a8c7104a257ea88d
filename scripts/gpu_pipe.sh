#!/bin/bash
# encoder parity (incl. concurrent streams) then the pipeline bench (synced + pipelined)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_encoders_gpu.py tests/test_rag_gpu.py -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_pipe.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_pipe.log | head -30; exit $rc; fi
STEPS=${STEPS:-40} timeout -k 10 400 python -u scripts/bench_pipeline.py > gpurun_out/pipeline.log 2>&1 || { rc=$?; tail -20 gpurun_out/pipeline.log; exit $rc; }
grep '^{' gpurun_out/pipeline.log
