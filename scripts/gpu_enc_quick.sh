#!/bin/bash
# encoder parity tests + the stage bench (no profiler)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_encoders_gpu.py tests/test_rag_gpu.py tests/test_gemm_gpu.py -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_encq.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_encq.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_encq.log | head -30; exit $rc; fi
grep -h "max|d|" gpurun_out/pytest_encq.log | head -0
CPU=0 timeout -k 10 300 python scripts/bench_stages.py > gpurun_out/stages_q.log 2>&1 || { rc=$?; tail -20 gpurun_out/stages_q.log; exit $rc; }
grep '^{' gpurun_out/stages_q.log
