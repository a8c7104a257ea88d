#!/bin/bash
# GEMM parity tests (both variants) then the TILE vs PIPE benchmark.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gemm.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_gemm.log | head -30; exit $rc; fi
timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || { rc=$?; tail -20 gpurun_out/bench_gemm.log; exit $rc; }
cat gpurun_out/bench_gemm.log
