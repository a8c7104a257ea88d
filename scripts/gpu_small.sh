#!/bin/bash
# query-batch GEMM variants: parity (fp64) then timing at query-batch token counts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -p no:cacheprovider -k "small" \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_small.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_small.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_small.log | head -30; exit $rc; fi
GEMM_M=${GEMM_M:-782,3056} GEMM_VARIANTS=${GEMM_VARIANTS:-5,10,1} timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/bench_small.log 2>&1 || { rc=$?; tail -20 gpurun_out/bench_small.log; exit $rc; }
grep fp16x3 gpurun_out/bench_small.log
