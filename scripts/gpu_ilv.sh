#!/bin/bash
# WS GEMM fragment-read order A/B (ws vs ws_ilv) + exactness of the new variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ilv.jsonl
: > $out
timeout -k 10 300 python -u -m pytest tests/test_gemm_exact_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 200 \
    --timeout-method thread -k "ws" > gpurun_out/ilv_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ilv_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/ilv_tests.log | head -20; exit $rc; fi
GEMM_VARIANTS=19,27 ROUNDS=${ROUNDS:-5} timeout -k 10 300 python -u scripts/bench_gemm.py >> $out 2> gpurun_out/ilv.err || { rc=$?; tail -20 gpurun_out/ilv.err; exit $rc; }
grep '^{' $out | grep layer
