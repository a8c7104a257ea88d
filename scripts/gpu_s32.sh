#!/bin/bash
# fp32 storage: its parity tests + the existing scan / exactness / store / rag suites
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_storage32_gpu.py tests/test_scan_gpu.py tests/test_exactness_gpu.py \
    tests/test_store_gpu.py tests/test_rag_gpu.py tests/test_coalesce_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/s32_tests.log 2>&1
rc=$?
tail -3 gpurun_out/s32_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/s32_tests.log | head -40; fi
exit $rc
