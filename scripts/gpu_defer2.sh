#!/bin/bash
# deferred LayerNorm parity + per-kernel rerank breakdown with it on and off (TAG)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest tests/test_deferred_ln_gpu.py tests/test_config3_gpu.py \
    -x -v -s -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_dl.log 2>&1
rc=$?; grep -E "max\|d\||passed|failed|Error" gpurun_out/pytest_dl.log | tail -20; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r02m} bash scripts/gpu_defer_prof.sh
