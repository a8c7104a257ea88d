#!/bin/bash
# deferred-LN epilogue stores in the plain epilogue's order: parity, the forward's per-GEMM
# HBM traffic, and the rerank / chunk-encode stages old vs new build (same box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_deferred_ln_gpu.py tests/test_config3_gpu.py -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/dls_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/dls_tests.log; exit $rc; }
tail -2 gpurun_out/dls_tests.log
bash scripts/gpu_fwd_pmc.sh || exit $?
TAG=r02u bash scripts/gpu_ab.sh
