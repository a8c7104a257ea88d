#!/bin/bash
# WS GEMM split last round: parity (GEMM, deferred-LN, encoder, config-3 suites), per-layer
# A/B against RAG_GEMM_WS_NOHALF, then the rerank / chunk-encode stages old vs new build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_deferred_ln_gpu.py tests/test_encoders_gpu.py \
    tests/test_config3_gpu.py tests/test_gemm_exact_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > gpurun_out/half_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/half_tests.log; exit $rc; }
tail -2 gpurun_out/half_tests.log
GEMM_M=117000,14800 GEMM_VARIANTS=19,33 timeout -k 10 300 python -u scripts/bench_gemm.py \
    > gpurun_out/half.jsonl 2> gpurun_out/half.err || { rc=$?; tail -20 gpurun_out/half.err; exit $rc; }
GEMM_M=117000 GEMM_VARIANTS=33,19 timeout -k 10 300 python -u scripts/bench_gemm.py \
    >> gpurun_out/half.jsonl 2>> gpurun_out/half.err || { rc=$?; tail -20 gpurun_out/half.err; exit $rc; }
grep layer_ms gpurun_out/half.jsonl
TAG=r02s bash scripts/gpu_ab.sh
