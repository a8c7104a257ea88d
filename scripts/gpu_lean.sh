#!/bin/bash
# split16x2 / lean attention block: attention + GEMM parity tests, attention variant A/B,
# GEMM per-layer timing (epilogue split change), rerank stage
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/lean.jsonl
: > $out
timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py tests/test_gemm_exact_gpu.py tests/test_gemm_gpu.py \
    -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/lean_tests.log 2>&1
rc=$?
tail -3 gpurun_out/lean_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/lean_tests.log | head -30; exit $rc; fi
VARIANTS=2,10,6,14,0,8 timeout -k 10 200 python -u scripts/bench_attn.py >> $out 2> gpurun_out/lean.err || { rc=$?; tail -20 gpurun_out/lean.err; exit $rc; }
GEMM_VARIANTS=19 timeout -k 10 200 python -u scripts/bench_gemm.py >> $out 2>> gpurun_out/lean.err || { rc=$?; tail -20 gpurun_out/lean.err; exit $rc; }
STAGES=rerank PRECS=fp16x3,fp16 CPU=0 timeout -k 10 200 python -u scripts/bench_stages.py >> $out 2>> gpurun_out/lean.err || { rc=$?; tail -20 gpurun_out/lean.err; exit $rc; }
grep '^{' $out | cut -c1-220
