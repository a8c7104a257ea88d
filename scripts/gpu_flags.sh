#!/bin/bash
# WS GEMM FULL/FREE counter ring (variant 32) vs the barrier ring (19): bitwise parity, then
# per-layer timing at the rerank and chunk-encode token counts; then the filtered / config-5
# lines (sampled launch timing restored for serial scan order)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -k ws_flag -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/flags_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/flags_tests.log; exit $rc; }
tail -2 gpurun_out/flags_tests.log
GEMM_M=117000,14800 GEMM_VARIANTS=19,32 timeout -k 10 300 python -u scripts/bench_gemm.py \
    > gpurun_out/flags.jsonl 2> gpurun_out/flags.err || { rc=$?; tail -20 gpurun_out/flags.err; exit $rc; }
GEMM_M=117000 GEMM_VARIANTS=32,19 timeout -k 10 300 python -u scripts/bench_gemm.py \
    >> gpurun_out/flags.jsonl 2>> gpurun_out/flags.err || { rc=$?; tail -20 gpurun_out/flags.err; exit $rc; }
grep -v layer_ms gpurun_out/flags.jsonl | grep 117000 | cut -c1-200
grep layer_ms gpurun_out/flags.jsonl
CONFIGS="filtered 5" bash scripts/gpu_lines.sh
