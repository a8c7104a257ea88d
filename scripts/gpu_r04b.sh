#!/bin/bash
# round 4: WS GEMM with 4 MFMA waves of 128 x 64 (RAG_GEMM_WS_BIG128) vs 8 of 64 x 64 (WS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gemm_exact_gpu.py -k "ws" > $O/t_gemm.log 2>&1 || { tail -40 $O/t_gemm.log; exit 1; }
tail -2 $O/t_gemm.log
GEMM_M=117000,14800 GEMM_VARIANTS=19,35,19,35 timeout -k 10 300 python3 -u scripts/bench_gemm.py > $O/gemm_big128.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
grep layer_ms $O/gemm_big128.jsonl
