#!/bin/bash
# round 4: L2 prefetch of the A panel in the WS loader (A/B): bit-exactness + layer timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_exact_gpu.py -k "l2pf" -x -q --timeout 120 --timeout-method thread > $O/t_l2pf.log 2>&1 || { tail -30 $O/t_l2pf.log; exit 1; }
tail -2 $O/t_l2pf.log
GEMM_M=117000 GEMM_VARIANTS=19,43,22,44 timeout -k 10 300 python3 -u scripts/bench_gemm.py > $O/gemm_l2pf.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
grep fp16x3 $O/gemm_l2pf.jsonl | cut -c1-200
