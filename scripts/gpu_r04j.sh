#!/bin/bash
# round 4: register-staged loader waves (WS A/B): bit-exactness + layer timing + intake probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_exact_gpu.py -k "regstage or ws-" -x -q --timeout 120 --timeout-method thread > $O/t_regst.log 2>&1 || { tail -30 $O/t_regst.log; exit 1; }
tail -2 $O/t_regst.log
GEMM_M=117000 GEMM_VARIANTS=19,41,22,42 timeout -k 10 300 python3 -u scripts/bench_gemm.py > $O/gemm_regst.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
cat $O/gemm_regst.jsonl
