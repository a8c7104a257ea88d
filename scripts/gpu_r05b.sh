#!/bin/bash
# round 5: PP vs WS bitwise at the forward's size; PP probes; large-k + device tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 300 python3 -u scripts/diag/pp_vs_ws.py > $O/pp_vs_ws.log 2>&1; echo "pp_vs_ws rc=$?"; cat $O/pp_vs_ws.log | tail -20
GEMM_M=117000 GEMM_PRECS=fp16x3 GEMM_VARIANTS=45,48,49,19 timeout -k 10 300 python3 -u scripts/bench_gemm.py > $O/gemm_pp2.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
cat $O/gemm_pp2.jsonl
timeout -k 10 600 python -u -m pytest tests/test_large_k_gpu.py tests/test_device_cpu.py -x -v --timeout 300 --timeout-method thread > $O/t_lk.log 2>&1; rc=$?
tail -30 $O/t_lk.log; echo "large-k rc=$rc"
