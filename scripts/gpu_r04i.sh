#!/bin/bash
# round 4: pipelined pair read-back (test + config-3 line) and the fp8-correction timing probes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rag_gpu.py -k build_pairs -x -q --timeout 120 --timeout-method thread > $O/t_pairs.log 2>&1 || { tail -30 $O/t_pairs.log; exit 1; }
tail -2 $O/t_pairs.log
GEMM_M=117000 GEMM_VARIANTS=19,39,40,20,22 timeout -k 10 300 python3 -u scripts/bench_gemm.py > $O/gemm_fp8probe.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
grep layer_ms $O/gemm_fp8probe.jsonl
CONFIGS="3" bash scripts/gpu_lines.sh
