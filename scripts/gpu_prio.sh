#!/bin/bash
# WS GEMM issue-priority A/B (s_setprio on the loader waves / on the MFMA waves), 117K tokens
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GEMM_M=117000,14800 GEMM_VARIANTS=19,30,31,19,30,31 timeout -k 10 300 python -u scripts/bench_gemm.py \
    > gpurun_out/prio.jsonl 2> gpurun_out/prio.err || { rc=$?; tail -20 gpurun_out/prio.err; exit $rc; }
grep layer_ms gpurun_out/prio.jsonl
