#!/bin/bash
# Round 5 measurement pass on one MI355X: default bench line (headline + config-2/3 legs) and
# the headline's rocprof evidence (profile.sh), the rerank forward's kernel trace and PMC
# passes, the query-batch GEMM K sweep (item 2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05a} bash scripts/profile.sh || exit $?
NK=40 bash scripts/gpu_rerank_trace.sh || exit $?
bash scripts/gpu_fwd_pmc.sh || exit $?
timeout -k 10 240 python3 -u scripts/diag/small_gemm_sweep.py > gpurun_out/small_sweep.jsonl 2> gpurun_out/small_sweep.err || { tail -5 gpurun_out/small_sweep.err; exit 1; }
echo measure-done
