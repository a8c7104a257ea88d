#!/bin/bash
# round 6 final build: rerank forward kernel trace + per-GEMM FETCH / WRITE / MFMA-busy PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_rerank_trace.sh || exit $?
bash scripts/gpu_fwd_pmc.sh || exit $?
