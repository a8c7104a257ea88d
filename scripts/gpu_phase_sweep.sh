#!/bin/bash
# WS GEMM phase-offset A/B (RAGMI_WS_PHASE = start delay of the odd workgroups, ~3.4 us units):
# one MiniLM layer's GEMMs at 117K tokens, then the rerank / encode_c stages
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/phase_gemm.jsonl; : > $out
for rep in 1 2; do for p in ${PHASES:-0 1 2 3 5}; do
  RAGMI_WS_PHASE=$p GEMM_M=117000 GEMM_VARIANTS=19 timeout -k 10 120 python3 -u scripts/bench_gemm.py 2>/dev/null \
    | sed "s/^{/{\"phase\": $p, \"rep\": $rep, /" >> $out || exit 1
done; done
grep layer_ms $out
ENVS="${ENVS:-RAGMI_WS_PHASE=0 RAGMI_WS_PHASE=2}" STAGES=rerank,encode_c PRECS=fp16x3 bash scripts/gpu_ab_env.sh | cut -c1-200
