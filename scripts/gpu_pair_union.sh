#!/bin/bash
# attention paired-query-block variants: parity, then A/B at the rerank shape; then the
# small-shard union-of-intervals timing (scripts/gpu_union.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/attn_tests.log; exit $rc; }
tail -2 gpurun_out/attn_tests.log
VARIANTS=10,26,2,18 PRECS=fp16x3 ROUNDS=7 timeout -k 10 200 python -u scripts/bench_attn.py > gpurun_out/attn_ab.jsonl 2>&1 \
    || { rc=$?; tail -20 gpurun_out/attn_ab.jsonl; exit $rc; }
cat gpurun_out/attn_ab.jsonl
bash scripts/gpu_union.sh
