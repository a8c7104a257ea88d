#!/bin/bash
# round 4: attention staging A/B (VAR bit 64: loads first; bit 1: rolling Q prefetch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_attn.log 2>&1 || { tail -30 $O/t_attn.log; exit 1; }
tail -2 $O/t_attn.log
VARIANTS=42,43,106,107 ROUNDS=7 timeout -k 10 300 python3 -u scripts/bench_attn.py > $O/attn_ab.jsonl 2> $O/attn.err || { tail -20 $O/attn.err; exit 1; }
cat $O/attn_ab.jsonl
