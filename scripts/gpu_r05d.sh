#!/bin/bash
# round 5: PP timing diagnostics — epilogue kinds, deferred-LN epilogues, start stagger
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
: > $O/pp_probe.jsonl
for st in 0 1 2; do
  RAGMI_PP_STAGGER=$st timeout -k 10 300 python3 -u scripts/diag/pp_probe.py >> $O/pp_probe.jsonl 2> $O/pp_probe.err || { tail -20 $O/pp_probe.err; exit 1; }
done
RAGMI_GEMM_PP=0 timeout -k 10 300 python3 -u scripts/diag/pp_probe.py >> $O/pp_probe.jsonl 2> $O/pp_probe.err || { tail -20 $O/pp_probe.err; exit 1; }
cat $O/pp_probe.jsonl
: > $O/pp_fwd_ab2.jsonl
for v in "1 0" "0 0" "1 1" "1 0" "0 0" "1 1"; do
  set -- $v
  RAGMI_GEMM_PP=$1 RAGMI_PP_STAGGER=$2 STAGES=rerank PRECS=fp16x3 CPU=0 REPS=5 timeout -k 10 300 python3 -u scripts/bench_stages.py 2>> $O/fwd.err | grep '^{' | sed "s/^{/{\"gemm_pp\": $1, \"stagger\": $2, /" >> $O/pp_fwd_ab2.jsonl || { tail $O/fwd.err; exit 1; }
done
cut -c1-120 $O/pp_fwd_ab2.jsonl
