#!/bin/bash
# round 6: attention VAR 554 (= 42 with the P scalings as scalar FMAs, no v_pk_fma beside the
# MFMAs): bitwise check vs 42, then interleaved timing at the rerank shape (diagnostic build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RAGMI_LIB_AB=$PWD/ab/diag.so RAGMI_TEST_DIAG_BUILD=1
VARIANTS=${BITWISE:-554} timeout -k 10 120 python -u scripts/diag/attn_bitwise.py > gpurun_out/r06n_bitwise.jsonl 2> gpurun_out/r06n.err \
  || { rc=$?; tail -5 gpurun_out/r06n.err; exit $rc; }
cat gpurun_out/r06n_bitwise.jsonl
rm -f gpurun_out/r06n_attn_ab.jsonl
for i in 1 2; do
  VARIANTS=${AB:-42,554,10} ROUNDS=7 REPS=10 PRECS=fp16x3 timeout -k 10 180 python -u scripts/bench_attn.py >> gpurun_out/r06n_attn_ab.jsonl 2> gpurun_out/r06n.err \
    || { rc=$?; tail -5 gpurun_out/r06n.err; exit $rc; }
done
cat gpurun_out/r06n_attn_ab.jsonl
