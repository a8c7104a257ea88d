#!/bin/bash
# round 5: ping-pong GEMM — parity (PP tests, GEMM exact suites, deferred-LN, encoders) then
# GEMM A/B per layer and the rerank forward A/B (RAGMI_GEMM_PP=1 vs 0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_pp.log 2>&1 || { tail -40 $O/t_pp.log; exit 1; }
tail -2 $O/t_pp.log
GEMM_M=117000 GEMM_PRECS=fp16x3 GEMM_VARIANTS=19,45,46,47,20,22 timeout -k 10 300 python3 -u scripts/bench_gemm.py > $O/gemm_pp.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
cat $O/gemm_pp.jsonl
timeout -k 10 600 python -u -m pytest tests/test_deferred_ln_gpu.py tests/test_config3_gpu.py tests/test_encoders_gpu.py tests/test_stress_weights_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t_enc.log 2>&1 || { tail -40 $O/t_enc.log; exit 1; }
tail -2 $O/t_enc.log
: > $O/pp_fwd_ab.jsonl
for v in 1 0 1 0; do
  RAGMI_GEMM_PP=$v STAGES=rerank PRECS=fp16x3 CPU=0 REPS=5 timeout -k 10 300 python3 -u scripts/bench_stages.py 2>> $O/fwd.err | grep '^{' | sed "s/^{/{\"gemm_pp\": $v, /" >> $O/pp_fwd_ab.jsonl || { tail $O/fwd.err; exit 1; }
done
cut -c1-260 $O/pp_fwd_ab.jsonl
