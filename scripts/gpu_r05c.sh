#!/bin/bash
# round 5: PP with counted epilogue waits — parity, GEMM layer A/B, large-k, encoder suites,
# rerank forward A/B (RAGMI_GEMM_PP=1 vs 0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_large_k_gpu.py tests/test_device_cpu.py -x -q --timeout 300 --timeout-method thread > $O/t_pp.log 2>&1 || { tail -40 $O/t_pp.log; exit 1; }
tail -2 $O/t_pp.log
for r in 1 2 3; do timeout -k 10 300 python3 -u scripts/diag/pp_vs_ws.py >> $O/pp_vs_ws.log 2>&1 || { tail -20 $O/pp_vs_ws.log; exit 1; }; done
grep mismatch $O/pp_vs_ws.log
GEMM_M=117000 GEMM_PRECS=fp16x3 GEMM_VARIANTS=19,45,48,46,47 timeout -k 10 300 python3 -u scripts/bench_gemm.py > $O/gemm_pp3.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
grep layer_ms $O/gemm_pp3.jsonl
: > $O/pp_fwd_ab.jsonl
for v in 1 0 1 0; do
  RAGMI_GEMM_PP=$v STAGES=rerank PRECS=fp16x3 CPU=0 REPS=5 timeout -k 10 300 python3 -u scripts/bench_stages.py 2>> $O/fwd.err | grep '^{' | sed "s/^{/{\"gemm_pp\": $v, /" >> $O/pp_fwd_ab.jsonl || { tail $O/fwd.err; exit 1; }
done
cut -c1-200 $O/pp_fwd_ab.jsonl
RAGMI_TEST_DIAGNOSTIC=1 RAGMI_GEMM_PP=0 timeout -k 10 600 python -u -m pytest tests/test_config3_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t_c3_ws.log 2>&1; echo "config3 with WS rc=$?"; tail -3 $O/t_c3_ws.log
timeout -k 10 900 python -u -m pytest tests/test_deferred_ln_gpu.py tests/test_config3_gpu.py tests/test_encoders_gpu.py tests/test_stress_weights_gpu.py -q --timeout 300 --timeout-method thread > $O/t_enc.log 2>&1; echo "encoders rc=$?"
grep -E "passed|failed|FAILED|max\|d\|" $O/t_enc.log | tail -20
