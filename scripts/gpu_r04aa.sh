#!/bin/bash
# round 4: last layer as K|V projection + CLS-only attention — encoder parity + rerank A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
RAGMI_TEST_DIAGNOSTIC=1 RAGMI_CLS_ATTN=1 timeout -k 10 900 python -u -m pytest tests/test_config3_gpu.py tests/test_deferred_ln_gpu.py tests/test_encoders_gpu.py tests/test_stress_weights_gpu.py tests/test_encoder_graph_gpu.py tests/test_rag_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t_cls.log 2>&1 || { tail -40 $O/t_cls.log; exit 1; }
tail -2 $O/t_cls.log
: > $O/cls_ab.jsonl
for v in 1 0 1 0; do
  RAGMI_CLS_ATTN=$v STAGES=rerank PRECS=fp16x3 CPU=0 REPS=5 timeout -k 10 300 python3 -u scripts/bench_stages.py 2>> $O/cls.err | grep '^{' | sed "s/^{/{\"cls_attn\": $v, /" >> $O/cls_ab.jsonl || { tail $O/cls.err; exit 1; }
done
cut -c1-260 $O/cls_ab.jsonl
