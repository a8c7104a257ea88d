#!/bin/bash
# round 4: query-batch deferred LayerNorm (PipeDlSmall): parity tests, encode_q A/B, config 2 line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_deferred_ln_gpu.py tests/test_encoders_gpu.py tests/test_encoder_graph_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t_dls.log 2>&1 || { tail -40 $O/t_dls.log; exit 1; }
tail -2 $O/t_dls.log
: > $O/encq_ab.jsonl
for v in 1 0 1 0; do
  RAGMI_DL_SMALL=$v STAGES=encode_q PRECS=fp16x3 CPU=0 REPS=50 timeout -k 10 200 python3 -u scripts/bench_stages.py 2>> $O/encq.err | grep '^{' | sed "s/^{/{\"dl_small\": $v, /" >> $O/encq_ab.jsonl || { tail $O/encq.err; exit 1; }
done
cut -c1-300 $O/encq_ab.jsonl
CONFIGS="2" bash scripts/gpu_lines.sh
