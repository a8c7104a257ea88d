#!/bin/bash
# vectorised add-LN (RAGMI_ADDLN_VEC) A/B: encoder suites, encode_q stage, config-2 line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_stress_weights_gpu.py tests/test_encoder_graph_gpu.py tests/test_rag_gpu.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/enc_tests.log 2>&1 || { tail -30 gpurun_out/enc_tests.log; exit 1; }
tail -1 gpurun_out/enc_tests.log
ENVS="RAGMI_ADDLN_VEC=0 RAGMI_ADDLN_VEC=1" STAGES=encode_q PRECS=fp16x3 bash scripts/gpu_ab_env.sh | cut -c1-220 || exit 1
out=gpurun_out/addln_c2.jsonl; : > $out
for rep in 1 2; do for v in 0 1; do
  RAGMI_ADDLN_VEC=$v timeout -k 10 300 python -u bench.py --config 2 --no-cpu 2> gpurun_out/c2.err | grep '^{' | sed "s/^{/{\"RAGMI_ADDLN_VEC\": $v, \"rep\": $rep, /" >> $out || { tail -20 gpurun_out/c2.err; exit 1; }
done; done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['RAGMI_ADDLN_VEC'], d['rep'], d['value'], d.get('id_input_qps'))"
