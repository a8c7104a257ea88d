#!/bin/bash
# attention VAR A/B: kernel tests, kernel timing by variant, forward A/B of two builds
# (ab/libragmi_old.so / _new.so), then the encoder suites on the in-tree build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
VARIANTS=${VARIANTS:-10,42} ROUNDS=7 timeout -k 10 200 python -u scripts/bench_attn.py > gpurun_out/attn_bench.jsonl || exit 1
cat gpurun_out/attn_bench.jsonl
STAGES=${STAGES:-rerank,encode_c,encode_q} TAG=${TAG:-attn} bash scripts/gpu_ab.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_config3_gpu.py tests/test_stress_weights_gpu.py tests/test_encoder_graph_gpu.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/enc_tests.log 2>&1 || { tail -30 gpurun_out/enc_tests.log; exit 1; }
tail -1 gpurun_out/enc_tests.log
