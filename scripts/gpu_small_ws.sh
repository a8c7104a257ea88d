#!/bin/bash
# small-tile loader-specialised GEMM (RAG_GEMM_WS_SMALL) for the query-batch QKV / FFN1:
# GEMM + encoder suites, then encode_q and the config-2 line with RAGMI_SMALL_WS=0 / 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_exact_gpu.py tests/test_gemm_gpu.py tests/test_encoders_gpu.py tests/test_encoder_graph_gpu.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/sws_tests.log 2>&1 || { tail -30 gpurun_out/sws_tests.log; exit 1; }
tail -1 gpurun_out/sws_tests.log
GEMM_M=782 GEMM_VARIANTS=5,34 timeout -k 10 120 python3 -u scripts/bench_gemm.py 2>/dev/null | grep fp16x3 | cut -c1-160
ENVS="RAGMI_SMALL_WS=0 RAGMI_SMALL_WS=1" STAGES=encode_q PRECS=fp16x3 bash scripts/gpu_ab_env.sh | cut -c1-160 || exit 1
VAR=RAGMI_SMALL_WS VALS="0 1" ARGS="--config 2 --no-cpu" OUT=gpurun_out/sws_c2.jsonl TMO=300 bash scripts/gpu_env_sweep.sh
