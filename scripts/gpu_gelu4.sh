#!/bin/bash
# vectorised erf-GELU epilogue: GEMM parity, then FFN1 WS timing and the rerank / encode_c stages
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles; TAG=${TAG:-r02o}
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_exact_gpu.py tests/test_deferred_ln_gpu.py \
    tests/test_config3_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_g4.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_g4.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|E )" gpurun_out/pytest_g4.log | head; exit $rc; }
timeout -k 10 300 python -u scripts/bench_dl_gemm.py | tee gpurun_out/profiles/${TAG}_dl_gemm.jsonl || exit $?
STAGES=rerank,encode_c PRECS=fp16x3,fp16 DEFERS=-1,0 CPU=0 REPS=20 timeout -k 10 300 \
    python -u scripts/bench_stages.py > gpurun_out/profiles/${TAG}_stages.jsonl || exit $?
cut -c1-140 gpurun_out/profiles/${TAG}_stages.jsonl
