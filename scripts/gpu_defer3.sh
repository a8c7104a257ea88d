#!/bin/bash
# deferred LayerNorm: epilogue parity, isolated GEMM timing, forward A/B (auto vs off) (TAG)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles; TAG=${TAG:-r02n}
timeout -k 10 300 python -u -m pytest tests/test_deferred_ln_gpu.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_dl.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_dl.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_dl_gemm.py | tee gpurun_out/profiles/${TAG}_dl_gemm.jsonl || exit $?
STAGES=rerank,encode_c PRECS=fp16x3 DEFERS=-1,0,-1,0 CPU=0 REPS=20 timeout -k 10 300 \
    python -u scripts/bench_stages.py > gpurun_out/profiles/${TAG}_defer_stages.jsonl || exit $?
cut -c1-130 gpurun_out/profiles/${TAG}_defer_stages.jsonl
