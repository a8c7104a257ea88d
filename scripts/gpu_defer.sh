#!/bin/bash
# deferred LayerNorm: parity (kernel epilogues + encoder forced/auto), then the rerank /
# encode_c stage times with it on and off, and a per-kernel rerank breakdown (TAG)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles
TAG=${TAG:-r02l}
timeout -k 10 600 python -u -m pytest tests/test_deferred_ln_gpu.py tests/test_config3_gpu.py \
    -x -v -s -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_dl.log 2>&1
rc=$?; grep -E "max err|max\|d\||passed|failed|Error" gpurun_out/pytest_dl.log | tail -60; [ $rc -eq 0 ] || exit $rc
STAGES=rerank,encode_c PRECS=fp16x3 DEFERS=-1,0,-1,0 CPU=0 REPS=20 timeout -k 10 300 \
    python -u scripts/bench_stages.py > gpurun_out/profiles/${TAG}_defer_stages.jsonl || exit $?
cat gpurun_out/profiles/${TAG}_defer_stages.jsonl
cd /tmp && export TMPDIR=/tmp
STAGES=rerank PRECS=fp16x3 DEFERS=-1 CPU=0 REPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    -d $GRAFT_REPO_ROOT/gpurun_out/prof_dl -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_stages.py \
    > $GRAFT_REPO_ROOT/gpurun_out/prof_dl.log 2>&1 || exit $?
f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_dl -name "*kernel_stats.csv" | head -1)
cp "$f" $GRAFT_REPO_ROOT/gpurun_out/profiles/${TAG}_defer_rerank_kernel_stats.csv
cut -c1-150 "$f" | head -20
