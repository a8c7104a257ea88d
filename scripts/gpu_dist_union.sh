#!/bin/bash
# N > 1 bench path at the 8-GPU shard size on one GPU: plain `python bench.py --gpus 2` (bench.py
# starts its two rank processes itself), gloo transport (RCCL cannot put two ranks on one GPU),
# 1.25M rows per rank, free scan order -> the union-of-intervals timing, max over ranks, packed
# all-gather + GPU merge, per-rank certification.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RAGMI_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --rows 2500000 --steps 50 --warmup 5 \
   --cpu-budget 5 > gpurun_out/bench_2rank_union.log 2>&1 || { rc=$?; tail -30 gpurun_out/bench_2rank_union.log; exit $rc; }
grep '^{' gpurun_out/bench_2rank_union.log | cut -c1-3000
