#!/bin/bash
# 1-GPU box rehearsal of the N>1 bench path: 2 ranks on cuda:0 with gloo transport (RCCL
# cannot put two ranks on one GPU), plus the single-rank bench at the 8-GPU shard size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RAGMI_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
   --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu \
   > gpurun_out/bench_2rank_gloo.log 2>&1 || { rc=$?; tail -30 gpurun_out/bench_2rank_gloo.log; exit $rc; }
grep '^{' gpurun_out/bench_2rank_gloo.log | cut -c1-600
timeout -k 10 300 python bench.py --rows 1250000 --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_1p25M.log 2>&1 || { rc=$?; tail -20 gpurun_out/bench_1p25M.log; exit $rc; }
grep '^{' gpurun_out/bench_1p25M.log | cut -c1-900
