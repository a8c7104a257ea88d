#!/bin/bash
# round 4: per-rank rehearsal (N = 2/4/8 shard sizes through the world-1 RCCL exchange, with
# cpu_baseline) + config lines 3, 2, filtered, 5 on the round-4 build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_per_rank.sh && CONFIGS="3 2 filtered" bash scripts/gpu_lines.sh
