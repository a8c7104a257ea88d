#!/bin/bash
# round 4 (final build): per-rank rehearsal lines + config lines 2, 3, filtered, 5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_per_rank.sh && CONFIGS="3 2 filtered 5" bash scripts/gpu_lines.sh
