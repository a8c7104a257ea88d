#!/bin/bash
# round 4 final: smoke + full GPU suite + headline bench + rocprof passes, then config lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04z} bash scripts/gpu_verify.sh && CONFIGS=${CONFIGS:-"2 filtered"} bash scripts/gpu_lines.sh
